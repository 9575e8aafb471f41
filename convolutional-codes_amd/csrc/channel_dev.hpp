// channel_dev.hpp -- on-device channel producers fused ahead of the register-trellis ACS
// (SURVEY.md section 8(f) #1): info bytes, encoder, mapper, AWGN (Box-Muller on Philox4x32-10) and
// demapper -- or the BSC bit flips -- generated per lane, step by step, in the order the decoder
// consumes them, so no channel data touches HBM. The draw sequence is the product's host Philox
// producer's (csrc/sim.cpp PhiloxSource / Gauss / awgn_block / bsc_block), which follows the
// reference drivers' rand() call order (optionally through the hard demapper,
// common/hard-demapper.c:62-102):
//   AWGN-channel/main.c:217-223 (info bytes, rand() % 256), :93-106 (per symbol: map, add
//   scaling * gengauss() per I/Q in double, demap); common/gaussian.c:18-38 (Box-Muller, cosine
//   half first, u1 == 0 redrawn); common/demapper.c:61-70 (squared distance / ndist in fp32);
//   binary-symmetric-channel/main.c:57-72 (per bit: rand() % 1000000 < p_ppm flips it).
// Info bits, symbols and BSC flips are bit-identical to the host producer. The AWGN samples use the
// domain-specific log / sqrt / sincos of channel_math.hpp instead of glibc's, so a sample may differ
// in the last place where the two round differently (tests/test_gpu_parity.py bounds how often).
// Compiled with -ffp-contract=off: x + scaling * g and dx*dx + dy*dy must not fuse.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "acs_multi.hpp"
#include "acs_persist.hpp"
#include "acs_reg.hpp"
#include "trellis.hpp"

#define CCV_HD __device__
__device__ __forceinline__ double ccv_rcp_approx(double d) { return __builtin_amdgcn_rcp(d); }
__device__ __forceinline__ double ccv_rsq_approx(double x) { return __builtin_amdgcn_rsq(x); }
// a * b + c with a loop-invariant c: the three-address v_fma_f64 (the compiler otherwise picks the
// two-address v_fmac_f64 and copies the hoisted constant into the accumulator first, one v_mov_b64
// per Horner step)
// The constant sits in an SGPR pair (one scalar operand per VALU instruction is allowed): held in
// VGPRs, the hoisted Horner constants took ~30 VGPRs from the channel kernels (K = 7 double noise:
// 146 -> 113 VGPRs, 3 -> 4 waves per SIMD; measured +2 % idiom, +13 % true parity, round 5).
__device__ __forceinline__ double ccv_fma_const(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
}
#include "channel_math.hpp"

namespace ccv {

struct ChanArgs {
  RegArgs r;                 // r.in unused; r.info = info_out (read back by the traceback)
  uint64_t seed;
  uint64_t first_block;      // block b of the batch is stream block first_block + b
  float scaling;             // AWGN: noise scaling (AWGN-channel/main.c:157-161)
  int32_t p_ppm;             // BSC: flip probability in ppm
  int hard_demap;            // AWGN: common/hard-demapper.c instead of common/demapper.c
  uint8_t* info_out;         // [nb][IB] transmitted info bytes (required)
  void* ch_out;              // optional export: soft float [nb][T][2^n] / hard uint8 [nb][T]
  int global_decisions;      // K <= 7: 1 decisions through r.dec in HBM, 0 in LDS, -1 by occupancy
  int noise_f32;             // AWGN: the fp32 Box-Muller (CCV_CHANNEL_NOISE_F32, opt-in) instead of double
  int iq_out;                // frames only (CCV_CHANNEL_IQ): ch_out gets the demapper's input, the received
                             // point (x, y) as float [nb][T][2], instead of its 2^n distances
};

// The opt-in fp32 Box-Muller (CCV_CHANNEL_NOISE_F32): the same uniforms k1, k2 / (2^31 - 1) as the
// double-precision path, R = sqrt(-2 ln u1) and (cos, sin)(2 pi u2) from the hardware transcendentals
// (v_log_f32 = log2, v_sqrt_f32, v_sin_f32 / v_cos_f32, whose argument is in revolutions: exactly
// 2 pi u2), and the noisy coordinate x + scaling * R * {cos, sin} rounded in fp32. Near u1 = 1, where
// -2 ln u1 is tiny and the fp32 rounding of u1 would dominate it, the series -2 ln(1 - v) =
// 2 (v + v^2/2 + v^3/3 + v^4/4) of v = (M - k1) / M is used instead (exact integer M - k1 < 2^24,
// truncation < 2^-30 relative). Not bit-exact with the double path (or glibc): the frames differ in
// the last fp32 places, so only the statistics can agree -- tools/chanmath_f32_check.hip bounds the
// errors over every k1 and k2, tests/test_gpu_ber.py checks the published curves in this mode.
__device__ __forceinline__ float neg2_log_f32(uint32_t k) {   // k in [1, 2^31 - 1]
  const uint32_t w = 2147483647u - k;
  const float v = (float)w * (1.0f / 2147483647.0f);
  const float series = 2.0f * v * (1.0f + v * (0.5f + v * (1.0f / 3.0f + v * 0.25f)));
  const float u = (float)k * (1.0f / 2147483647.0f);
  const float lg = -1.38629436111989061883f * __builtin_amdgcn_logf(u);   // -2 ln 2 * log2(u)
  return w < (1u << 24) ? series : lg;
}
// R = sqrt(-2 ln u1) with the raw v_sqrt_f32 (1 ulp; its argument is >= 9.3e-10, never denormal, so
// the IEEE sqrt's scaling and two correction steps buy nothing here)
__device__ __forceinline__ float radius_f32(uint32_t k1) { return __builtin_amdgcn_sqrtf(neg2_log_f32(k1)); }
__device__ __forceinline__ void box_muller_f32(uint32_t k1, uint32_t k2, float& c, float& s, float& r) {
  r = radius_f32(k1);
  const float u2 = (float)k2 * (1.0f / 2147483647.0f);
  c = __builtin_amdgcn_cosf(u2);
  s = __builtin_amdgcn_sinf(u2);
}

// Philox4x32-10 with one counter stream per block (key = seed, counter = (block, draw, 0, tag)).
struct Philox {
  uint32_t k0, k1, c0, c1, c2;
  uint32_t b0, b1, b2, b3;
  int used;
  __device__ __forceinline__ void init(uint64_t seed, uint64_t block) {
    k0 = (uint32_t)seed; k1 = (uint32_t)(seed >> 32);
    c0 = (uint32_t)block; c1 = (uint32_t)(block >> 32); c2 = 0;
    used = 4;
  }
  __device__ __forceinline__ void refill() {
    uint32_t x0 = c0, x1 = c1, x2 = c2, x3 = 0x43435631u, y0 = k0, y1 = k1;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      // one v_mad_u64_u32 per product (hi and lo together) instead of v_mul_hi + v_mul_lo
      const uint64_t p0 = (uint64_t)0xD2511F53u * x0, p1 = (uint64_t)0xCD9E8D57u * x2;
      const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
      const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
      x0 = h1 ^ x1 ^ y0; x1 = l1;
      x2 = h0 ^ x3 ^ y1; x3 = l0;
      y0 += 0x9E3779B9u; y1 += 0xBB67AE85u;
    }
    b0 = x0; b1 = x1; b2 = x2; b3 = x3;
    ++c2;
    used = 0;
  }
  // 31-bit value, like rand()
  __device__ __forceinline__ uint32_t next() {
    if (used == 4) refill();
    const uint32_t r = b0;
    b0 = b1; b1 = b2; b2 = b3;
    ++used;
    return r >> 1;
  }
  // the next two values (x first): one refill site and selects instead of two next() (a pair
  // straddles a refill when one word is left, used == 3)
  __device__ __forceinline__ void next2(uint32_t& x, uint32_t& y) {
    const bool odd = used == 3;
    const uint32_t last = b0;
    if (used >= 3) refill();
    x = (odd ? last : b0) >> 1;
    y = (odd ? b0 : b1) >> 1;
    const uint32_t n0 = odd ? b1 : b2, n1 = odd ? b2 : b3;
    b2 = b3;   // meaningful only when odd (three words left)
    b0 = n0;
    b1 = n1;
    used = odd ? 1 : used + 2;
  }
};

// Division by the channel's two constants in three instructions instead of the IEEE sequence
// (v_div_scale / v_div_fmas / v_div_fixup, ~10): Markstein's correction q0 = a*r, e = fma(-q0, b, a)
// (exact), q = fma(e, r, q0) with r = RN(1/b). Checked bit-identical to IEEE division, on the device,
// for EVERY operand of the domain (tools/divcheck.hip, profiles/r02_divcheck.txt):
//  * k / 2147483647.0 for all k < 2^31 (gaussian.c:23-24: the uniform draws);
//  * x / ndist for all 2^-60 <= x < 2^64, for the ndist of the n = 1, 2, 3 constellations
//    (demapper.c:70). The squared distances stay in that range: a nonzero |x - p| is at least half an
//    ulp of a constellation coordinate (>= 2^-25), and |noise| <= 6.56 * scaling (Box-Muller of a
//    31-bit uniform), so the host requires scaling < 2^28 (ccv_simulate_device) -- Eb/N0 > -160 dB.
__device__ __forceinline__ double div_rand_max(uint32_t k) {
  constexpr double M = 2147483647.0, R = 1.0 / M;
  const double a = (double)k;
  const double q0 = a * R;
  const double e = __builtin_fma(-q0, M, a);
  return __builtin_fma(e, R, q0);
}
template <float B>
__device__ __forceinline__ float div_const(float a) {
  constexpr float R = 1.0f / B;
  const float q0 = a * R;
  const float e = __builtin_fmaf(-q0, B, a);
  return __builtin_fmaf(e, R, q0);
}

// common/constellations.c:6-28 (index = symbol value).
template <int N>
struct Constellation;
template <>
struct Constellation<1> {
  static constexpr float pts[4] = {0.707107f, 0.707107f, -0.707107f, -0.707107f};
};
template <>
struct Constellation<2> {
  static constexpr float pts[8] = {0.707107f, 0.707107f, 0.707107f, -0.707107f,
                                   -0.707107f, 0.707107f, -0.707107f, -0.707107f};
};
template <>
struct Constellation<3> {
  static constexpr float pts[16] = {0.408248f, 0.408248f, 0.408248f, 1.224745f,
                                    -0.408248f, 0.408248f, -1.224745f, 0.408248f,
                                    0.408248f, -0.408248f, 1.224745f, -0.408248f,
                                    -0.408248f, -0.408248f, -0.408248f, -1.224745f};
};

// Encoder (common/encoder.c:84-119), bit-sliced over 32 steps: output stream k of step t is the parity
// of the taps j of poly k over the info bits i(t - j) (the reference's shift register holds i(t - j)
// at bit 63 - j), so a whole word of it is the XOR of the info word shifted right by each tap j
// (funnelled with the previous word), computed once per 32 steps; the x86 idiom (GEN_REF_X86: the
// result cleared when the taps at register bits 4 mod 8 have odd parity) is one more such XOR. Per
// step: the symbol's bits are the streams' top bits, then one shift each. The info bits are MSB-first,
// cleared from blen on (the tail steps shift in zeros); init assembles all eight window words in
// w[0..7], start() keeps the current and the next word in registers and parks words 2..7 in LDS
// (6 words x 64 lanes), read back one per 32 steps, a whole word period before they are needed
// (~10 fewer VGPRs; the LDS-decision kernel, whose occupancy is set by its LDS, keeps them in
// registers).
template <CodeSpec C, bool PARK = true>   // PARK false: the whole window stays in registers
struct Encoder {
  static_assert(C.K >= 2 && C.K <= 32, "bit-sliced encoder: taps within one word");
  uint32_t w[8];     // init: the whole window; PARK: from start() on only w[0] (current), w[1] (next)
  uint32_t e[C.n];   // stream k of the current 32-step word, the current step in bit 31
  int t;
  __device__ __forceinline__ static uint32_t* park() {   // this lane's column of words 2..7, [6][64]
    __shared__ uint32_t parked[6 * kRegThreads];
    return parked + threadIdx.x;
  }
  __device__ __forceinline__ void start(int blen) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int valid = blen - 32 * k;
      w[k] &= valid >= 32 ? ~0u : (valid <= 0 ? 0u : ~0u << (32 - valid));
    }
    if constexpr (PARK) {
#pragma unroll
      for (int k = 2; k < 8; ++k) park()[(k - 2) * kRegThreads] = w[k];
    }
    t = 0;
    fill(0u, w[0]);
  }
  __device__ __forceinline__ void fill(uint32_t prev, uint32_t cur) {
#pragma unroll
    for (int k = 0; k < C.n; ++k) {
      uint32_t x = 0, tw = 0;
#pragma unroll
      for (int j = 0; j < C.K; ++j) {
        if (((C.poly[k] >> (63 - j)) & 1u) == 0) continue;
        uint32_t s = cur;
        if (j > 0) s = (cur >> j) | (prev << (32 - j));
        x ^= s;
        if (C.gen == GEN_REF_X86 && (63 - j) % 8 == 4) tw ^= s;
      }
      e[k] = C.gen == GEN_REF_X86 ? (x & ~tw) : x;
    }
  }
  // bit 31 = output bit k of the current step (k = 0: the symbol's MSB)
  __device__ __forceinline__ uint32_t msb(int k) const { return e[k] & 0x80000000u; }
  __device__ __forceinline__ uint32_t symbol() const {
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < C.n; ++k) s = (s << 1) | (e[k] >> 31);
    return s;
  }
  // the window moves by a word every 32 steps behind a real (wave-uniform) branch: the empty volatile
  // asm keeps the compiler from speculating the word shift into selects on every step
  __device__ __forceinline__ void advance() {
    ++t;
    if ((t & 31) == 0) {
      const uint32_t prev = w[0];
      if constexpr (PARK) {
        w[0] = w[1];
        const int next = (t >> 5) - 1;   // words 2, 3, ... come in at t = 32, 64, ...
        const uint32_t nw = park()[(next < 6 ? next : 5) * kRegThreads];
        w[1] = next < 6 ? nw : 0u;
      } else {
#pragma unroll
        for (int k = 0; k < 7; ++k) w[k] = w[k + 1];
        w[7] = 0;
      }
      fill(prev, w[0]);
      asm volatile("");
    } else {
#pragma unroll
      for (int k = 0; k < C.n; ++k) e[k] <<= 1;
    }
  }
};

// Encoder of a code known only at run time (ccv_simulate_device CCV_CHANNEL_FRAMES_ONLY: any plan, K <=
// 64): the reference's shift-register arithmetic step by step, with a 64-bit state; the same window.
template <int NP>
struct EncoderRT {
  uint32_t w[8];
  uint64_t state;
  int t;
  int K, gen;
  uint64_t poly[NP];
  __device__ __forceinline__ void start(int blen) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int valid = blen - 32 * k;
      w[k] &= valid >= 32 ? ~0u : (valid <= 0 ? 0u : ~0u << (32 - valid));
    }
    state = 0;
    t = 0;
  }
  __device__ __forceinline__ uint32_t symbol() const {
    const uint64_t i = w[0] >> 31;
    const uint64_t sr = (K < 64 ? state << (64 - K) : state) | (i << 63);
    uint32_t e = 0;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const uint64_t v = sr & poly[k];
      uint32_t p = (uint32_t)__popcll(v) & 1u;
      if (gen == GEN_REF_X86) p &= ((uint32_t)__popcll(v & 0x1010101010101010ull) & 1u) ^ 1u;
      e = (e << 1) | p;
    }
    return e;
  }
  __device__ __forceinline__ uint32_t msb(int k) const { return ((symbol() >> (NP - 1 - k)) & 1u) << 31; }
  __device__ __forceinline__ void advance() {
    state = (state >> 1) | ((uint64_t)(w[0] >> 31) << (K - 2));
    ++t;
    if ((t & 31) == 0) {
#pragma unroll
      for (int k = 0; k < 7; ++k) w[k] = w[k + 1];
      w[7] = 0;
      asm volatile("");
    } else {
      w[0] <<= 1;
    }
  }
};

// F32: the opt-in fp32 Box-Muller (CCV_CHANNEL_NOISE_F32) -- a compile-time choice, so the fp32
// kernels do not hold the double-precision path's registers (108 instead of 157 VGPRs at K = 7 true
// parity: one more wave per SIMD).
template <CodeSpec C, bool HARD, class Enc = Encoder<C>, bool F32 = false, bool IQ = false>
struct ChannelSource {
  static constexpr int NS = 1 << C.n;
  using MT = typename std::conditional<HARD, uint32_t, float>::type;
  Philox rng;
  Enc enc;
  int T, blen;
  float scaling;
  int32_t p_ppm;
  bool hard_demap;
  void* out;       // export row of this block, or null

  // Draw the info bytes (first in the stream), write them to info_out, prime the encoder.
  __device__ __forceinline__ void init(const ChanArgs& a, int block, bool owner) {
    T = a.r.T; blen = a.r.blen;
    scaling = a.scaling; p_ppm = a.p_ppm; hard_demap = a.hard_demap != 0;
    rng.init(a.seed, a.first_block + (uint64_t)block);
    const int IB = (blen + 7) >> 3;
#pragma unroll
    for (int k = 0; k < 8; ++k) enc.w[k] = 0;
    uint8_t* info = a.info_out + (size_t)block * IB;
#pragma unroll 1
    for (int j = 0; j < IB; ++j) {
      const uint32_t byte = rng.next() % 256u;
      if (owner) info[j] = (uint8_t)byte;
      // shift the byte in at the bottom of the 256-bit register (indices stay static)
#pragma unroll
      for (int k = 0; k < 7; ++k) enc.w[k] = (enc.w[k] << 8) | (enc.w[k + 1] >> 24);
      enc.w[7] = (enc.w[7] << 8) | byte;
    }
    // the IB bytes now sit in the low 8*IB bits of the 256-bit register w[0..7] (w[0] most
    // significant); shift left by 256 - 8*IB bits so that info bit 0 is the MSB of w[0]
    const int shift_words = 8 - ((IB + 3) >> 2);
    const int shift_bytes = (4 - (IB & 3)) & 3;
#pragma unroll 1
    for (int s = 0; s < shift_words; ++s) {
#pragma unroll
      for (int k = 0; k < 7; ++k) enc.w[k] = enc.w[k + 1];
      enc.w[7] = 0;
    }
    if (shift_bytes) {
      const int sb = shift_bytes * 8;
#pragma unroll
      for (int k = 0; k < 7; ++k) enc.w[k] = (enc.w[k] << sb) | (enc.w[k + 1] >> (32 - sb));
      enc.w[7] <<= sb;
    }
    enc.start(blen);
    out = a.ch_out && owner
              ? (void*)((char*)a.ch_out + (size_t)block * T * (HARD ? 1 : (IQ ? 2 : NS) * sizeof(float)))
              : nullptr;
  }

  // A soft step in two phases: draw() -- the symbol's bits from the encoder and the step's two
  // uniforms (the branches: Philox refill, window shift, the u1 = 0 redraw) -- then compute() -- the
  // noise, the demapper, the branch metrics. (Round 5 measured a software-pipelined loop that puts
  // step t + 1's compute() in one basic block with step t's ACS: hipcc does not interleave them, and
  // it ran within 1 % of the plain loop, profiles/r05_chan/.)
  struct Draw {
    uint32_t sx, sy;   // n <= 2: the sign words of the point's coordinates; n = 3: sx = the symbol
    uint32_t k1, k2;
    int t;
  };
  __device__ __forceinline__ Draw draw() {
    Draw d;
    d.t = enc.t;
    if constexpr (C.n <= 2) {
      d.sx = enc.msb(0);
      d.sy = enc.msb(C.n - 1);
    } else {
      d.sx = enc.symbol();
      d.sy = 0;
    }
    enc.advance();
    rng.next2(d.k1, d.k2);
    if (__builtin_expect(d.k1 == 0u, 0)) {   // u1 == 0 redrawn (gaussian.c:23-27)
      do {
        rng.next2(d.k1, d.k2);
      } while (d.k1 == 0u);
    }
    return d;
  }
  __device__ __forceinline__ void compute(const Draw& d, float (&BM)[NS]) const {
    static_assert(C.n >= 1 && C.n <= 3, "the reference has constellations for n = 1..3");
    constexpr const float* pts = Constellation<C.n>::pts;
    float x = 0.f, y = 0.f;
    if constexpr (C.n <= 2) {
      // n = 1, 2: the points are (+-a, +-a), the signs the symbol's bits (n = 2: x <- bit 1,
      // y <- bit 0; n = 1: both <- bit 0) -- two sign flips instead of a compare-select chain
      static_assert(pts[0] == pts[1] && (C.n == 1 ? pts[2] == -pts[0] : pts[4] == -pts[0] && pts[3] == -pts[1]));
      const uint32_t a = __builtin_bit_cast(uint32_t, pts[0]);
      x = __builtin_bit_cast(float, a ^ d.sx);
      y = __builtin_bit_cast(float, a ^ d.sy);
    } else {
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        x = d.sx == (uint32_t)k ? pts[2 * k] : x;
        y = d.sx == (uint32_t)k ? pts[2 * k + 1] : y;
      }
    }
    if constexpr (F32) {
      float cf, sf, rf;
      box_muller_f32(d.k1, d.k2, cf, sf, rf);
      x = x + scaling * (rf * cf);
      y = y + scaling * (rf * sf);
    } else {
      const double u1 = div_rand_max(d.k1), u2 = div_rand_max(d.k2);
      // R = sqrt(-2 ln u1), (sin, cos)(2 pi u2): channel_math.hpp (a few ulp in double; 2e-8 or
      // fewer of the fp32 samples differ from glibc's, 268 M host draws, profiles/r04_chanmath_check.txt)
      const double R = chanmath::sqrt_nonneg(chanmath::neg2_log(u1));
      double sn, cs;
      chanmath::sincos_2pi(u2, &sn, &cs);
      x = (float)((double)x + (double)scaling * (R * cs));
      y = (float)((double)y + (double)scaling * (R * sn));
    }
    if (hard_demap) {   // common/hard-demapper.c:66-80: snap to the first nearest point
      float min_val = __builtin_inff();
      float sx = pts[0], sy = pts[1];
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        const float dx = x - pts[2 * k], dy = y - pts[2 * k + 1];
        const float dd = (dx * dx) + (dy * dy);
        const bool lt = dd < min_val;
        min_val = lt ? dd : min_val;
        sx = lt ? pts[2 * k] : sx;
        sy = lt ? pts[2 * k + 1] : sy;
      }
      x = sx;
      y = sy;
    }
    if constexpr (IQ) {   // the demapper's input: the received point (the snapped one with hard_demap)
      if (out && d.t < T) reinterpret_cast<float2*>(out)[d.t] = make_float2(x, y);
      return;
    }
    constexpr float ndx = pts[0] - pts[2], ndy = pts[1] - pts[3];
    constexpr float nd = (ndx * ndx) + (ndy * ndy);
    // the points as compile-time constants (a loop over pts[] reads them from memory), so the
    // coordinates the points share give one subtraction and one square each
    [&]<int... k>(std::integer_sequence<int, k...>) __attribute__((always_inline)) {
      ((BM[k] = div_const<nd>(((x - Constellation<C.n>::pts[2 * k]) * (x - Constellation<C.n>::pts[2 * k])) +
                              ((y - Constellation<C.n>::pts[2 * k + 1]) * (y - Constellation<C.n>::pts[2 * k + 1])))),
       ...);
    }(std::make_integer_sequence<int, NS>{});
  }
  __device__ __forceinline__ void export_soft(int t, const float (&BM)[NS]) const {
    if (out && t < T) {
      float* o = reinterpret_cast<float*>(out) + (size_t)t * NS;
#pragma unroll
      for (int k = 0; k < NS; ++k) o[k] = BM[k];
    }
  }

  __device__ __forceinline__ void next(MT (&BM)[NS]) {
    if constexpr (HARD) {
      const int t = enc.t;
      uint32_t sym = enc.symbol();
      enc.advance();
      if constexpr (C.n == 2) {   // draw k flips bit k
        uint32_t r0, r1;
        rng.next2(r0, r1);
        sym ^= ((int32_t)(r0 % 1000000u) < p_ppm ? 1u : 0u) | ((int32_t)(r1 % 1000000u) < p_ppm ? 2u : 0u);
      } else {
#pragma unroll
        for (int k = 0; k < C.n; ++k)
          if ((int32_t)(rng.next() % 1000000u) < p_ppm) sym ^= 1u << k;
      }
#pragma unroll
      for (int k = 0; k < NS; ++k) BM[k] = (uint32_t)__builtin_popcount((uint32_t)k ^ sym);
      if (out && t < T) reinterpret_cast<uint8_t*>(out)[t] = (uint8_t)sym;
    } else {
      const Draw d = draw();
      compute(d, BM);
      if constexpr (!IQ) export_soft(d.t, BM);
    }
  }
};

// step(t) for t in [t0, t1), unrolled by U = K - 1 with a rolled remainder. An in-place trellis step
// leaves new state j in the register old state 2j held (acs_step), a permutation of period K - 1: a
// rolled loop pays ~30 register copies per step at its back edge to put every metric back, an
// unrolled period none.
template <int U, class F>
__device__ __forceinline__ void for_steps(int t0, int t1, F&& step) {
  int t = t0;
#pragma unroll 1
  for (; t + U <= t1; t += U) {
    [&]<int... u>(std::integer_sequence<int, u...>) __attribute__((always_inline)) {
      (step(t + u), ...);
    }(std::make_integer_sequence<int, U>{});
  }
#pragma unroll 1
  for (; t < t1; ++t) step(t);
}

// K <= 7: one lane per block (acs_reg.hpp), input generated in registers.
template <CodeSpec C, bool HARD, bool F32 = false>
__global__ __launch_bounds__(kRegThreads) void viterbi_channel_reg(ChanArgs a) {
  constexpr int S = 1 << (C.K - 1);
  constexpr int NS = 1 << C.n;
  using DW = DecWord<S>;
  using Src = ChannelSource<C, HARD, Encoder<C>, F32>;
  using MT = typename Src::MT;
  const int b = blockIdx.x * kRegThreads + threadIdx.x;
  const int T = a.r.T, nb = a.r.nblocks;
  const int bc = b < nb ? b : nb - 1;
  DW* dec = reinterpret_cast<DW*>(a.r.dec) + b;
  const size_t dstride = (size_t)a.r.dec_stride;
  Src src;
  src.init(a, bc, b < nb);
  MT M[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if constexpr (HARD) M[s] = s ? 0xFF00u : 0u;
    else M[s] = s ? __builtin_inff() : 0.0f;
  }
  auto run = [&](auto sat, int t0, int t1) {
    for_steps<C.K - 1>(t0, t1, [&](int t) __attribute__((always_inline)) {
      MT BM[NS];
      src.next(BM);
      dec[(size_t)t * dstride] = acs_step<C, decltype(sat)::value, MT>(M, BM);
    });
  };
  // BSC saturation (reference :127-130) only matters while states are unreachable (t < K-1);
  // afterwards the hard ACS runs on 16-bit metrics (uint16_t), like viterbi_hard_reg
  const int t0 = HARD ? (T < C.K - 1 ? T : C.K - 1) : 0;
  if constexpr (HARD) {
    run(std::true_type{}, 0, t0);
    uint16_t M16[S];
#pragma unroll
    for (int s = 0; s < S; ++s) M16[s] = (uint16_t)M[s];
    for_steps<C.K - 1>(t0, T, [&](int t) __attribute__((always_inline)) {
      MT BM[NS];
      src.next(BM);
      uint16_t B16[NS];
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        B16[k] = (uint16_t)BM[k];
        asm volatile("" : "+v"(B16[k]));   // no v_bcnt-folded adds
      }
      dec[(size_t)t * dstride] = acs_step<C, false, uint16_t>(M16, B16);
    });
#pragma unroll
    for (int s = 0; s < S; ++s) M[s] = M16[s];
  } else {
    run(std::false_type{}, t0, T);
  }
  uint32_t errors = 0;
  if (b < nb) {
    MT best;
    const uint32_t st = (uint32_t)argmin_state<S, MT>(M, HARD ? (MT)0xFF00u : (MT)__builtin_inff(), best);
    if constexpr (HARD) {
      if (a.r.path_metric) a.r.path_metric[b] = (int32_t)best;
    }
    errors = traceback<C.K>(a.r, b, st);
  }
  accumulate_errors(a.r, errors);
}

// K <= 7 with the survivor decisions in LDS instead of HBM (the BSC default, core.hip):
// the main steps' words go to lds[t - G][lane] (20 KiB per wave at K=7, blen 40), the first K-1
// steps are growth steps (acs_persist.hpp growth_step: one add per reachable state, decision 0,
// nothing stored), and the traceback reads the lane's column back with the history word of
// traceback_regs -- no decision traffic to HBM (2 x 8 B per step per block). The column caps a CU at
// 8 waves: BSC gains (108.6 vs 96.6 Gbit/s, K=7), the double-precision AWGN channel, whose
// viterbi_channel_reg runs 12 waves per CU, loses (60.3 vs 62.5).
// The output bit of step t is bit t of H = (st << F) | sum d_m 2^m (F = T - (K-1) main steps, d_m the
// decision read at main step m): byte k is bit-reversed bits 8k .. 8k+7, emitted as the walk passes.
template <int K, typename DW>
__device__ __forceinline__ uint32_t traceback_lds(const RegArgs& a, const DW* col, int b, uint32_t st,
                                                  bool owner) {
  constexpr uint32_t S = 1u << (K - 1);
  const int T = a.T, F = T - (K - 1), OB = (T + 7) >> 3, IB = (a.blen + 7) >> 3;
  uint8_t* out = a.out + (size_t)b * OB;
  const uint8_t* info = a.info != nullptr ? a.info + (size_t)b * IB : nullptr;
  uint32_t errors = 0;
  auto emit = [&](int k, uint32_t bits8) {   // bits8: bit j = output of step 8k + j
    const uint32_t byte = __builtin_bitreverse32(bits8) >> 24;
    if (owner) out[k] = (uint8_t)byte;
    if (info != nullptr && k < IB) {
      const int valid = a.blen - 8 * k;
      const uint32_t mask = valid >= 8 ? 0xFFu : (0xFFu << (8 - valid)) & 0xFFu;
      errors += __builtin_popcount((byte ^ info[k]) & mask);
    }
  };
  // bytes made of final-state bits only
  for (int k = OB - 1; 8 * k >= F; --k) emit(k, (st >> (8 * k - F)) & 0xFFu);
  uint32_t h = st;
#pragma unroll 8
  for (int m = F - 1; m >= 0; --m) {
    const uint32_t d = (uint32_t)(col[(size_t)m * kRegThreads] >> (h & (S - 1)));
    h = (h << 1) | (d & 1u);
    if ((m & 7) == 0) emit(m >> 3, h & 0xFFu);
  }
  return owner ? errors : 0u;
}

template <CodeSpec C, bool HARD, bool F32 = false>
__global__ __launch_bounds__(kRegThreads) void viterbi_channel_lds(ChanArgs a) {
  constexpr int S = 1 << (C.K - 1);
  constexpr int NS = 1 << C.n;
  constexpr int G = C.K - 1;
  using DW = DecWord<S>;
  // the encoder window stays in registers: its LDS words would cost this kernel a wave per CU
  using Src = ChannelSource<C, HARD, Encoder<C, false>, F32>;
  using SM = typename Src::MT;                                      // source metric type
  // ACS metric type: uint16_t for the BSC (fp32, exact here as in the persistent BSC kernel,
  // acs_persist.hpp, measured 1 % slower in this kernel, whose time is the channel's, and mixed
  // after the unrolled loop: profiles/r05d/, profiles/r05_chan/chan_bench_bsc_f32_ab.jsonl)
  using MT = typename std::conditional<HARD, uint16_t, float>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char chan_lds[];
  DW* dl = reinterpret_cast<DW*>(chan_lds);
  const int lane = threadIdx.x;
  const int b = blockIdx.x * kRegThreads + lane;
  const int T = a.r.T, nb = a.r.nblocks;
  const int bc = b < nb ? b : nb - 1;
  Src src;
  src.init(a, bc, b < nb);
  MT M[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if constexpr (HARD) M[s] = (MT)(s ? 0xFF00u : 0u);   // viterbi-decoder.c:225-228
    else M[s] = s ? __builtin_inff() : 0.0f;           // viterbi-decoder.c:212-218
  }
  auto next_bm = [&](MT (&BM)[NS]) __attribute__((always_inline)) {
    SM raw[NS];
    src.next(raw);
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      BM[k] = (MT)raw[k];
      if constexpr (std::is_same_v<MT, uint16_t>) asm volatile("" : "+v"(BM[k]));   // no v_bcnt-folded adds (acs_reg.hpp)
    }
  };
  // T >= K > G: every block has its K-1 growth steps
  [&]<int... ts>(std::integer_sequence<int, ts...>) __attribute__((always_inline)) {
    ([&]() __attribute__((always_inline)) {
      MT BM[NS];
      next_bm(BM);
      growth_step<C, ts, MT>(M, BM, HARD ? (MT)0xFF00u : (MT)__builtin_inff());
    }(), ...);
  }(std::make_integer_sequence<int, G>{});
  for_steps<C.K - 1>(G, T, [&](int t) __attribute__((always_inline)) {
    MT BM[NS];
    next_bm(BM);
    dl[(size_t)(t - G) * kRegThreads + lane] = acs_step<C, false, MT>(M, BM);
  });
  // each lane reads back only its own column: no barrier
  using AM = typename std::conditional<std::is_same_v<MT, uint16_t>, uint32_t, float>::type;
  AM Ma[S];
#pragma unroll
  for (int s = 0; s < S; ++s) Ma[s] = (AM)M[s];
  AM best;
  const uint32_t st = (uint32_t)argmin_state<S, AM>(Ma, HARD ? (AM)0xFF00u : (AM)__builtin_inff(), best);
  if constexpr (HARD) {
    if (b < nb && a.r.path_metric) a.r.path_metric[b] = (int32_t)best;
  }
  const uint32_t errors = traceback_lds<C.K, DW>(a.r, dl + lane, bc, st, b < nb);
  accumulate_errors(a.r, errors);
}

// Frames only: one lane per block draws its info bytes and its whole decoder input and writes them
// to a.info_out / a.ch_out (soft float [nb][T][2^n] at n = 2); no decode. The K = 9 sweep decodes
// these frames with the one-lane-per-block kernel (acs_wide.hpp) instead of running the channel once
// per lane of a block's four-lane group (viterbi_channel_multi below).
// Rows go out through LDS, 8 steps at a time: lane-per-row 16-byte stores put one wave's 64 stores
// in 64 different 128-byte lines, which L2 evicts half-written (WRITE_SIZE 2.5x the frame bytes,
// DESIGN.md 4.4); staged, store instruction j writes rows 8j .. 8j+7, 8 lanes per 128-byte line.
template <CodeSpec C, bool HARD, bool F32 = false>
__global__ __launch_bounds__(kRegThreads) void channel_frames(ChanArgs a) {
  static_assert(!HARD && C.n == 2, "soft r = 1/2 frames");
  using Src = ChannelSource<C, HARD, Encoder<C>, F32>;
  constexpr int CH = 8;   // steps per staged chunk: CH x 16 B = one 128-byte line of a row
  __shared__ float4 stage[CH][kRegThreads];
  const int lane = threadIdx.x;
  const int b0 = blockIdx.x * kRegThreads;
  const int nb = a.r.nblocks, T = a.r.T;
  const int b = b0 + lane;
  Src src;
  src.init(a, b < nb ? b : nb - 1, b < nb);   // every lane runs: the stores below are cooperative
  src.out = nullptr;
  const int sub = lane & (CH - 1), rsub = lane / CH;
  float4* frame = reinterpret_cast<float4*>(a.ch_out);
#pragma unroll 1
  for (int c0 = 0; c0 < T; c0 += CH) {
    const int n = T - c0 < CH ? T - c0 : CH;
#pragma unroll 1
    for (int k = 0; k < n; ++k) {
      float BM[4];
      src.next(BM);
      stage[k][lane] = float4{BM[0], BM[1], BM[2], BM[3]};
    }
    __syncthreads();
#pragma unroll 2
    for (int j = 0; j < kRegThreads / CH; ++j) {
      const int r = j * CH + rsub;
      if (sub < n && b0 + r < nb) frame[(size_t)(b0 + r) * T + c0 + sub] = stage[sub][r];
    }
    __syncthreads();
  }
}

// Frames only, any code (CCV_CHANNEL_FRAMES_ONLY): one lane per block writes the info bytes and the
// decoder input of its block (float [T][2^n] or uint8 [T]) in the same draw order, with no decode --
// the producer of the sequential decoders' device sweeps (K = 15, WSPR K = 32). Rows are written by
// the source's per-step export (a lane's own row; these decoders take far longer than the channel).
struct CodeRT {
  int K, gen;
  uint64_t poly[3];
};
template <int NP, bool HARD, bool F32 = false, bool IQ = false>
__global__ __launch_bounds__(kRegThreads) void channel_frames_rt(ChanArgs a, CodeRT code) {
  constexpr CodeSpec C{NP, 3, {0, 0, 0, 0, 0, 0, 0, 0}, GEN_REF_X86};   // n only: the encoder is RT
  using Src = ChannelSource<C, HARD, EncoderRT<NP>, F32, IQ>;
  using MT = typename Src::MT;
  const int b = blockIdx.x * kRegThreads + threadIdx.x;
  if (b >= a.r.nblocks) return;
  Src src;
  src.enc.K = code.K;
  src.enc.gen = code.gen;
#pragma unroll
  for (int k = 0; k < NP; ++k) src.enc.poly[k] = code.poly[k];
  src.init(a, b, true);
#pragma unroll 1
  for (int t = 0; t < a.r.T; ++t) {
    MT BM[Src::NS];
    src.next(BM);
  }
}

// K = 8, 9: multilane kernel (acs_multi.hpp); every lane of a block's group generates the block's
// input (the same draws), lane q = 0 owns the info and export writes.
template <CodeSpec C, bool HARD, bool F32 = false>
__global__ __launch_bounds__(kRegThreads) void viterbi_channel_multi(ChanArgs a) {
  using X = Multi<C>;
  constexpr int NS = X::NS;
  constexpr int n = X::n;
  using Src = ChannelSource<C, HARD, Encoder<C>, F32>;
  using MT = typename Src::MT;
  const int lane = threadIdx.x;
  const int q = lane & (X::L - 1);
  const bool qb0 = (q & 1) != 0, qb1 = (q & 2) != 0;
  const int blk = (blockIdx.x * kRegThreads + lane) / X::L;
  const int T = a.r.T, nb = a.r.nblocks;
  const int bc = blk < nb ? blk : nb - 1;
  const bool writer = q == 0 && blk < nb;
  uint64_t* dec = reinterpret_cast<uint64_t*>(a.r.dec) + (size_t)blockIdx.x * kRegThreads + lane;
  const size_t dstride = (size_t)a.r.dec_stride;
  Src src;
  src.init(a, bc, writer);
  MT M[64];
#pragma unroll
  for (int r = 0; r < 64; ++r) {
    if constexpr (HARD) M[r] = (q == 0 && r == 0) ? 0u : 0xFF00u;
    else M[r] = (q == 0 && r == 0) ? 0.0f : __builtin_inff();
  }
  // the ring runs n steps ahead of the ACS; the source is sequential, so refills past T only draw
  // numbers nobody uses
  struct Step { MT v[NS]; };
  auto load = [&](int) { Step s; src.next(s.v); return s; };
  auto metrics = [](const Step& in, MT (&BM)[NS]) {
#pragma unroll
    for (int k = 0; k < NS; ++k) BM[k] = in.v[k];
  };
  Step ring[n];
#pragma unroll
  for (int k = 0; k < n; ++k) ring[k] = load(k);
  auto sink = [&](auto, int t, uint64_t w) { dec[(size_t)t * dstride] = w; };
  if constexpr (HARD) {
    multi_period<C, true, MT, 0>(0, T, M, ring, load, metrics, sink, qb0, qb1);
    for (int t = n; t < T; t += n)
      multi_period<C, false, MT, 0>(t, T, M, ring, load, metrics, sink, qb0, qb1);
  } else {
    for (int t = 0; t < T; t += n)
      multi_period<C, false, MT, 0>(t, T, M, ring, load, metrics, sink, qb0, qb1);
  }
  MT best;
  const MT sentinel = HARD ? (MT)0xFF00u : (MT)__builtin_inff();
  const uint32_t st = multi_argmin<C, MT>(M, T % n, q, sentinel, best);
  if constexpr (HARD) {
    if (writer && a.r.path_metric) a.r.path_metric[blk] = (int32_t)best;
  }
  const uint32_t errors = multi_traceback<C>(a.r, blk, st, writer);
  accumulate_errors(a.r, errors);
}

}  // namespace ccv
