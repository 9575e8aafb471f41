// acs_reg.hpp -- register-trellis Viterbi kernels for CDNA4 (gfx950), specialised per code.
//
// One lane decodes one whole trellis block: all 2^(K-1) path metrics live in VGPRs, the trellis
// (expected symbols, hence which branch metric feeds which add) is a compile-time constant, and the
// add-compare-select of reference AWGN-channel/viterbi-decoder.c:108-141 (soft) or
// binary-symmetric-channel/viterbi-decoder.c:114-150 (hard) reduces to straight-line VALU code:
//   per butterfly j (old states 2j, 2j+1 -> new states j, j + S/2), per input i:
//     m0 = M[2j] + bm(2j, i), m1 = M[2j+1] + bm(2j+1, i)
//     M'[j + i*S/2] = min(m0, m1)                       (v_min)
//     decision bit  = sign(m1 - m0)  == (m1 < m0)       (v_sub + v_alignbit shift-in)
// which is the reference's "ascending s, inputs 0 then 1, strict <" rule in closed form: the even
// predecessor is visited first and is kept on ties. No permutation between lanes is ever needed,
// so the only per-state cost is 2 adds + min + sub + shift-in.
//
// Decisions (S bits per step) go to a [T][dec_stride] array of 32/64-bit words (dec_stride = nblocks
// rounded up to a whole wave, so every lane stores unconditionally), one coalesced store per wave per
// step; after the last step the same lane finds the lowest-index minimum and walks its own
// decisions back (reference :71-90), writing the reference's MSB-first output buffer (tail bits
// included) and, optionally, counting bit errors against the transmitted info bits
// (consumer AWGN-channel/main.c:118-144) with one atomic per wave.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "trellis.hpp"

namespace ccv {

template <int S>
using DecWord = typename std::conditional<(S > 32), uint64_t, uint32_t>::type;

// fp32 min without the IEEE-mode canonicalisation (v_max x,x) hipcc inserts around fminf. Inputs
// are always results of v_add_f32 (or +inf), so no signalling NaN can reach it.
__device__ __forceinline__ float vmin(float a, float b) {
#ifdef CCV_VMIN_BUILTIN
  return __builtin_fminf(a, b);
#else
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
#endif
}
__device__ __forceinline__ uint32_t vmin(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint16_t vmin(uint16_t a, uint16_t b) { return a < b ? a : b; }
// 16-bit metrics (the BSC reference keeps uint16_t ones): v_add_u16 / v_min_u16 issue at full rate on
// gfx950 where v_min_u32 is half rate (profiles/r01_rates_packed16.txt). The hard kernels use plain
// uint16_t: hipcc selects v_add_u16 / v_min_u16, knows they zero the high half, so the decision is
// the sign of the full-rate 32-bit m1 - m0 with no extension; two things keep it there: the branch
// metrics pass through an empty asm (else every add becomes a half-rate v_bcnt with accumulate) and
// the decision words start from an opaque zero (acs_step). H16 below pins the same ops by inline asm
// (the round-2 first cut, kept as the viterbi_hard_persist MMODE 0 ablation): hipcc cannot see into
// the asm and puts an s_nop after every such op whose result is read next, 6 % slower.
struct H16 {
  uint32_t v;
};
__device__ __forceinline__ H16 operator+(H16 a, H16 b) {
  H16 r;
  asm("v_add_u16_e32 %0, %1, %2" : "=v"(r.v) : "v"(a.v), "v"(b.v));
  return r;
}
__device__ __forceinline__ H16 vmin(H16 a, H16 b) {
  H16 r;
  asm("v_min_u16_e32 %0, %1, %2" : "=v"(r.v) : "v"(a.v), "v"(b.v));
  return r;
}

// shift the decision (m1 < m0) into d: sign bit of m1 - m0 (exact for finite fp32 and for
// finite-vs-inf; inf-inf only occurs at states no traceback can reach).
__device__ __forceinline__ uint32_t shift_in(uint32_t d, float m0, float m1) {
  return (d << 1) | (__float_as_uint(m1 - m0) >> 31);
}
__device__ __forceinline__ uint32_t shift_in(uint32_t d, uint32_t m0, uint32_t m1) {
  return (d << 1) | ((m1 - m0) >> 31);
}
__device__ __forceinline__ uint32_t shift_in(uint32_t d, uint16_t m0, uint16_t m1) {
  return __builtin_amdgcn_alignbit(d, (uint32_t)m1 - (uint32_t)m0, 31);
}
__device__ __forceinline__ uint32_t shift_in(uint32_t d, H16 m0, H16 m1) {
  uint32_t diff;
  asm("v_sub_u32_e32 %0, %1, %2" : "=v"(diff) : "v"(m1.v), "v"(m0.v));
  return __builtin_amdgcn_alignbit(d, diff, 31);
}

// The first of 32 inserts into a word on integer metrics: every bit of the word it starts from is
// shifted out again, so hipcc drops the opaque zero and turns alignbit(0, m1 - m0, 31) into
// v_cmp -> VCC -> v_cndmask (a VCC round trip per word per step in the BSC kernels). The sign of
// m1 - m0 by an explicit full-rate v_lshrrev_b32 instead.
__device__ __forceinline__ uint32_t first_in(uint16_t m0, uint16_t m1) {
  uint32_t r;
  asm("v_lshrrev_b32 %0, 31, %1" : "=v"(r) : "v"((uint32_t)m1 - (uint32_t)m0));
  return r;
}
__device__ __forceinline__ uint32_t first_in(uint32_t m0, uint32_t m1) {
  uint32_t r;
  asm("v_lshrrev_b32 %0, 31, %1" : "=v"(r) : "v"(m1 - m0));
  return r;
}
template <typename MT>
__device__ __forceinline__ uint32_t insert_first(uint32_t d, MT m0, MT m1) {
  if constexpr (std::is_same_v<MT, uint16_t> || std::is_same_v<MT, uint32_t>) return first_in(m0, m1);
  else return shift_in(d, m0, m1);
}

// Insert the decision (m1 < m0) at bit `holes` of (d << (holes + 1)), leaving `holes` don't-care
// bits below it for positions that are filled by copy_collapsed (v_alignbit takes the top
// holes + 1 bits of m1 - m0: the sign, then garbage).
template <int HOLES>
__device__ __forceinline__ uint32_t shift_in_n(uint32_t d, float m0, float m1) {
  if constexpr (HOLES == 0) return shift_in(d, m0, m1);
  else return __builtin_amdgcn_alignbit(d, __float_as_uint(m1 - m0), 31 - HOLES);
}
template <int HOLES>
__device__ __forceinline__ uint32_t shift_in_n(uint32_t d, uint32_t m0, uint32_t m1) {
  if constexpr (HOLES == 0) return shift_in(d, m0, m1);
  else return __builtin_amdgcn_alignbit(d, m1 - m0, 31 - HOLES);
}
template <int HOLES>
__device__ __forceinline__ uint32_t shift_in_n(uint32_t d, uint16_t m0, uint16_t m1) {
  return __builtin_amdgcn_alignbit(d, (uint32_t)m1 - (uint32_t)m0, 31 - HOLES);
}
template <int HOLES>
__device__ __forceinline__ uint32_t shift_in_n(uint32_t d, H16 m0, H16 m1) {
  uint32_t diff;
  asm("v_sub_u32_e32 %0, %1, %2" : "=v"(diff) : "v"(m1.v), "v"(m0.v));
  return __builtin_amdgcn_alignbit(d, diff, 31 - HOLES);
}

// Butterfly j (old states 2j, 2j+1) is "collapsed" when both old states emit the same symbol for
// input 0 and input 1 (the x86-idiom codes: 16 of the 32 butterflies of K=7 (171,133)). Then new
// states j and j + S/2 have bit-identical candidates, hence the same metric (the compiler keeps
// one) and the same decision: the upper word takes those bits from the lower word with ONE
// v_bitop3 select instead of one v_alignbit each.
template <CodeSpec C>
constexpr bool collapsed_butterfly(int j) {
  return expected_symbol(C, 2 * j, 0) == expected_symbol(C, 2 * j, 1) &&
         expected_symbol(C, 2 * j + 1, 0) == expected_symbol(C, 2 * j + 1, 1);
}
template <CodeSpec C>
constexpr uint32_t collapsed_mask() {
  uint32_t m = 0;
  for (int j = 0; j < (1 << (C.K - 2)); ++j)
    if (collapsed_butterfly<C>(j)) m |= 1u << j;
  return m;
}
// consecutive collapsed butterflies directly below j (filled later, skipped by j's insert)
template <CodeSpec C>
constexpr int collapsed_below(int j) {
  int h = 0;
  for (int k = j - 1; k >= 0 && collapsed_butterfly<C>(k); --k) ++h;
  return h;
}

// v_bitop3_b32 truth table index = (src0 << 2) | (src1 << 1) | src2 (checked on the device:
// tools/acs_unit.hip), so src0 ? src1 : src2 is 0xCA.
__device__ __forceinline__ uint32_t select_bits(uint32_t mask, uint32_t if_set, uint32_t if_clear) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r) : "s"(mask), "v"(if_set), "v"(if_clear));
  return r;
}

template <int NS>
struct SoftStep {
  float v[NS];
};

template <int NS, int NT = 0>
__device__ __forceinline__ SoftStep<NS> load_soft_step(const float* p) {
  SoftStep<NS> r;
  if constexpr (NS == 2) {
    float2 a = *reinterpret_cast<const float2*>(p);
    r.v[0] = a.x; r.v[1] = a.y;
  } else if constexpr (NS % 4 == 0) {
#pragma unroll
    for (int q = 0; q < NS / 4; ++q) {
      float4 a;
      if constexpr (NT) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p) + q);
        a = float4{v.x, v.y, v.z, v.w};
      } else {
        a = reinterpret_cast<const float4*>(p)[q];
      }
      r.v[4 * q] = a.x; r.v[4 * q + 1] = a.y; r.v[4 * q + 2] = a.z; r.v[4 * q + 3] = a.w;
    }
  } else {
#pragma unroll
    for (int q = 0; q < NS; ++q) r.v[q] = p[q];
  }
  return r;
}

// One trellis step for one block held in registers. BM[k] = branch metric of expected symbol k.
template <CodeSpec C, bool SAT, typename MT>
__device__ __forceinline__ DecWord<(1 << (C.K - 1))> acs_step(MT (&M)[1 << (C.K - 1)],
                                                              const MT (&BM)[1 << C.n]) {
  constexpr int S = 1 << (C.K - 1);
  constexpr int H = S / 2;
  MT N[S];
  uint32_t dlo = 0, dhi = 0;
  constexpr bool kIntMetric = std::is_same_v<MT, uint16_t> || std::is_same_v<MT, uint32_t>;
  if constexpr (kIntMetric) {
    // an opaque zero: alignbit(0, m1 - m0, 31) on integer metrics is otherwise folded into
    // v_cmp -> VCC -> v_cndmask (~7 ns per instruction on gfx950, tools/raterbench6.hip)
    asm volatile("" : "+v"(dlo));
    asm volatile("" : "+v"(dhi));
  }
  if constexpr (collapsed_mask<C>() == 0) {
#pragma unroll
    for (int j = H - 1; j >= 0; --j) {
      MT a0 = M[2 * j] + BM[expected_symbol(C, 2 * j, 0)];
      MT a1 = M[2 * j + 1] + BM[expected_symbol(C, 2 * j + 1, 0)];
      MT b0 = M[2 * j] + BM[expected_symbol(C, 2 * j, 1)];
      MT b1 = M[2 * j + 1] + BM[expected_symbol(C, 2 * j + 1, 1)];
      if constexpr (SAT) {  // binary-symmetric-channel/viterbi-decoder.c:127-130
        a0 = vmin(a0, (MT)0xFF00); a1 = vmin(a1, (MT)0xFF00);
        b0 = vmin(b0, (MT)0xFF00); b1 = vmin(b1, (MT)0xFF00);
      }
      N[j] = vmin(a0, a1);
      if (kIntMetric && H >= 32 && j == H - 1) dlo = insert_first(dlo, a0, a1);
      else dlo = shift_in(dlo, a0, a1);
      N[j + H] = vmin(b0, b1);
      if (kIntMetric && H >= 32 && j == H - 1) dhi = insert_first(dhi, b0, b1);
      else dhi = shift_in(dhi, b0, b1);
    }
  } else [&]<int... js>(std::integer_sequence<int, js...>) __attribute__((always_inline)) {
    ([&]() __attribute__((always_inline)) {
      constexpr int j = H - 1 - js;   // descending: state j ends up in bit j
      MT a0 = M[2 * j] + BM[expected_symbol(C, 2 * j, 0)];
      MT a1 = M[2 * j + 1] + BM[expected_symbol(C, 2 * j + 1, 0)];
      MT b0 = M[2 * j] + BM[expected_symbol(C, 2 * j, 1)];
      MT b1 = M[2 * j + 1] + BM[expected_symbol(C, 2 * j + 1, 1)];
      if constexpr (SAT) {  // binary-symmetric-channel/viterbi-decoder.c:127-130
        a0 = vmin(a0, (MT)0xFF00); a1 = vmin(a1, (MT)0xFF00);
        b0 = vmin(b0, (MT)0xFF00); b1 = vmin(b1, (MT)0xFF00);
      }
      N[j] = vmin(a0, a1);
      if constexpr (kIntMetric && H >= 32 && j == H - 1) dlo = insert_first(dlo, a0, a1);
      else dlo = shift_in(dlo, a0, a1);
      N[j + H] = vmin(b0, b1);
      if constexpr (!collapsed_butterfly<C>(j)) dhi = shift_in_n<collapsed_below<C>(j)>(dhi, b0, b1);
    }(), ...);
  }(std::make_integer_sequence<int, H>{});
  if constexpr (collapsed_mask<C>() != 0) dhi = select_bits(collapsed_mask<C>(), dlo, dhi);
#pragma unroll
  for (int s = 0; s < S; ++s) M[s] = N[s];
  if constexpr (S > 32) return ((uint64_t)dhi << 32) | dlo;
  else return (dhi << H) | dlo;
}

struct RegArgs {
  const void* in;          // soft: float [nb][T][2^n] (or [T][nb][2^n], step-major); hard: uint8 [nb][T]
  int T;
  int nblocks;
  int blen;
  int dec_stride;          // blocks per decision row: nblocks rounded up to kRegThreads
  uint8_t* out;            // [nb][OB]
  int32_t* path_metric;    // hard only, may be null
  void* dec;               // [T][dec_stride] DecWord
  const uint8_t* info;     // optional [nb][IB] transmitted info bytes (error counting)
  unsigned long long* err; // optional error accumulator
  uint32_t* queue;         // persistent kernels: the group queue (acs_persist.hpp GroupQueue), zeroed
  uint32_t* stamps;        // diagnostic builds only (kPersistStamp): 8 words per wave
};

constexpr int kRegThreads = 64;   // one wave per workgroup: spreads small batches over more CUs

// Lowest-index minimum (reference traceback :72-79, strict < from the sentinel) without a
// compare/select chain: hipcc turns `lt = M[s] < best; best = lt ? ..; idx = lt ? ..` into
// v_cmp -> VCC -> two v_cndmask per state, ~20 ns per state per SIMD on gfx950 (VCC round trip,
// tools/raterbench6.hip) -- as much as seven K=7 ACS steps per block. Instead: a v_min3 tree for the
// minimum mn, then per state the sign of mn - M[s] -- 0 exactly when M[s] == mn -- shifted into a
// "differs" mask (one v_sub and one v_alignbit per state), whose lowest clear bit is the state.
// mn - M[s] is +0 on equality because path metrics are never -0 (sums that start from the +0 reset
// metric: x + y is -0 only when both are) and never NaN (finite inputs); a larger M[s], +inf
// included, gives a negative difference. Hard metrics are u32 below 2^31: the integer difference.
__device__ __forceinline__ uint32_t min_minus(float mn, float m) { return __float_as_uint(mn - m); }
__device__ __forceinline__ uint32_t min_minus(uint32_t mn, uint32_t m) { return mn - m; }
__device__ __forceinline__ float vmin3(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t vmin3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
template <int N, typename MT>
__device__ __forceinline__ MT tree_min(const MT* v) {
  if constexpr (N == 1) return v[0];
  else if constexpr (N == 2) return vmin(v[0], v[1]);
  else {
    constexpr int P = (N + 2) / 3;   // parents: min3 over triples, a ragged tail as min / copy
    MT p[P];
#pragma unroll
    for (int i = 0; i < P; ++i) {
      if (3 * i + 2 < N) p[i] = vmin3(v[3 * i], v[3 * i + 1], v[3 * i + 2]);
      else if (3 * i + 1 < N) p[i] = vmin(v[3 * i], v[3 * i + 1]);
      else p[i] = v[3 * i];
    }
    return tree_min<P, MT>(p);
  }
}
template <int S, typename MT>
__device__ __forceinline__ int argmin_state(const MT (&M)[S], MT sentinel, MT& best) {
  constexpr int W = (S + 31) / 32;
  const MT mn = tree_min<S, MT>(M);
  uint32_t ne[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    ne[w] = S < 32 ? ~0u : 0u;   // states past S differ
    constexpr int top = S < 32 ? S : 32;
#pragma unroll
    for (int k = top - 1; k >= 0; --k)   // descending: state 32w + k ends up in bit k
      ne[w] = __builtin_amdgcn_alignbit(ne[w], min_minus(mn, M[32 * w + k]), 31);
  }
  int idx;
  if constexpr (W == 1) idx = __builtin_ctz(~ne[0]);
  else idx = __builtin_ctzll(~(((uint64_t)ne[1] << 32) | ne[0]));
  const bool found = mn < sentinel;   // nothing below the sentinel: state 0, best = sentinel
  best = found ? mn : sentinel;
  return found ? idx : 0;
}

// Walk decisions back from `st`, write the MSB-first output buffer, count errors.
template <int K>
__device__ __forceinline__ uint32_t traceback(const RegArgs& a, int b, uint32_t st) {
  constexpr int S = 1 << (K - 1);
  using DW = DecWord<S>;
  const DW* dec = reinterpret_cast<const DW*>(a.dec) + b;
  const int T = a.T, OB = (T + 7) >> 3, IB = (a.blen + 7) >> 3;
  const size_t stride = (size_t)a.dec_stride;
  uint32_t errors = 0;
  for (int lo = (T - 1) & ~7; lo >= 0; lo -= 8) {
    DW d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = dec[(size_t)(lo + k < T ? lo + k : T - 1) * stride];
    uint32_t acc = 0;
#pragma unroll
    for (int k = 7; k >= 0; --k) {
      if (lo + k < T) {
        uint32_t bit = (uint32_t)(d[k] >> st) & 1u;
        acc |= (st >> (K - 2)) << (7 - k);
        st = ((st << 1) & (S - 1)) | bit;
      }
    }
    a.out[(size_t)b * OB + (lo >> 3)] = (uint8_t)acc;
    if (a.info != nullptr && (lo >> 3) < IB) {
      int valid = a.blen - lo;
      valid = valid > 8 ? 8 : valid;
      uint32_t mask = (0xFFu << (8 - valid)) & 0xFFu;
      errors += __builtin_popcount((acc ^ a.info[(size_t)b * IB + (lo >> 3)]) & mask);
    }
  }
  return errors;
}

__device__ __forceinline__ void accumulate_errors(const RegArgs& a, uint32_t errors) {
  if (a.err == nullptr) return;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) errors += __shfl_xor(errors, off, 64);
  if ((threadIdx.x & 63) == 0 && errors) atomicAdd(a.err, (unsigned long long)errors);
}

// Steps [t_begin, T) with PF steps of input in flight. The main loop is straight-line (no bounds
// checks, every load and store unconditional) so the compiler can wait for each load with a counted
// vmcnt instead of draining the memory pipe (stores included) every iteration.
template <int PF, class In, class Load, class Step>
__device__ __forceinline__ void pipelined_steps(int t_begin, int T, Load&& load, Step&& step) {
  In ring[PF];
#pragma unroll
  for (int k = 0; k < PF; ++k) ring[k] = load(t_begin + k < T ? t_begin + k : T - 1);
  int t = t_begin;
  for (; t + 2 * PF <= T; t += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      // consume the slot, then refill it: the load can land in the same registers, so the loop
      // back-edge needs no copies (a copy would wait for the load and collapse the prefetch)
      step(ring[u], t + u);
      ring[u] = load(t + u + PF);
      __builtin_amdgcn_sched_barrier(0);   // keep each refill at its step (the scheduler sinks them)
    }
  }
  for (; t < T; t += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      if (t + u < T) {
        In cur = ring[u];
        if (t + u + PF < T) ring[u] = load(t + u + PF);
        step(cur, t + u);
      }
    }
  }
}

// How a lane gets its block's per-step input.
enum SoftLoad : int {
  kLoadPerStep = 0,    // block-major input, each lane loads its own step (64 cache lines per load)
  kLoadStepMajor = 2,  // step-major input [T][nblocks][2^n]: one 1 KiB coalesced load per step
  kLoadLdsDma = 3,     // block-major input, the wave stages PF steps of its 64 blocks in LDS with
                       // global_load_lds (LDS-DMA, no VGPR staging); each lane then reads its own
                       // chunk into registers and the next chunk's DMA runs under the ACS
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Ablation switches for timing studies (tools/kbench.hip); production kernels use 0.
enum : int { kAblateDecStore = 1, kAblateTraceback = 2, kAblateLoads = 4 };

// Soft-decision register-trellis kernel. MODE selects the input path (SoftLoad); PF is the input
// prefetch depth in steps (per-step modes) or the steps staged per LDS round (kLoadLdsDma).
template <CodeSpec C, int MODE, int PF, int ABLATE = 0, int NT = 0, int WAVES = 1>
__global__ __launch_bounds__(kRegThreads) __attribute__((amdgpu_waves_per_eu(WAVES)))
void viterbi_soft_reg(RegArgs a) {
  constexpr int S = 1 << (C.K - 1);
  constexpr int NS = 1 << C.n;
  using DW = DecWord<S>;
  const int lane = threadIdx.x;
  const int block0 = blockIdx.x * kRegThreads;
  const int b = block0 + lane;
  const int T = a.T, nb = a.nblocks;
  DW* dec = reinterpret_cast<DW*>(a.dec) + b;   // padded rows: every lane owns a column
  const size_t dstride = (size_t)a.dec_stride;
  float M[S];
#pragma unroll
  for (int s = 0; s < S; ++s) M[s] = s ? __builtin_inff() : 0.0f;   // viterbi-decoder.c:212-218
  auto step = [&](const SoftStep<NS>& in, int t) {
    DW d = acs_step<C, false, float>(M, in.v);
    if constexpr ((ABLATE & kAblateDecStore) != 0) asm volatile("" ::"v"(d));
    else dec[(size_t)t * dstride] = d;
  };

  if constexpr (MODE == kLoadLdsDma) {
    static_assert(NS >= 4, "LDS-DMA staging needs 16-byte trellis steps");
    constexpr int SB = NS * 4;                 // bytes per trellis step
    constexpr int UPR = PF * SB / 16;          // 16-byte units per block per chunk (= DMAs per chunk)
    static_assert(UPR == 4 || UPR == 8 || UPR == 16, "chunk must be 64, 128 or 256 bytes per block");
    constexpr int ROWB = UPR * 16;
    constexpr int GRP = 16 / UPR;
    // LDS image [block r][slot j]: slot j of row r holds 16-byte unit j ^ sw(r) of block r's chunk.
    // The DMA writes lane-linearly, so the swizzle is applied to the per-lane SOURCE address; with
    // sw(r) = (r / GRP) % UPR every ds_read_b128 lane group (MI355X_MICROARCH.md, LDS) touches 16
    // distinct 16-byte bank groups: conflict-free.
    __shared__ __attribute__((aligned(16))) unsigned char lds[kRegThreads * ROWB];
    const unsigned char* in = reinterpret_cast<const unsigned char*>(a.in);
    const size_t block_bytes = (size_t)T * SB;
    auto issue_chunk = [&](int t0) {
#pragma unroll
      for (int k = 0; k < UPR; ++k) {
        const int unit = k * kRegThreads + lane;
        const int r = unit / UPR, j = unit % UPR;
        const int su = j ^ ((r / GRP) % UPR);
        const int gb = block0 + r < nb ? block0 + r : nb - 1;
        size_t off = (size_t)t0 * SB + (size_t)su * 16;
        off = off < block_bytes ? off : block_bytes - 16;   // past the block: clamped, never read
        // NT: the input is read exactly once -- keep it from displacing the decision scratch
        __builtin_amdgcn_global_load_lds(in + (size_t)gb * block_bytes + off,
                                         (lds_ptr_t)(lds + k * kRegThreads * 16), 16, 0, NT ? 2 : 0);
      }
    };
    const int sw = (lane / GRP) % UPR;
    const unsigned char* row = lds + lane * ROWB;
    // Decisions of a chunk are held in registers and stored right after the NEXT chunk's DMA is
    // issued: the LDS read at a chunk start must wait for the DMA (vmcnt counts stores too, and the
    // compiler waits for all of them), so only operations issued a whole chunk earlier may be
    // pending there -- otherwise every chunk start drains the stores just issued.
    DW dbuf[PF];
    auto store_chunk = [&](int tc, bool full) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        if constexpr ((ABLATE & kAblateDecStore) != 0) asm volatile("" ::"v"(dbuf[u]));
        else if (full || tc + u < T) dec[(size_t)(tc + u) * dstride] = dbuf[u];
      }
    };
    auto read_chunk = [&](float4 (&chunk)[UPR]) {
#pragma unroll
      for (int x = 0; x < UPR; ++x) chunk[x] = *reinterpret_cast<const float4*>(row + ((x ^ sw) * 16));
    };
    auto acs = [&](const float4 (&chunk)[UPR], int u) {
      SoftStep<NS> cur;
#pragma unroll
      for (int q = 0; q < NS / 4; ++q) {
        const float4 v = chunk[u * (NS / 4) + q];
        cur.v[4 * q] = v.x; cur.v[4 * q + 1] = v.y; cur.v[4 * q + 2] = v.z; cur.v[4 * q + 3] = v.w;
      }
      dbuf[u] = acs_step<C, false, float>(M, cur.v);
      __builtin_amdgcn_sched_barrier(0);   // schedule step by step: interleaving steps only adds VGPRs
    };
    issue_chunk(0);
    const int full_end = T / PF * PF;
    int t0 = 0;
    // full chunks: straight-line steps (no per-step guards for the compiler to if-convert)
    for (; t0 < full_end; t0 += PF) {
      float4 chunk[UPR];
      read_chunk(chunk);
      if (t0 + PF < T) {
        // the chunk is in registers once these reads return; only then may the DMA overwrite it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue_chunk(t0 + PF);                  // lands while this chunk is decoded
      }
      if (t0 > 0) store_chunk(t0 - PF, true);
#pragma unroll
      for (int u = 0; u < PF; ++u) acs(chunk, u);
    }
    if (t0 < T) {
      // the partial last chunk: one step per iteration straight from LDS (a rolled loop -- unrolled
      // guarded steps make the register allocator keep two copies of the metrics)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (t0 > 0) store_chunk(t0 - PF, true);
#pragma unroll 1
      for (int u = 0; t0 + u < T; ++u) {
        SoftStep<NS> cur;
#pragma unroll
        for (int q = 0; q < NS / 4; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(row + (((u * (NS / 4) + q) ^ sw) * 16));
          cur.v[4 * q] = v.x; cur.v[4 * q + 1] = v.y; cur.v[4 * q + 2] = v.z; cur.v[4 * q + 3] = v.w;
        }
        const DW d = acs_step<C, false, float>(M, cur.v);
        if constexpr ((ABLATE & kAblateDecStore) != 0) asm volatile("" ::"v"(d));
        else dec[(size_t)(t0 + u) * dstride] = d;
      }
    } else {
      store_chunk(t0 - PF, true);
    }
  } else {
    // per-lane step loads: block-major (64 distinct lines per load) or step-major (coalesced)
    const int bc = b < nb ? b : nb - 1;   // lanes past the batch replay a valid block
    const float* p = reinterpret_cast<const float*>(a.in) +
                     (MODE == kLoadStepMajor ? (size_t)bc * NS : (size_t)bc * T * NS);
    const size_t stride = MODE == kLoadStepMajor ? (size_t)nb * NS : (size_t)NS;
    if constexpr ((ABLATE & kAblateLoads) != 0) {
      for (int t = 0; t < T; ++t) {   // synthetic input from registers: VALU-only timing
        SoftStep<NS> in;
#pragma unroll
        for (int k = 0; k < NS; ++k) in.v[k] = (float)((lane + t + k) & 7);
        step(in, t);
      }
    } else {
      pipelined_steps<PF, SoftStep<NS>>(0, T, [&](int t) { return load_soft_step<NS, NT>(p + t * stride); },
                                        step);
    }
  }
  uint32_t errors = 0;
  if (b < nb) {
    float best;
    uint32_t st = (uint32_t)argmin_state<S, float>(M, __builtin_inff(), best);
    if constexpr ((ABLATE & kAblateTraceback) != 0) a.out[b] = (uint8_t)st;
    else errors = traceback<C.K>(a, b, st);
  }
  accumulate_errors(a, errors);
}

// ---------------------------------------------------------------------------------------------
// Register-resident decisions (r = 1/2 codes, K <= 7, T <= kRegDecMaxChunks * 8).
//
// The decision bits of a whole block (T x 2^(K-1) bits: 368 B at K=7, T=46) stay in VGPRs, so the
// kernel writes no decision scratch and its traceback reads no memory: HBM traffic is the input
// stream plus the output bytes (decisions are part of the algorithmic bytes, but
// they never leave the chip). The price is ~96 more VGPRs, i.e. 2 waves per SIMD instead of 3.
//
// The block is cut into 8-step chunks that end at step T: the first chunk is padded in FRONT with
// `pad = 8*nch - T` neutral steps whose branch metrics are {0 for symbol 0, +inf otherwise}. From the
// reset metrics (0, +inf, ...) such a step reproduces them exactly (state 0 -> 0 via symbol 0; every
// other new state sees +inf), provided the input-1 branch out of state 0 has a non-zero expected
// symbol (checked on the host). Every chunk is then a full straight-line 8-step chunk, and decision
// word u of chunk c belongs to real step 8c + u - pad: static register indices throughout.
constexpr int kRegDecMaxChunks = 6;

template <CodeSpec C, int MAXC = kRegDecMaxChunks>
__global__ __launch_bounds__(kRegThreads) __attribute__((amdgpu_waves_per_eu(2, 2)))
void viterbi_soft_regdec(RegArgs a) {
  constexpr int S = 1 << (C.K - 1);
  constexpr int NS = 1 << C.n;
  static_assert(NS == 4, "register-resident decisions: 16-byte steps (r = 1/2)");
  constexpr int PF = 8;                      // steps per chunk
  constexpr int UPR = PF;                    // 16-byte units per block per chunk (one per step)
  constexpr int ROWB = UPR * 16;
  constexpr int GRP = 16 / UPR;
  using DW = DecWord<S>;
  const int lane = threadIdx.x;
  const int block0 = blockIdx.x * kRegThreads;
  const int b = block0 + lane;
  const int T = a.T, nb = a.nblocks;
  const int nch = (T + PF - 1) / PF;         // host guarantees 1 <= nch <= MAXC
  const int pad = nch * PF - T;
  float M[S];
#pragma unroll
  for (int s = 0; s < S; ++s) M[s] = s ? __builtin_inff() : 0.0f;   // viterbi-decoder.c:212-218

  __shared__ __attribute__((aligned(16))) unsigned char lds[kRegThreads * ROWB];
  const unsigned char* in = reinterpret_cast<const unsigned char*>(a.in);
  const long block_bytes = (long)T * 16;
  // chunk c holds real steps [c*PF - pad, c*PF - pad + PF); units before step 0 are replaced by the
  // neutral step after the read, so their source is clamped to step 0
  auto issue_chunk = [&](int c) {
#pragma unroll
    for (int k = 0; k < UPR; ++k) {
      const int unit = k * kRegThreads + lane;
      const int r = unit / UPR, j = unit % UPR;
      const int su = j ^ ((r / GRP) % UPR);
      const int gb = block0 + r < nb ? block0 + r : nb - 1;
      long off = ((long)c * PF - pad + su) * 16;
      off = off < 0 ? 0 : off;
      __builtin_amdgcn_global_load_lds(in + (size_t)gb * block_bytes + off,
                                       (lds_ptr_t)(lds + k * kRegThreads * 16), 16, 0, 0);
    }
  };
  const int sw = (lane / GRP) % UPR;
  const unsigned char* row = lds + lane * ROWB;

  DW D[MAXC][PF];
  // one copy of the chunk code per chunk index (template expansion, not a loop the unroller may
  // keep rolled): every D[c][u] index is a constant, so the decisions stay in VGPRs
  auto chunk_at = [&]<int c>() {
    if (c < nch) {
      float4 chunk[UPR];
#pragma unroll
      for (int x = 0; x < UPR; ++x) chunk[x] = *reinterpret_cast<const float4*>(row + ((x ^ sw) * 16));
      if (c + 1 < nch) {
        // the chunk is in registers once these reads return; only then may the DMA overwrite it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue_chunk(c + 1);                    // lands while this chunk is decoded
      }
      if constexpr (c == 0) {
#pragma unroll
        for (int x = 0; x < UPR; ++x)
          if (x < pad) chunk[x] = float4{0.0f, __builtin_inff(), __builtin_inff(), __builtin_inff()};
      }
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const float bm[4] = {chunk[u].x, chunk[u].y, chunk[u].z, chunk[u].w};
        D[c][u] = acs_step<C, false, float>(M, bm);
        __builtin_amdgcn_sched_barrier(0);   // schedule step by step: interleaving steps only adds VGPRs
      }
    }
  };
  issue_chunk(0);
  [&]<int... cs>(std::integer_sequence<int, cs...>) {
    (chunk_at.template operator()<cs>(), ...);
  }(std::make_integer_sequence<int, MAXC>{});

  uint32_t errors = 0;
  if (b < nb) {
    float best;
    uint32_t st = (uint32_t)argmin_state<S, float>(M, __builtin_inff(), best);
    // traceback (reference :71-90) over register decisions; the decoded bits of steps T-1 ... 0
    // are shifted in from the top, so bit 63 ends up holding step 0 (MSB-first output)
    uint64_t bits = 0;
    auto back_chunk = [&]<int c>() {
      if (c < nch) {
#pragma unroll
        for (int u = PF - 1; u >= 0; --u) {
          if (c > 0 || u >= pad) {
            const uint32_t d = (uint32_t)(D[c][u] >> st) & 1u;
            bits = (bits >> 1) | ((uint64_t)(st >> (C.K - 2)) << 63);
            st = ((st << 1) & (S - 1)) | d;
          }
        }
      }
    };
    [&]<int... cs>(std::integer_sequence<int, cs...>) {
      (back_chunk.template operator()<MAXC - 1 - cs>(), ...);
    }(std::make_integer_sequence<int, MAXC>{});
    const int OB = (T + 7) >> 3, IB = (a.blen + 7) >> 3;
    uint8_t* o = a.out + (size_t)b * OB;
    for (int k = 0; k < OB; ++k) o[k] = (uint8_t)(bits >> (56 - 8 * k));
    if (a.info != nullptr) {   // consumer AWGN-channel/main.c:118-144: errors in the first blen bits
      const uint8_t* inf = a.info + (size_t)b * IB;
      uint64_t ref = 0;
      for (int k = 0; k < IB; ++k) ref |= (uint64_t)inf[k] << (56 - 8 * k);
      const uint64_t mask = a.blen >= 64 ? ~0ull : ~(~0ull >> a.blen);
      errors = (uint32_t)__builtin_popcountll((bits ^ ref) & mask);
    }
  }
  accumulate_errors(a, errors);
}

// Production input path for block-major soft input: LDS-DMA staging where a step is at least 16
// bytes (n >= 2) -- 8-step (128-byte) chunks for n = 2, 4-step chunks for n = 3 -- per-lane loads
// otherwise (tools/kbench.hip compares the paths; profiles/r01_kbench_variants.txt).
template <int NS>
inline constexpr int kSoftMode = NS >= 4 ? kLoadLdsDma : kLoadPerStep;
template <int NS>
inline constexpr int kSoftPF = NS == 4 ? 8 : (NS >= 8 ? 4 : 8);
constexpr int kSoftStepMajorPF = 4;        // prefetch depth, step-major input
constexpr int kHardPF = 8;                 // prefetch depth, hard decision

template <CodeSpec C>
__global__ __launch_bounds__(kRegThreads) void viterbi_hard_reg(RegArgs a) {
  constexpr int S = 1 << (C.K - 1);
  constexpr int NS = 1 << C.n;
  using DW = DecWord<S>;
  const int b = blockIdx.x * kRegThreads + threadIdx.x;
  const int T = a.T, nb = a.nblocks;
  const int bc = b < nb ? b : nb - 1;
  const uint8_t* p = reinterpret_cast<const uint8_t*>(a.in) + (size_t)bc * T;
  DW* dec = reinterpret_cast<DW*>(a.dec) + b;
  const size_t dstride = (size_t)a.dec_stride;
  constexpr uint32_t kMask = NS - 1;   // decoder_input masks to n bits (viterbi-decoder.c:235-237)
  uint32_t M[S];
#pragma unroll
  for (int s = 0; s < S; ++s) M[s] = s ? 0xFF00u : 0u;   // viterbi-decoder.c:225-228
  auto branch_metrics = [](uint32_t sym, uint32_t (&BM)[NS]) {
#pragma unroll
    for (int k = 0; k < NS; ++k) BM[k] = __builtin_popcount((uint32_t)k ^ (sym & kMask));
  };
  // The first K-1 steps still have unreachable states, whose metrics saturate at 0xFF00 as in the
  // reference; afterwards every metric is <= n*T < 0xFF00 - n and saturation is a no-op.
  const int t0 = T < C.K - 1 ? T : C.K - 1;
  for (int t = 0; t < t0; ++t) {
    uint32_t BM[NS];
    branch_metrics(p[t], BM);
    dec[(size_t)t * dstride] = acs_step<C, true, uint32_t>(M, BM);
  }
  // afterwards every metric is <= n*T < 2^15: the ACS runs on 16-bit metrics, exactly the
  // reference's uint16_t arithmetic
  uint16_t M16[S];
#pragma unroll
  for (int s = 0; s < S; ++s) M16[s] = (uint16_t)M[s];
  pipelined_steps<kHardPF, uint32_t>(t0, T, [&](int t) { return (uint32_t)p[t]; },
                                     [&](uint32_t sym, int t) {
                                       uint16_t BM[NS];
#pragma unroll
                                       for (int k = 0; k < NS; ++k) {
                                         BM[k] = (uint16_t)__builtin_popcount((uint32_t)k ^ (sym & kMask));
                                         asm volatile("" : "+v"(BM[k]));   // no v_bcnt-folded adds
                                       }
                                       dec[(size_t)t * dstride] = acs_step<C, false, uint16_t>(M16, BM);
                                     });
#pragma unroll
  for (int s = 0; s < S; ++s) M[s] = M16[s];
  uint32_t errors = 0;
  if (b < nb) {
    uint32_t best;
    uint32_t st = (uint32_t)argmin_state<S, uint32_t>(M, 0xFF00u, best);
    if (a.path_metric) a.path_metric[b] = (int32_t)best;
    errors = traceback<C.K>(a, b, st);
  }
  accumulate_errors(a, errors);
}

}  // namespace ccv
