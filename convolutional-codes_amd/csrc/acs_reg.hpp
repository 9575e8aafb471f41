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
// Decisions (S bits per step) go to a [T][nblocks] array of 32/64-bit words, one coalesced store per
// wave per step; after the last step the same lane finds the lowest-index minimum and walks its own
// decisions back (reference :71-90), writing the reference's MSB-first output buffer (tail bits
// included) and, optionally, counting bit errors against the transmitted info bits
// (consumer AWGN-channel/main.c:118-144) with one atomic per wave.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "trellis.hpp"

namespace ccv {

template <int S>
using DecWord = typename std::conditional<(S > 32), uint64_t, uint32_t>::type;

// fp32 min without the IEEE-mode canonicalisation (v_max x,x) hipcc inserts around fminf. Inputs
// are always results of v_add_f32 (or +inf), so no signalling NaN can reach it.
__device__ __forceinline__ float vmin(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ uint32_t vmin(uint32_t a, uint32_t b) { return a < b ? a : b; }

// shift the decision (m1 < m0) into d: sign bit of m1 - m0 (exact for finite fp32 and for
// finite-vs-inf; inf-inf only occurs at states no traceback can reach).
__device__ __forceinline__ uint32_t shift_in(uint32_t d, float m0, float m1) {
  return (d << 1) | (__float_as_uint(m1 - m0) >> 31);
}
__device__ __forceinline__ uint32_t shift_in(uint32_t d, uint32_t m0, uint32_t m1) {
  return (d << 1) | ((m1 - m0) >> 31);
}

template <int NS>
struct SoftStep {
  float v[NS];
};

template <int NS>
__device__ __forceinline__ SoftStep<NS> load_soft_step(const float* p) {
  SoftStep<NS> r;
  if constexpr (NS == 2) {
    float2 a = *reinterpret_cast<const float2*>(p);
    r.v[0] = a.x; r.v[1] = a.y;
  } else if constexpr (NS % 4 == 0) {
#pragma unroll
    for (int q = 0; q < NS / 4; ++q) {
      float4 a = reinterpret_cast<const float4*>(p)[q];
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
    dlo = shift_in(dlo, a0, a1);
    N[j + H] = vmin(b0, b1);
    dhi = shift_in(dhi, b0, b1);
  }
#pragma unroll
  for (int s = 0; s < S; ++s) M[s] = N[s];
  if constexpr (S > 32) return ((uint64_t)dhi << 32) | dlo;
  else return (dhi << H) | dlo;
}

struct RegArgs {
  const void* in;          // soft: float [nb][T][2^n]; hard: uint8 [nb][T]
  int T;
  int nblocks;
  int blen;
  uint8_t* out;            // [nb][OB]
  int32_t* path_metric;    // hard only, may be null
  void* dec;               // [T][nb] DecWord
  const uint8_t* info;     // optional [nb][IB] transmitted info bytes (error counting)
  unsigned long long* err; // optional error accumulator
};

// Lowest-index minimum (reference traceback :72-79, strict < from the sentinel).
template <int S, typename MT>
__device__ __forceinline__ int argmin_state(const MT (&M)[S], MT sentinel, MT& best) {
  int idx = 0;
  best = sentinel;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    bool lt = M[s] < best;
    best = lt ? M[s] : best;
    idx = lt ? s : idx;
  }
  return idx;
}

// Walk decisions back from `st`, write the MSB-first output buffer, count errors.
template <int K>
__device__ __forceinline__ uint32_t traceback(const RegArgs& a, int b, uint32_t st) {
  constexpr int S = 1 << (K - 1);
  using DW = DecWord<S>;
  const DW* dec = reinterpret_cast<const DW*>(a.dec);
  const int T = a.T, nb = a.nblocks, OB = (T + 7) >> 3, IB = (a.blen + 7) >> 3;
  uint32_t errors = 0;
  for (int lo = (T - 1) & ~7; lo >= 0; lo -= 8) {
    DW d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (lo + k < T) d[k] = dec[(size_t)(lo + k) * nb + b];
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

constexpr int kRegThreads = 64;   // one wave per workgroup: spreads small batches over more CUs
constexpr int kPrefetch = 4;      // trellis steps of input kept in flight per lane

template <CodeSpec C>
__global__ __launch_bounds__(kRegThreads) void viterbi_soft_reg(RegArgs a) {
  constexpr int S = 1 << (C.K - 1);
  constexpr int NS = 1 << C.n;
  using DW = DecWord<S>;
  const int b = blockIdx.x * kRegThreads + threadIdx.x;
  uint32_t errors = 0;
  if (b < a.nblocks) {
    const int T = a.T, nb = a.nblocks;
    const float* p = reinterpret_cast<const float*>(a.in) + (size_t)b * T * NS;
    DW* dec = reinterpret_cast<DW*>(a.dec) + b;
    float M[S];
#pragma unroll
    for (int s = 0; s < S; ++s) M[s] = s ? __builtin_inff() : 0.0f;   // viterbi-decoder.c:212-218
    SoftStep<NS> ring[kPrefetch];
#pragma unroll
    for (int k = 0; k < kPrefetch; ++k)
      if (k < T) ring[k] = load_soft_step<NS>(p + k * NS);
    for (int t = 0; t < T; t += kPrefetch) {
#pragma unroll
      for (int u = 0; u < kPrefetch; ++u) {
        if (t + u < T) {
          SoftStep<NS> cur = ring[u];
          if (t + u + kPrefetch < T) ring[u] = load_soft_step<NS>(p + (t + u + kPrefetch) * NS);
          dec[(size_t)(t + u) * nb] = acs_step<C, false, float>(M, cur.v);
        }
      }
    }
    float best;
    uint32_t st = (uint32_t)argmin_state<S, float>(M, __builtin_inff(), best);
    errors = traceback<C.K>(a, b, st);
  }
  accumulate_errors(a, errors);
}

template <CodeSpec C>
__global__ __launch_bounds__(kRegThreads) void viterbi_hard_reg(RegArgs a) {
  constexpr int S = 1 << (C.K - 1);
  constexpr int NS = 1 << C.n;
  using DW = DecWord<S>;
  const int b = blockIdx.x * kRegThreads + threadIdx.x;
  uint32_t errors = 0;
  if (b < a.nblocks) {
    const int T = a.T, nb = a.nblocks;
    const uint8_t* p = reinterpret_cast<const uint8_t*>(a.in) + (size_t)b * T;
    DW* dec = reinterpret_cast<DW*>(a.dec) + b;
    constexpr uint32_t kMask = NS - 1;   // decoder_input masks to n bits (viterbi-decoder.c:235-237)
    uint32_t M[S];
#pragma unroll
    for (int s = 0; s < S; ++s) M[s] = s ? 0xFF00u : 0u;   // viterbi-decoder.c:225-228
    // The first K-1 steps still have unreachable states, whose metrics saturate at 0xFF00 as in
    // the reference; afterwards every metric is <= n*T < 0xFF00 - n and saturation is a no-op.
    const int t0 = T < C.K - 1 ? T : C.K - 1;
    for (int t = 0; t < t0; ++t) {
      uint32_t sym = p[t] & kMask;
      uint32_t BM[NS];
#pragma unroll
      for (int k = 0; k < NS; ++k) BM[k] = __builtin_popcount((uint32_t)k ^ sym);
      dec[(size_t)t * nb] = acs_step<C, true, uint32_t>(M, BM);
    }
    uint32_t ring[kPrefetch];
#pragma unroll
    for (int k = 0; k < kPrefetch; ++k)
      if (t0 + k < T) ring[k] = p[t0 + k];
    for (int t = t0; t < T; t += kPrefetch) {
#pragma unroll
      for (int u = 0; u < kPrefetch; ++u) {
        if (t + u < T) {
          uint32_t sym = ring[u] & kMask;
          if (t + u + kPrefetch < T) ring[u] = p[t + u + kPrefetch];
          uint32_t BM[NS];
#pragma unroll
          for (int k = 0; k < NS; ++k) BM[k] = __builtin_popcount((uint32_t)k ^ sym);
          dec[(size_t)(t + u) * nb] = acs_step<C, false, uint32_t>(M, BM);
        }
      }
    }
    uint32_t best;
    uint32_t st = (uint32_t)argmin_state<S, uint32_t>(M, 0xFF00u, best);
    if (a.path_metric) a.path_metric[b] = (int32_t)best;
    errors = traceback<C.K>(a, b, st);
  }
  accumulate_errors(a, errors);
}

}  // namespace ccv
