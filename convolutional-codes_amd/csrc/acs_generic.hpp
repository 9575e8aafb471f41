// acs_generic.hpp -- table-driven Viterbi kernel for any code (K <= 12, n <= 8), soft or hard.
//
// Used for codes without a register-trellis specialisation (acs_reg.hpp), notably K >= 8. One
// workgroup decodes one trellis block with one thread per new state (up to 256 threads, then SPT
// states per thread): the block's input is staged in LDS, path metrics ping-pong in LDS, each wave
// packs its decisions with a 64-bit ballot into an LDS decision array holding the whole block, and
// one lane walks the decisions back. Expected symbols come from a run-time table exp[2*s + i].
// Same ACS, tie and traceback rules as acs_reg.hpp / reference AWGN-channel/viterbi-decoder.c:71-141
// and binary-symmetric-channel/viterbi-decoder.c:75-150.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "trellis.hpp"

namespace ccv {

struct GenericArgs {
  const void* in;          // soft: float [nb][T][2^n]; hard: uint8 [nb][T]
  const uint8_t* exp;      // [S][2] expected symbols
  int n, K, T, blen, nblocks;
  int chunk;               // soft: trellis steps of input staged in LDS at a time
  uint8_t* out;            // [nb][OB]
  int32_t* path_metric;    // hard only, may be null
  const uint8_t* info;     // optional, for error counting
  unsigned long long* err; // optional
};

constexpr int kGenericMaxThreads = 256;

// Unreachable-state metric: +inf (AWGN-channel/viterbi-decoder.c:215-218) or 0xFF00
// (binary-symmetric-channel/viterbi-decoder.c:225-228).
template <bool HARD>
__device__ __forceinline__ auto unreachable_metric() {
  if constexpr (HARD) return (uint32_t)0xFF00u;
  else return __builtin_inff();
}

// LDS bytes the generic kernel needs for a code (see the carve-up in viterbi_generic).
inline size_t generic_lds_bytes(int n, int K, int T, int chunk, bool hard) {
  const size_t S = (size_t)1 << (K - 1), NS = (size_t)1 << n;
  const size_t words = (S + 63) / 64;
  size_t bytes = 2 * S * 4;                                   // metrics ping-pong
  bytes += hard ? ((size_t)T + 15) / 16 * 16 + NS * 4 : (size_t)chunk * NS * 4;  // input
  bytes += (size_t)T * words * 8;                             // decisions of the whole block
  bytes += 16 * 8;                                            // argmin scratch
  return bytes;
}

// One block, decoded by the whole workgroup (the body of viterbi_generic and of the streaming
// service kernel viterbi_service).
template <int SPT, bool HARD>
__device__ __forceinline__ void generic_decode_block(const GenericArgs& a, int b, unsigned char* lds) {
  using MT = typename std::conditional<HARD, uint32_t, float>::type;
  const int S = 1 << (a.K - 1), NS = 1 << a.n, T = a.T;
  const int tid = threadIdx.x, nthr = blockDim.x, lane = tid & 63, wave = tid >> 6;
  const int words = (S + 63) >> 6;

  MT* Ma = reinterpret_cast<MT*>(lds);
  MT* Mb = Ma + S;
  unsigned char* p = lds + 2 * (size_t)S * 4;
  float* rx_s = reinterpret_cast<float*>(p);                    // soft: [chunk][NS]
  uint8_t* sym_s = p;                                           // hard: [T] symbols
  uint32_t* hd_s = reinterpret_cast<uint32_t*>(p + (T + 15) / 16 * 16);   // hard: [NS]
  p += HARD ? (size_t)(T + 15) / 16 * 16 + (size_t)NS * 4 : (size_t)a.chunk * NS * 4;
  uint64_t* dec_s = reinterpret_cast<uint64_t*>(p);             // [T][words]
  p += (size_t)T * words * 8;
  MT* red_v = reinterpret_cast<MT*>(p);                         // [<=4] per-wave argmin
  int* red_i = reinterpret_cast<int*>(p + 32);

  // per-thread states ns = k*nthr + tid and their two expected symbols
  uint8_t e0[SPT], e1[SPT];
#pragma unroll
  for (int k = 0; k < SPT; ++k) {
    const int ns = k * nthr + tid;
    if (ns < S) {
      const int i = ns >> (a.K - 2);
      const int s0 = (ns << 1) & (S - 1);
      e0[k] = a.exp[2 * s0 + i];
      e1[k] = a.exp[2 * (s0 | 1) + i];
    }
  }
  for (int s = tid; s < S; s += nthr) Ma[s] = s ? unreachable_metric<HARD>() : (MT)0;
  if constexpr (HARD) {
    const uint8_t* src = reinterpret_cast<const uint8_t*>(a.in) + (size_t)b * T;
    for (int t = tid; t < T; t += nthr) sym_s[t] = src[t] & (uint8_t)(NS - 1);
  }
  for (int w = tid; w < T * words; w += nthr) dec_s[w] = 0;
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    if constexpr (HARD) {
      const uint32_t sym = sym_s[t];
      for (int k = tid; k < NS; k += nthr) hd_s[k] = __builtin_popcount((uint32_t)k ^ sym);
    } else {
      if (t % a.chunk == 0) {   // stage the next chunk of input steps (coalesced)
        const int steps = (T - t) < a.chunk ? (T - t) : a.chunk;
        const float* src = reinterpret_cast<const float*>(a.in) + ((size_t)b * T + t) * NS;
        for (int k = tid; k < steps * NS; k += nthr) rx_s[k] = src[k];
      }
    }
    __syncthreads();
    const float* rxt = rx_s + (size_t)(t % a.chunk) * NS;
#pragma unroll
    for (int k = 0; k < SPT; ++k) {
      const int ns = k * nthr + tid;
      bool d = false;
      if (ns < S) {
        const int s0 = (ns << 1) & (S - 1);
        MT m0, m1;
        if constexpr (HARD) {
          m0 = Ma[s0] + hd_s[e0[k]];
          m1 = Ma[s0 | 1] + hd_s[e1[k]];
          m0 = m0 > 0xFF00u ? 0xFF00u : m0;   // binary-symmetric-channel/viterbi-decoder.c:127-130
          m1 = m1 > 0xFF00u ? 0xFF00u : m1;
        } else {
          m0 = Ma[s0] + rxt[e0[k]];
          m1 = Ma[s0 | 1] + rxt[e1[k]];
        }
        d = m1 < m0;
        Mb[ns] = d ? m1 : m0;
      }
      const uint64_t bal = __ballot(d);
      const int base = k * nthr + wave * 64;
      if (lane == 0 && base < S) dec_s[t * words + (base >> 6)] = bal;
    }
    __syncthreads();
    MT* tmp = Ma; Ma = Mb; Mb = tmp;
  }

  // lowest-index minimum (reference traceback :72-79)
  MT best = unreachable_metric<HARD>();
  int idx = 0x7fffffff;
  for (int s = tid; s < S; s += nthr)
    if (Ma[s] < best) { best = Ma[s]; idx = s; }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    MT ob = __shfl_xor(best, off, 64);
    int oi = __shfl_xor(idx, off, 64);
    if (ob < best || (ob == best && oi < idx)) { best = ob; idx = oi; }
  }
  if (lane == 0) { red_v[wave] = best; red_i[wave] = idx; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < (nthr + 63) / 64; ++w)
      if (red_v[w] < best || (red_v[w] == best && red_i[w] < idx)) { best = red_v[w]; idx = red_i[w]; }
    uint32_t st = idx == 0x7fffffff ? 0u : (uint32_t)idx;
    const int OB = (T + 7) >> 3, IB = (a.blen + 7) >> 3;
    uint32_t acc = 0, errors = 0;
    for (int t = T - 1; t >= 0; --t) {
      const uint32_t bit = (uint32_t)(dec_s[t * words + (st >> 6)] >> (st & 63)) & 1u;
      acc |= (st >> (a.K - 2)) << (7 - (t & 7));
      st = ((st << 1) & (uint32_t)(S - 1)) | bit;
      if ((t & 7) == 0) {
        a.out[(size_t)b * OB + (t >> 3)] = (uint8_t)acc;
        if (a.info != nullptr && (t >> 3) < IB) {
          int valid = a.blen - t;
          valid = valid > 8 ? 8 : valid;
          const uint32_t mask = (0xFFu << (8 - valid)) & 0xFFu;
          errors += __builtin_popcount((acc ^ a.info[(size_t)b * IB + (t >> 3)]) & mask);
        }
        acc = 0;
      }
    }
    if constexpr (HARD) {
      if (a.path_metric) a.path_metric[b] = (int32_t)best;
    }
    if (a.err != nullptr && errors) atomicAdd(a.err, (unsigned long long)errors);
  }
}

template <int SPT, bool HARD>
__global__ __launch_bounds__(kGenericMaxThreads) void viterbi_generic(GenericArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  generic_decode_block<SPT, HARD>(a, blockIdx.x, lds);
}

}  // namespace ccv
