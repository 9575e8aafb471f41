// acs_latency.hpp -- one block, decoded by one wave as fast as a single block can go (K <= 7).
//
// The streaming reference API completes ONE block per decoder_input() call and fires the callback
// inside it (AWGN-channel/viterbi-decoder.c:132-139), so what matters there is the latency of a
// single block, not throughput. The register trellis (acs_reg.hpp) spends ~17 us on a lone block (one
// lane walks 46 steps of ~200 VALU at a lone wave's issue rate); the table kernel (acs_generic.hpp)
// 16.6 us (rocprof; two workgroup barriers and LDS round trips per step). Here lane s holds the path
// metric of state s: per step each lane fetches its two predecessors' metrics from lanes 2s mod S and
// 2s+1 mod S (two ds_bpermute, in flight together), adds the branch metrics of its two transitions
// (read from the block's rows in LDS), keeps the survivor (strict <: the even predecessor wins ties)
// and the wave's decisions are ONE ballot word per step (bit s = state s), kept in LDS. The argmin is
// a wave reduction (lowest index among the minima via a ballot), and the traceback walks the ballot
// words with the state uniform across the wave. Same arithmetic and tie rules as the reference
// (AWGN-channel/viterbi-decoder.c:71-141, binary-symmetric-channel/viterbi-decoder.c:75-150).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "acs_generic.hpp"

namespace ccv {

constexpr int kLatencyMaxK = 7;   // S <= 64: one state per lane

// LDS bytes: the block's rows (soft: T x 2^n floats; hard: T bytes) and T ballot words.
inline size_t latency_lds_bytes(int n, int T, bool hard) {
  const size_t rows = hard ? ((size_t)T + 15) / 16 * 16 : (size_t)T * ((size_t)4 << n);
  return rows + (size_t)T * 8;
}

template <bool HARD>
__device__ __forceinline__ void latency_decode_block(const GenericArgs& a, int b, unsigned char* lds) {
  using MT = typename std::conditional<HARD, uint32_t, float>::type;
  const int lane = threadIdx.x;
  const int S = 1 << (a.K - 1), H = S / 2, NS = 1 << a.n, T = a.T;
  const int OB = (T + 7) >> 3;
  float* rows_f = reinterpret_cast<float*>(lds);
  uint8_t* rows_b = lds;
  const size_t rows_bytes = HARD ? ((size_t)T + 15) / 16 * 16 : (size_t)T * NS * 4;
  uint64_t* dec = reinterpret_cast<uint64_t*>(lds + rows_bytes);
  // stage the block (coalesced; from page-locked host memory on the streaming path)
  if constexpr (HARD) {
    const uint8_t* src = reinterpret_cast<const uint8_t*>(a.in) + (size_t)b * T;
    for (int k = lane; k < T; k += 64) rows_b[k] = src[k] & (uint8_t)(NS - 1);
  } else {
    const float* src = reinterpret_cast<const float*>(a.in) + (size_t)b * T * NS;
    for (int k = lane; k < T * NS; k += 64) rows_f[k] = src[k];
  }
  // this lane's state ns (lanes >= S mirror state ns mod S and are ignored), its predecessors and
  // the expected symbols of their transitions into ns
  const int ns = lane & (S - 1);
  const int i = ns >> (a.K - 2);
  const int s0 = (ns & (H - 1)) << 1;
  const uint32_t e0 = a.exp[2 * s0 + i], e1 = a.exp[2 * (s0 | 1) + i];
  const int addr0 = s0 << 2, addr1 = (s0 | 1) << 2;   // ds_bpermute byte addresses of lanes s0, s1
  MT M = ns == 0 ? (MT)0 : unreachable_metric<HARD>();
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    MT bm0, bm1;
    if constexpr (HARD) {
      const uint32_t sym = rows_b[t];
      bm0 = (MT)__builtin_popcount(e0 ^ sym);
      bm1 = (MT)__builtin_popcount(e1 ^ sym);
    } else {
      bm0 = rows_f[t * NS + e0];
      bm1 = rows_f[t * NS + e1];
    }
    MT m0, m1;
    if constexpr (HARD) {
      m0 = (MT)__builtin_amdgcn_ds_bpermute(addr0, (int)M);
      m1 = (MT)__builtin_amdgcn_ds_bpermute(addr1, (int)M);
      m0 = m0 + bm0;
      m1 = m1 + bm1;
      m0 = m0 > 0xFF00u ? 0xFF00u : m0;   // binary-symmetric-channel/viterbi-decoder.c:127-130
      m1 = m1 > 0xFF00u ? 0xFF00u : m1;
    } else {
      m0 = __int_as_float(__builtin_amdgcn_ds_bpermute(addr0, __float_as_int(M))) + bm0;
      m1 = __int_as_float(__builtin_amdgcn_ds_bpermute(addr1, __float_as_int(M))) + bm1;
    }
    const bool d = m1 < m0;
    M = d ? m1 : m0;
    const uint64_t w = __ballot(d && lane < S);
    if (lane == 0) dec[t] = w;
  }
  // lowest-index minimum (reference traceback :72-79): min over the wave, then the first lane
  // holding it (metrics are never NaN or -0, so == is exact)
  MT mn = lane < S ? M : unreachable_metric<HARD>();
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const MT o = __shfl_xor(mn, off, 64);
    mn = o < mn ? o : mn;
  }
  const uint64_t at_min = __ballot(lane < S && M == mn);
  const bool found = mn < unreachable_metric<HARD>();
  uint32_t st = found && at_min ? (uint32_t)__builtin_ctzll(at_min) : 0u;
  __syncthreads();   // dec[] written by lane 0 is visible to every lane
  if (lane == 0) {
    uint8_t* o = a.out + (size_t)b * OB;
    uint32_t acc = 0;
    for (int t = T - 1; t >= 0; --t) {
      const uint32_t bit = (uint32_t)(dec[t] >> st) & 1u;
      acc |= (st >> (a.K - 2)) << (7 - (t & 7));
      st = ((st << 1) & (uint32_t)(S - 1)) | bit;
      if ((t & 7) == 0) {
        o[t >> 3] = (uint8_t)acc;
        acc = 0;
      }
    }
    if constexpr (HARD) {
      if (a.path_metric) a.path_metric[b] = (int32_t)(found ? mn : unreachable_metric<HARD>());
    }
  }
}

template <bool HARD>
__global__ __launch_bounds__(64) void viterbi_latency(GenericArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  latency_decode_block<HARD>(a, blockIdx.x, lds);
}

// ---------------------------------------------------------------------------------------------
// Streaming service (the reference API's decoder_input: one block completes per call and the
// callback fires inside the call). A kernel launch plus a synchronise per block costs ~27 us; instead
// one workgroup stays resident and polls a mailbox in page-locked, fine-grained host memory: the host
// writes the block into page-locked memory and bumps `req`, the workgroup decodes it straight from
// host memory (latency_decode_block for K <= 7, else generic_decode_block), writes the output bytes
// back to host memory and publishes
// `done`. The kernel always ends: after `idle_ticks` of the 100 MHz real-time counter without a
// request, on `stop`, or after `max_polls` polls; it then sets `exited`, and the host relaunches it on
// the next request. Mailbox words are read and written with system-scope atomics.
struct ServiceMailbox {
  uint32_t req;       // host -> device: request sequence number
  uint32_t nblocks;   // host -> device: blocks of the request
  uint32_t done;      // device -> host: last request served
  uint32_t stop;      // host -> device: end now
  uint32_t exited;    // device -> host: the kernel has left its loop
  uint32_t pad[11];
};

template <int SPT, bool HARD, bool LAT>
__global__ __launch_bounds__(kGenericMaxThreads) void viterbi_service(GenericArgs a, ServiceMailbox* mb,
                                                                      uint32_t served, uint64_t idle_ticks,
                                                                      uint32_t max_polls) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  __shared__ uint32_t cmd[2];
  for (;;) {
    if (threadIdx.x == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t seq = served, stop = 0;
      for (uint32_t polls = 0; polls < max_polls; ++polls) {
        seq = __hip_atomic_load(&mb->req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        stop = __hip_atomic_load(&mb->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (seq != served || stop) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) break;
        __builtin_amdgcn_s_sleep(1);
      }
      cmd[0] = (seq != served && !stop) ? seq : served;
      cmd[1] = (seq != served && !stop) ? __hip_atomic_load(&mb->nblocks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
    }
    __syncthreads();
    const uint32_t seq = cmd[0], nb = cmd[1];
    if (seq == served) break;   // idle, stopped or out of polls
    for (uint32_t b = 0; b < nb; ++b) {
      if constexpr (LAT) latency_decode_block<HARD>(a, (int)b, lds);
      else generic_decode_block<SPT, HARD>(a, (int)b, lds);
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      __threadfence_system();
      __hip_atomic_store(&mb->done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    served = seq;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(&mb->exited, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace ccv
