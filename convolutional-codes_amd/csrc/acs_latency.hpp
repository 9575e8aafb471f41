// acs_latency.hpp -- one block, decoded by one wave as fast as a single block can go (K <= 7).
//
// The streaming reference API completes ONE block per decoder_input() call and fires the callback
// inside it (AWGN-channel/viterbi-decoder.c:132-139), so what matters there is the latency of a
// single block, not throughput. The register trellis (acs_reg.hpp) spends ~17 us on a lone block (one
// lane walks 46 steps of ~200 VALU at a lone wave's issue rate); the table kernel (acs_generic.hpp)
// 16.6 us (rocprof; two workgroup barriers and LDS round trips per step); one lane per state with the
// predecessors fetched by ds_bpermute 10.8 us. Here one lane per state runs the IN-PLACE trellis
// (below), so a step's cross-lane move is a DPP / permlane instruction for 5 of the 6 phases at K = 7,
// and the wave's decisions are one 64-bit mask per step, built from two compares (kept in LDS). The
// argmin is a wave reduction (lowest logical index among the minima), and the traceback walks the
// masks with the state uniform across the wave. Same arithmetic and tie rules as the reference
// (AWGN-channel/viterbi-decoder.c:71-141, binary-symmetric-channel/viterbi-decoder.c:75-150).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "acs_generic.hpp"

namespace ccv {

constexpr int kLatencyMaxK = 7;   // S <= 64: one state per lane

#ifdef CCV_LAT_STAMPS   // tools/lat_probe.hip: 100 MHz real-time stamps of the kernel's phases
__device__ unsigned long long ccv_lat_stamps[16];   // [0..7] real time, [8..15] shader clock
#define CCV_LAT_STAMP(i) \
  do { if (threadIdx.x == 0) { ccv_lat_stamps[i] = __builtin_amdgcn_s_memrealtime(); \
                               ccv_lat_stamps[8 + (i)] = __builtin_amdgcn_s_memtime(); } } while (0)
#else
#define CCV_LAT_STAMP(i) do {} while (0)
#endif

// LDS bytes: the block's rows (soft: T x 2^n floats; hard: T bytes) and the decision masks (T
// rounded up to 64 words).
__host__ __device__ inline size_t latency_rows_bytes(int n, int T, bool hard) {
  return hard ? ((size_t)T + 15) / 16 * 16 : ((size_t)T * ((size_t)4 << n) + 15) / 16 * 16;
}
inline size_t latency_lds_bytes(int n, int T, bool hard) {
  return latency_rows_bytes(n, T, hard) + ((size_t)T + 63) / 64 * 64 * 8;
}

// The value of lane (lane ^ (1 << P)) for this lane: quad_perm moves for P = 0, 1, half-row mirror +
// quad reversal for 2, row rotation by 8 for 3, an LDS-crossbar swizzle for 4, the half-wave swap
// for 5 -- all but the swizzle plain VALU.
template <int P>
__device__ __forceinline__ uint32_t xor_lane(uint32_t x) {
  if constexpr (P == 0) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);   // [1,0,3,2]
  else if constexpr (P == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);   // [2,3,0,1]
  else if constexpr (P == 2) {
    const int m = __builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, true);   // row_half_mirror: i -> 7-i
    return (uint32_t)__builtin_amdgcn_mov_dpp(m, 0x1B, 0xF, 0xF, true);     // quad_perm [3,2,1,0]
  } else if constexpr (P == 3) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, true);   // row_ror:8
  } else if constexpr (P == 4) {
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x401F);            // xor 16 within 32
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap((int)x, (int)x, false, false);
    return (uint32_t)((threadIdx.x & 32) ? r[0] : r[1]);
  }
}

// In-place trellis (as the multilane kernels, acs_multi.hpp): lane l holds physical state l, which at
// phase p = t mod (K-1) is logical state rotr(l, p). Step t pairs the lanes that differ in bit p: the
// one with the bit clear holds the even predecessor s0, its partner the odd one s1, and each computes
// the new state whose input bit is its own bit p. So a step is one cross-lane move (no LDS round trip
// for p < 4), two adds, the min, and the decisions straight from two compares (the survivor is the
// partner's candidate when partner < own for a lane holding s0, when own < partner for a lane holding
// s1: strict < with the even predecessor winning ties, as the reference).
// Per-lane constants of a plan (computed once; the service kernel keeps them across blocks): per
// phase the expected symbols of this lane's own and partner candidates and the lanes holding s1.
struct LatencyLane {
  uint32_t eown[6], epar[6];
  uint64_t odd[6];
  uint64_t valid;
};

__device__ __forceinline__ uint32_t latency_rotr(uint32_t x, int p, int n) {
  return p == 0 ? x : (((x >> p) | (x << (n - p))) & ((1u << n) - 1u));
}

template <int NK>
__device__ __forceinline__ LatencyLane latency_setup(const GenericArgs& a) {
  LatencyLane L{};
  constexpr int n = NK, S = 1 << n;
  const uint32_t l = threadIdx.x & (uint32_t)(S - 1);   // lanes >= S mirror lane l (ignored)
#pragma unroll
  for (int p = 0; p < 6; ++p) {
    if (p < n) {
      const uint32_t bit = (l >> p) & 1u;                    // input bit of this lane's new state
      L.eown[p] = a.exp[2 * latency_rotr(l, p, n) + bit];    // logical predecessors
      L.epar[p] = a.exp[2 * latency_rotr(l ^ (1u << p), p, n) + bit];
      L.odd[p] = __ballot(bit);                              // lanes holding s1 at phase p
    }
  }
  if constexpr (S >= 64) L.valid = ~0ull;
  else L.valid = (1ull << S) - 1ull;
  return L;
}

template <int P>
__device__ __forceinline__ float xor_lane_f(float x) { return __uint_as_float(xor_lane<P>(__float_as_uint(x))); }
template <int P>
__device__ __forceinline__ uint32_t xor_lane_u(uint32_t x) { return xor_lane<P>(x); }

// In-place trellis (as the multilane kernels, acs_multi.hpp): lane l holds physical state l, which at
// phase p = t mod (K-1) is logical state rotr(l, p). Step t pairs the lanes that differ in bit p: the
// one with the bit clear holds the even predecessor s0, its partner the odd one s1, and each computes
// the new state whose input bit is its own bit p. So a step is one cross-lane move (no LDS round trip
// for p < 4), two adds, the min, and the decisions straight from two compares (the survivor is the
// partner's candidate when partner < own for a lane holding s0, when own < partner for a lane holding
// s1: strict < with the even predecessor winning ties, as the reference). The branch metrics of a
// group of K-1 steps are read from LDS before its ACS chain; the decision masks (scalar registers)
// are gathered into lane t mod 64 of a register pair and written to LDS 64 steps at a time. The
// traceback runs on scalar registers, reading each mask back with v_readlane, and the output bits go
// out as one byte per lane.
// NK = K - 1 (1..6) is a template argument: the phase loop unrolls into straight-line code.
template <bool HARD, int NK>
__device__ __forceinline__ void latency_decode_block(const GenericArgs& a, int b, unsigned char* lds,
                                                     const LatencyLane& L) {
  using MT = typename std::conditional<HARD, uint32_t, float>::type;
  const int lane = threadIdx.x;
  constexpr int n = NK, S = 1 << n;
  const int NS = 1 << a.n, T = a.T;
  const int OB = (T + 7) >> 3;
  float* rows_f = reinterpret_cast<float*>(lds);
  uint8_t* rows_b = lds;
  uint64_t* dec = reinterpret_cast<uint64_t*>(lds + latency_rows_bytes(a.n, T, HARD));
  CCV_LAT_STAMP(0);
  // stage the block: up to 4 loads per lane in flight at once (one PCIe round trip for a K <= 7 block
  // from page-locked host memory on the streaming path)
  if constexpr (HARD) {
    const uint8_t* src = reinterpret_cast<const uint8_t*>(a.in) + (size_t)b * T;
    for (int k0 = 0; k0 < T; k0 += 256) {   // clamped loads (all in flight), guarded stores
      const int k1 = k0 + lane, k2 = k1 + 64, k3 = k1 + 128, k4 = k1 + 192, last = T - 1;
      const uint8_t v1 = src[k1 < last ? k1 : last], v2 = src[k2 < last ? k2 : last];
      const uint8_t v3 = src[k3 < last ? k3 : last], v4 = src[k4 < last ? k4 : last];
      const uint8_t mask = (uint8_t)(NS - 1);
      if (k1 < T) rows_b[k1] = v1 & mask;
      if (k2 < T) rows_b[k2] = v2 & mask;
      if (k3 < T) rows_b[k3] = v3 & mask;
      if (k4 < T) rows_b[k4] = v4 & mask;
    }
  } else {
    const float* src = reinterpret_cast<const float*>(a.in) + (size_t)b * T * NS;
    const int N = T * NS;
    if ((N & 3) == 0 && ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
      const float4* s4 = reinterpret_cast<const float4*>(src);
      float4* r4 = reinterpret_cast<float4*>(rows_f);
      const int N4 = N >> 2;
      for (int k0 = 0; k0 < N4; k0 += 256) {
        const int k1 = k0 + lane, k2 = k1 + 64, k3 = k1 + 128, k4 = k1 + 192, last = N4 - 1;
        const float4 v1 = s4[k1 < last ? k1 : last], v2 = s4[k2 < last ? k2 : last];
        const float4 v3 = s4[k3 < last ? k3 : last], v4 = s4[k4 < last ? k4 : last];
        if (k1 < N4) r4[k1] = v1;
        if (k2 < N4) r4[k2] = v2;
        if (k3 < N4) r4[k3] = v3;
        if (k4 < N4) r4[k4] = v4;
      }
    } else {
      for (int k = lane; k < N; k += 64) rows_f[k] = src[k];
    }
  }
  const uint32_t l = (uint32_t)lane & (uint32_t)(S - 1);
  MT M = l == 0 ? (MT)0 : unreachable_metric<HARD>();
  uint32_t wlo = 0, whi = 0;   // lane j: the decision mask of step 64c + j
  __syncthreads();
  CCV_LAT_STAMP(1);
  auto bm = [&](int t, uint32_t e) __attribute__((always_inline)) -> MT {
    if constexpr (HARD) return (MT)__builtin_popcount(e ^ (uint32_t)rows_b[t]);
    else return rows_f[t * NS + e];
  };
  auto partner = [&](int p) __attribute__((always_inline)) -> MT {
    if constexpr (HARD) {
      switch (p) {
        case 0: return xor_lane_u<0>(M);
        case 1: return xor_lane_u<1>(M);
        case 2: return xor_lane_u<2>(M);
        case 3: return xor_lane_u<3>(M);
        case 4: return xor_lane_u<4>(M);
        default: return xor_lane_u<5>(M);
      }
    } else {
      switch (p) {
        case 0: return xor_lane_f<0>(M);
        case 1: return xor_lane_f<1>(M);
        case 2: return xor_lane_f<2>(M);
        case 3: return xor_lane_f<3>(M);
        case 4: return xor_lane_f<4>(M);
        default: return xor_lane_f<5>(M);
      }
    }
  };
  // argmin over the lanes: the minimum metric and the lowest LOGICAL index holding it (reference
  // traceback :72-79); at the end the lanes are at phase T mod (K-1), so lane l holds logical state
  // rotr(l, T mod (K-1))
  const int pe = T % n;
  auto argmin = [&](MT& mn) __attribute__((always_inline)) -> uint32_t {
    // butterflies over the lane-index bits (DPP / swizzle / permlane moves); lanes >= S mirror
    // lanes < S, so the whole wave reduces to the same answer
    uint32_t m = HARD ? (uint32_t)M : __float_as_uint(M);
    auto red = [&](uint32_t v, auto op) __attribute__((always_inline)) {
      v = op(v, xor_lane_u<0>(v));
      v = op(v, xor_lane_u<1>(v));
      v = op(v, xor_lane_u<2>(v));
      v = op(v, xor_lane_u<3>(v));
      v = op(v, xor_lane_u<4>(v));
      return op(v, xor_lane_u<5>(v));
    };
    if constexpr (HARD) {
      m = red(m, [](uint32_t x, uint32_t y) { return x < y ? x : y; });
      mn = (MT)m;
    } else {
      m = red(m, [](uint32_t x, uint32_t y) {
        return __float_as_uint(__builtin_fminf(__uint_as_float(x), __uint_as_float(y)));
      });
      mn = __uint_as_float(m);
    }
    uint32_t cand = M == mn ? latency_rotr(l, pe, n) : 0xFFFFFFFFu;
    cand = red(cand, [](uint32_t x, uint32_t y) { return x < y ? x : y; });
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(mn < unreachable_metric<HARD>() ? cand : 0u));
  };
  if (T <= 64) {
    // REGISTER EXCHANGE (blocks of at most 64 steps): each lane carries its survivor's decoded bits
    // in a register pair, taking its partner's pair when the partner's candidate survives and
    // appending the new state's input bit (bit p of the lane: the top bit of logical state
    // rotr(l, p+1)); the best state's pair IS the decoded block, so there is no traceback.
    uint32_t plo = 0, phi = 0;
    auto xstep = [&](int p, MT bo, MT bp) __attribute__((always_inline)) {
      const MT pm = partner(p);
      uint32_t qlo, qhi;
      switch (p) {
        case 0: qlo = xor_lane_u<0>(plo); qhi = xor_lane_u<0>(phi); break;
        case 1: qlo = xor_lane_u<1>(plo); qhi = xor_lane_u<1>(phi); break;
        case 2: qlo = xor_lane_u<2>(plo); qhi = xor_lane_u<2>(phi); break;
        case 3: qlo = xor_lane_u<3>(plo); qhi = xor_lane_u<3>(phi); break;
        case 4: qlo = xor_lane_u<4>(plo); qhi = xor_lane_u<4>(phi); break;
        default: qlo = xor_lane_u<5>(plo); qhi = xor_lane_u<5>(phi); break;
      }
      MT ao = M + bo, ap = pm + bp;
      if constexpr (HARD) {
        ao = ao > 0xFF00u ? 0xFF00u : ao;   // binary-symmetric-channel/viterbi-decoder.c:127-130
        ap = ap > 0xFF00u ? 0xFF00u : ap;
      }
      // the metric chain is adds and a min (equal candidates are equal values); the partner's path
      // survives when its candidate is strictly better for a lane holding s0, not worse for one
      // holding s1 (two compares combined on the scalar unit, used as the lane mask of the selects)
      if constexpr (HARD) M = ao < ap ? ao : ap;
      else M = __builtin_fminf(ao, ap);
      const uint64_t tk = (__ballot(ap < ao) & ~L.odd[p]) | (__ballot(!(ao < ap)) & L.odd[p]);
      const bool take = __builtin_amdgcn_inverse_ballot_w64(tk);
      const uint32_t nlo = take ? qlo : plo, nhi = take ? qhi : phi;
      phi = (nhi << 1) | (nlo >> 31);
      plo = (nlo << 1) | ((l >> p) & 1u);
    };
    int t0 = 0;
    for (; t0 + n <= T; t0 += n) {
      MT bo[6], bp[6];
#pragma unroll
      for (int p = 0; p < n; ++p) {
        bo[p] = bm(t0 + p, L.eown[p]);
        bp[p] = bm(t0 + p, L.epar[p]);
      }
#pragma unroll
      for (int p = 0; p < n; ++p) xstep(p, bo[p], bp[p]);
    }
#pragma unroll
    for (int p = 0; p < n - 1; ++p)
      if (t0 + p < T) xstep(p, bm(t0 + p, L.eown[p]), bm(t0 + p, L.epar[p]));
    CCV_LAT_STAMP(2);
    MT mn;
    const uint32_t st = argmin(mn);
    CCV_LAT_STAMP(3);
    const uint32_t src = (((st << pe) | (st >> (n - pe))) & (uint32_t)(S - 1));   // its physical lane
    const uint64_t path = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)phi, (int)src) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)plo, (int)src);
    // bit T-1-t: step t. Output byte k holds steps 8k..8k+7, the earliest in the most significant bit.
    const uint64_t top = path << (64 - T);
    uint8_t* o = a.out + (size_t)b * OB;
    if (lane < OB) o[lane] = (uint8_t)(top >> (56 - 8 * lane));
    CCV_LAT_STAMP(4);
    if constexpr (HARD) {
      if (lane == 0 && a.path_metric) a.path_metric[b] = (int32_t)mn;
    }
    return;
  }
  auto step = [&](int t, int p, MT bo, MT bp) __attribute__((always_inline)) {
    MT ao = M + bo, ap = partner(p) + bp;
    if constexpr (HARD) {
      ao = ao > 0xFF00u ? 0xFF00u : ao;   // binary-symmetric-channel/viterbi-decoder.c:127-130
      ap = ap > 0xFF00u ? 0xFF00u : ap;
    }
    const uint64_t lt = __ballot(ap < ao), gt = __ballot(ao < ap);
    const uint64_t d = ((lt & ~L.odd[p]) | (gt & L.odd[p])) & L.valid;
    M = ao < ap ? ao : ap;   // min: equal candidates are equal values
    const int j = t & 63;
    wlo = lane == j ? (uint32_t)d : wlo;
    whi = lane == j ? (uint32_t)(d >> 32) : whi;
    if (j == 63) dec[(t & ~63) + lane] = ((uint64_t)whi << 32) | wlo;
  };
  int t0 = 0;
  for (; t0 + n <= T; t0 += n) {
    MT bo[6], bp[6];
#pragma unroll
    for (int p = 0; p < 6; ++p)
      if (p < n) {
        bo[p] = bm(t0 + p, L.eown[p]);
        bp[p] = bm(t0 + p, L.epar[p]);
      }
#pragma unroll
    for (int p = 0; p < 6; ++p)
      if (p < n) step(t0 + p, p, bo[p], bp[p]);
  }
#pragma unroll
  for (int p = 0; p < n - 1; ++p)   // the last T mod (K-1) steps
    if (t0 + p < T) step(t0 + p, p, bm(t0 + p, L.eown[p]), bm(t0 + p, L.epar[p]));
  if (T & 63) dec[(T & ~63) + lane] = ((uint64_t)whi << 32) | wlo;
  CCV_LAT_STAMP(2);
  MT mn;
  uint32_t st = argmin(mn);   // logical state
  __syncthreads();
  CCV_LAT_STAMP(3);
  // traceback, 64 steps per chunk, wave-uniform: the survivors of step t sit at the phase-(t+1)
  // positions, physical = rotl(st, (t+1) mod (K-1))
  uint8_t* o = a.out + (size_t)b * OB;
  int q = pe;   // (t + 1) mod (K-1) for t = T-1
  for (int c = (T - 1) >> 6; c >= 0; --c) {
    const uint64_t w = dec[c * 64 + lane];
    const uint32_t w0 = (uint32_t)w, w1 = (uint32_t)(w >> 32);
    uint64_t ob = 0;   // bit j: the decoded bit of step 64c + j
    const int tl = (T - 1 - c * 64) < 63 ? (T - 1 - c * 64) : 63;
    for (int j = tl; j >= 0; --j) {
      const uint32_t phys = q == 0 ? st : (((st << q) | (st >> (n - q))) & (uint32_t)(S - 1));
      const uint32_t word = phys < 32 ? (uint32_t)__builtin_amdgcn_readlane((int)w0, j)
                                      : (uint32_t)__builtin_amdgcn_readlane((int)w1, j);
      const uint32_t bit = (word >> (phys & 31)) & 1u;
      ob |= (uint64_t)(st >> (n - 1)) << j;
      st = ((st << 1) & (uint32_t)(S - 1)) | bit;
      q = q == 0 ? n - 1 : q - 1;
    }
    // output byte k of the chunk holds steps 8k..8k+7, the earliest in the most significant bit
    if (lane < 8 && c * 8 + lane < OB)
      o[c * 8 + lane] = (uint8_t)(__builtin_bitreverse32((uint32_t)(ob >> (8 * lane))) >> 24);
  }
  CCV_LAT_STAMP(4);
  if constexpr (HARD) {
    if (lane == 0 && a.path_metric) a.path_metric[b] = (int32_t)mn;
  }
}

template <bool HARD, int NK>
__global__ __launch_bounds__(64) void viterbi_latency(GenericArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const LatencyLane L = latency_setup<NK>(a);
  latency_decode_block<HARD, NK>(a, blockIdx.x, lds, L);
}

// ---------------------------------------------------------------------------------------------
// Streaming service (the reference API's decoder_input: one block completes per call and the
// callback fires inside the call). A kernel launch plus a synchronise per block costs ~16 us (the
// launch and completion round trips, ~11 us, around a ~5 us decode); instead one workgroup stays
// resident and polls a mailbox in page-locked, fine-grained host memory: the host writes the block
// into page-locked memory and bumps `req`, the workgroup decodes it straight from host memory
// (latency_decode_block for K <= 7, else generic_decode_block), writes the output bytes back to host
// memory and publishes `done` (~11 us per block end to end). The kernel always ends: after `idle_ticks` of the 100 MHz real-time counter without a
// request, on `stop`, or after `max_polls` polls; it then sets `exited`, and the host relaunches it on
// the next request. Mailbox words are read and written with system-scope atomics.
struct ServiceMailbox {
  uint64_t req;       // host -> device: request sequence number (low word) | blocks (high word)
  uint32_t done;      // device -> host: last request served
  uint32_t stop;      // host -> device: end now
  uint32_t exited;    // device -> host: the kernel has left its loop
  uint32_t pad[11];
};

// LATN = 0: the table kernel's block decode; LATN = K - 1: the one-wave latency decode.
template <int SPT, bool HARD, int LATN>
__global__ __launch_bounds__(kGenericMaxThreads) void viterbi_service(GenericArgs a, ServiceMailbox* mb,
                                                                      uint32_t served, uint64_t idle_ticks,
                                                                      uint32_t max_polls) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  __shared__ uint32_t cmd[2];
  LatencyLane L{};
  if constexpr (LATN > 0) L = latency_setup<LATN>(a);
  for (;;) {
    if (threadIdx.x == 0) {
      // one PCIe read per poll (sequence number and block count in one word); `stop` every 64th
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint64_t r = served;
      uint32_t stop = 0;
      for (uint32_t polls = 0; polls < max_polls; ++polls) {
        r = __hip_atomic_load(&mb->req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((uint32_t)r != served) break;
        if ((polls & 63u) == 63u) {
          stop = __hip_atomic_load(&mb->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if (stop || __builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      const bool go = (uint32_t)r != served && !stop;
      cmd[0] = go ? (uint32_t)r : served;
      cmd[1] = go ? (uint32_t)(r >> 32) : 0u;
    }
    __syncthreads();
    const uint32_t seq = cmd[0], nb = cmd[1];
    if (seq == served) break;   // idle, stopped or out of polls
    for (uint32_t b = 0; b < nb; ++b) {
      if constexpr (LATN > 0) latency_decode_block<HARD, LATN>(a, (int)b, lds, L);
      else generic_decode_block<SPT, HARD>(a, (int)b, lds);
      __syncthreads();
    }
    // the system-scope release orders the output stores (to page-locked host memory) before `done`
    if (threadIdx.x == 0) __hip_atomic_store(&mb->done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    served = seq;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(&mb->exited, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace ccv
