// acs_multi2.hpp -- persistent K = 9 r = 1/2 soft Viterbi with TWO lanes per block (128 metrics per
// lane), gfx950: the production path of the textbook (561,753) code, whose 256 metrics are all
// distinct (no value-numbering twins, so the one-lane-per-block kernel of acs_wide.hpp cannot hold
// them in 256 VGPRs).
//
// Why two lanes and not four (acs_multi.hpp): the in-place trellis pairs on one physical state bit per
// step, and a lane bit costs its phase a DPP read of both predecessors (two half-rate v_add_f32_dpp per
// state) plus per-lane branch-metric selects. With four lanes two of eight phases are cross-lane and
// the stream's half-rate share (v_min, v_alignbit, DPP adds, v_cndmask_e64) reaches ~50 %, where
// gfx950 stops hiding them behind full-rate ops: the four-lane kernel issued VALU at
// 0.50 of peak with its waves issue-stalled 45 % of their lifetime, fully unrolled or as a loop
// (profiles/pmc_workloads.json, k9:true:frames32:block). Two lanes: one cross phase in eight and a
// single lane bit in every select.
//
// Layout: physical state = register bits with the lane bit inserted at bit LB; the ACS is in place, so
// at phase p = t mod 8 the logical state held at phys is rotr_8(phys, p) (acs_multi.hpp). Decisions:
// 128 bits per lane and step -- in-lane phases put the survivor of register R (bit k clear, input 0)
// at bit compress_k(R) and of R | 1 << k (input 1) at 64 + compress_k(R); the cross phase puts
// register R at bit R -- one buffer_store_dwordx4 per step into a per-wave scratch slot ([main
// step][lane][16 B], 40 KiB per wave, rewritten by every group the wave decodes). The main periods
// run as a loop; the traceback drains the stores and reads them back with agent-scope loads, a period
// at a time (acs_multi.hpp viterbi_multi_slot).
//
// Arithmetic as AWGN-channel/viterbi-decoder.c:108-141 (fp32 adds, strict compare = sign of m1 - m0,
// even predecessor on ties, +inf reset metrics) and traceback :71-90 (lowest-index argmin).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "acs_multi.hpp"

namespace ccv {

template <CodeSpec C, int LB = 7>
struct Multi2 {
  static constexpr int n = C.K - 1;        // state bits (8)
  static constexpr int S = 1 << n;         // 256
  static constexpr int NR = S / 2;         // registers per lane (128)
  static_assert(LB >= 0 && LB < n, "lane bit");
  static constexpr bool is_lane(int P) { return P == LB; }
  static constexpr int reg_bit(int P) { return P < LB ? P : P - 1; }
  static constexpr uint32_t phys(int q, int r) {
    const uint32_t low = (uint32_t)r & ((1u << LB) - 1u);
    const uint32_t high = ((uint32_t)r >> LB) << (LB + 1);
    return high | ((uint32_t)q << LB) | low;
  }
  static constexpr uint32_t rotr(uint32_t x, int p) {
    p %= n;
    return p == 0 ? x : (((x >> p) | (x << (n - p))) & (S - 1));
  }
  static constexpr uint32_t logical(int q, int r, int p) { return rotr(phys(q, r), p); }
  // r without bit k (6 bits)
  static constexpr uint32_t compress(uint32_t r, int k) {
    return ((r >> (k + 1)) << k) | (r & ((1u << k) - 1u));
  }
};

// compress / phys at run time (argmin, traceback)
__device__ __forceinline__ uint32_t compress_bit(uint32_t r, int k) {
  return ((r >> (k + 1)) << k) | (r & ((1u << k) - 1u));
}
template <int LB>
__device__ __forceinline__ uint32_t multi2_phys(uint32_t q, uint32_t r) {
  return ((r >> LB) << (LB + 1)) | (q << LB) | (r & ((1u << LB) - 1u));
}

// One butterfly (in-lane phase, register R with bit k clear) or one new state (cross phase), in place;
// decision bits shifted into D[] (see the header).
template <CodeSpec C, int P, int R, class X>
__device__ __forceinline__ void multi2_acs(float (&M)[X::NR], const float (&BM)[4], bool qb, uint32_t (&D)[4]) {
  if constexpr (!X::is_lane(P)) {
    constexpr int k = X::reg_bit(P);
    if constexpr ((R & (1 << k)) == 0) {
      constexpr int R1 = R | (1 << k);
      constexpr auto e = [](int q, int odd, int in) {
        return expected_symbol(C, X::logical(q, R, P) | (uint32_t)odd, in);
      };
      const float a0 = M[R] + select_bm<2, e(0, 0, 0), e(1, 0, 0), 0, 0>(BM, qb, false);
      const float a1 = M[R1] + select_bm<2, e(0, 1, 0), e(1, 1, 0), 0, 0>(BM, qb, false);
      const float b0 = M[R] + select_bm<2, e(0, 0, 1), e(1, 0, 1), 0, 0>(BM, qb, false);
      const float b1 = M[R1] + select_bm<2, e(0, 1, 1), e(1, 1, 1), 0, 0>(BM, qb, false);
      constexpr uint32_t c = X::compress((uint32_t)R, k);
      M[R] = vmin(a0, a1);
      D[c >> 5] = shift_in(D[c >> 5], a0, a1);
      M[R1] = vmin(b0, b1);
      D[2 + (c >> 5)] = shift_in(D[2 + (c >> 5)], b0, b1);
    }
  } else {
    static_assert(!X::is_lane(P), "the cross phase runs in multi2_cross_swz");
  }
}

// Growth step (t = P < K-1, from the reset metrics): the odd predecessor is still unreachable (+inf,
// never wins the strict compare), so a new state is its even predecessor plus the branch metric and
// its decision 0 -- adds only (acs_multi.hpp multi_growth).
template <CodeSpec C, int P, int R, class X>
__device__ __forceinline__ void multi2_growth(float (&M)[X::NR], const float (&BM)[4], bool qb) {
  if constexpr (!X::is_lane(P)) {
    constexpr int k = X::reg_bit(P);
    if constexpr ((R & (1 << k)) == 0) {
      constexpr int R1 = R | (1 << k);
      constexpr auto e = [](int q, int in) { return expected_symbol(C, X::logical(q, R, P), in); };
      const float even = M[R];
      M[R] = even + select_bm<2, e(0, 0), e(1, 0), 0, 0>(BM, qb, false);
      M[R1] = even + select_bm<2, e(0, 1), e(1, 1), 0, 0>(BM, qb, false);
    }
  } else {
    static_assert(!X::is_lane(P), "the growth cross phase runs in multi2_growth_cross_swz");
  }
}

// The cross phase through ds_swizzle: any DPP / permlane /
// readlane VALU instruction drops the wave's whole VALU stream to about half rate for ~800
// instructions on gfx950, and the cross phase issues 256 of them per period, so the
// even / odd predecessors come from the pair's lanes through the LDS crossbar instead -- registers in
// chunks of G, the swizzles of chunk c + 1 issued before the ACS of chunk c.
#ifndef CCV_MULTI2_XG
#define CCV_MULTI2_XG 8
#endif
template <CodeSpec C, int P, class X, int G = CCV_MULTI2_XG>
__device__ __forceinline__ void multi2_cross_swz(float (&M)[X::NR], const float (&BM)[4], bool qb,
                                                 uint32_t (&D)[4]) {
  static_assert(X::is_lane(P), "cross-lane phase");
  constexpr int NR = X::NR;
  constexpr int NC = NR / G;
  static_assert(NR % G == 0, "whole chunks");
  float E[2][G], O[2][G];
  auto issue = [&]<int c>() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int R = NR - 1 - (c * G + i);
      E[c & 1][i] = swz_quad<0, 0, 2, 2>(M[R]);
      O[c & 1][i] = swz_quad<1, 1, 3, 3>(M[R]);
    }
  };
  auto compute = [&]<int c>() __attribute__((always_inline)) {
    [&]<int... is>(std::integer_sequence<int, is...>) __attribute__((always_inline)) {
      ([&]() __attribute__((always_inline)) {
        constexpr int R = NR - 1 - (c * G + is);
        constexpr auto e = [](int q, int odd) { return expected_symbol(C, X::logical(0, R, P) | (uint32_t)odd, q); };
        const float a0 = E[c & 1][is] + select_bm<2, e(0, 0), e(1, 0), 0, 0>(BM, qb, false);
        const float a1 = O[c & 1][is] + select_bm<2, e(0, 1), e(1, 1), 0, 0>(BM, qb, false);
        M[R] = vmin(a0, a1);
        D[R >> 5] = shift_in(D[R >> 5], a0, a1);
      }(), ...);
    }(std::make_integer_sequence<int, G>{});
  };
  issue.template operator()<0>();
  [&]<int... cs>(std::integer_sequence<int, cs...>) __attribute__((always_inline)) {
    ([&]() __attribute__((always_inline)) {
      if constexpr (cs + 1 < NC) issue.template operator()<cs + 1>();
      __builtin_amdgcn_sched_barrier(0);
      compute.template operator()<cs>();
      __builtin_amdgcn_sched_barrier(0);
    }(), ...);
  }(std::make_integer_sequence<int, NC>{});
}

// Growth cross phase through ds_swizzle: every new state is its even predecessor (the pair's
// lane 0, same register) plus the branch metric, in chunks of G registers.
template <CodeSpec C, int P, class X, int G = CCV_MULTI2_XG>
__device__ __forceinline__ void multi2_growth_cross_swz(float (&M)[X::NR], const float (&BM)[4], bool qb) {
  static_assert(X::is_lane(P), "cross-lane phase");
  constexpr int NR = X::NR;
  auto chunk = [&]<int c>() __attribute__((always_inline)) {
    float E[G];
#pragma unroll
    for (int i = 0; i < G; ++i) E[i] = swz_quad<0, 0, 2, 2>(M[c * G + i]);
    [&]<int... is>(std::integer_sequence<int, is...>) __attribute__((always_inline)) {
      ([&]() __attribute__((always_inline)) {
        constexpr int R = c * G + is;
        constexpr auto e = [](int q) { return expected_symbol(C, X::logical(0, R, P), q); };
        M[R] = E[is] + select_bm<2, e(0), e(1), 0, 0>(BM, qb, false);
      }(), ...);
    }(std::make_integer_sequence<int, G>{});
  };
  [&]<int... cs>(std::integer_sequence<int, cs...>) __attribute__((always_inline)) {
    (chunk.template operator()<cs>(), ...);
  }(std::make_integer_sequence<int, NR / G>{});
}

// the pair's other lane (quad_perm [1,0,3,2]) through ds_swizzle: the argmin and the traceback keep
// no cross-lane VALU either (with DPP there the kernel ran 34.8 instead of 37.6 Gbit/s)
__device__ __forceinline__ uint32_t pair_swap_u32(uint32_t x) { return swz_quad_u32<1, 0, 3, 2>(x); }
__device__ __forceinline__ float pair_swap(float x) { return swz_quad<1, 0, 3, 2>(x); }

// Registers per scheduling group: a scheduling barrier after every kMulti2Group registers keeps the
// compiler from hoisting the adds of many butterflies ahead of their mins (with 128 independent
// butterflies per step it otherwise keeps old and new metrics alive together: 256 VGPRs + spills).
#ifndef CCV_MULTI2_GROUP
#define CCV_MULTI2_GROUP 16
#endif
constexpr int kMulti2Group = CCV_MULTI2_GROUP;

template <CodeSpec C, int P, class X, size_t... I>
__device__ __forceinline__ void multi2_step_impl(float (&M)[X::NR], const float (&BM)[4], bool qb,
                                                 uint32_t (&D)[4], std::index_sequence<I...>) {
  // descending registers
  ((multi2_acs<C, P, X::NR - 1 - (int)I, X>(M, BM, qb, D),
    (kMulti2Group && (I + 1) % kMulti2Group == 0 ? __builtin_amdgcn_sched_barrier(0) : (void)0)),
   ...);
}
template <CodeSpec C, int P, class X, size_t... I>
__device__ __forceinline__ void multi2_growth_impl(float (&M)[X::NR], const float (&BM)[4], bool qb,
                                                   std::index_sequence<I...>) {
  (multi2_growth<C, P, X::NR - 1 - (int)I, X>(M, BM, qb), ...);
}

template <CodeSpec C, int BLEN>
constexpr size_t multi2_slot_bytes() {
  return (size_t)BLEN * kRegThreads * 16;   // main steps (T - (K-1) = BLEN) x 64 lanes x 16 B
}

// Ablation (timing only, output wrong): every decision store and traceback load goes to the slot's
// first step row, so the slot traffic stays in L1 / L2 while the instruction stream is unchanged --
// the ceiling of any slot-traffic reduction (round 5).
#ifndef CCV_MULTI2_SLOT_ABLATE
#define CCV_MULTI2_SLOT_ABLATE 0
#endif
constexpr int kMulti2StepOff(int step, int stepb) { return CCV_MULTI2_SLOT_ABLATE ? 0 : step * stepb; }

#ifndef CCV_MULTI2_WAVES
#define CCV_MULTI2_WAVES 2
#endif
template <CodeSpec C, int BLEN, int LB = 7, int OPT = 0>
__global__ __launch_bounds__(kRegThreads) __attribute__((amdgpu_waves_per_eu(CCV_MULTI2_WAVES)))
void viterbi_multi2_slot(RegArgs a, int ngroups) {
  using X = Multi2<C, LB>;
  static_assert(C.K == 9 && C.n == 2, "K = 9, r = 1/2: the period (8 steps) is the 8-step chunk");
  constexpr int n = X::n;                     // 8 phases per period
  constexpr int NR = X::NR;
  constexpr int T = BLEN + C.K - 1;
  static_assert(T % n == 0 && T / n >= 2, "whole periods");
  constexpr int NPER = T / n;                 // periods = chunks
  constexpr int NMAIN = NPER - 1;
  static_assert(NMAIN == 5, "K = 9 at blen 40: five main periods");
  constexpr int BPG = kRegThreads / 2;        // blocks per group (32)
  constexpr int ROWB = n * 16;                // one chunk of one block: 128 bytes
  constexpr int BUF = BPG * ROWB;             // 4 KiB
  constexpr int UNITS = BUF / 16;             // 256 DMA units per chunk: 4 instructions
  constexpr int IB = (BLEN + 7) >> 3, OB = (T + 7) >> 3;
  constexpr uint32_t block_bytes = (uint32_t)T * 16;
  constexpr int STEPB = kRegThreads * 16;     // slot bytes per main step
  static_assert(multi2_slot_bytes<C, BLEN>() == (size_t)NMAIN * n * STEPB, "slot layout");
  static_assert(NPER % 2 == 0, "buffer = chunk parity across groups");
  const int lane = threadIdx.x;
  const int q = lane & 1;
  const bool qb = q != 0;
  const int nb = a.nblocks;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * BUF];
  const unsigned char* in = reinterpret_cast<const unsigned char*>(a.in);
  // DMA k of a chunk: unit k*64 + lane = block r (of 32), LDS slot j of its row, holding step
  // j ^ (r & 7) of the chunk (XOR swizzle: the 32 rows sit 128 B apart, so without it every block's
  // step s would share one bank group)
  auto issue_chunk = [&](int g, int c, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < UNITS / kRegThreads; ++k) {
      const int unit = k * kRegThreads + lane;
      const int r = unit / n, j = unit % n;
      const int gb = g * BPG + r < nb ? g * BPG + r : nb - 1;
      __builtin_amdgcn_global_load_lds(in + (size_t)gb * block_bytes + (uint32_t)(c * n + (j ^ (r & 7))) * 16,
                                       (lds_ptr_t)(lds + buf * BUF + k * kRegThreads * 16), 16, 0, 0);
    }
  };
  const int rblk = lane / 2;
  const uint32_t row = (uint32_t)(uintptr_t)(lds_ptr_t)lds + (uint32_t)(rblk * ROWB);
  const uint32_t swz = (uint32_t)(rblk & 7) * 16;
  const uint8_t* info_src = a.info != nullptr ? a.info : reinterpret_cast<const uint8_t*>(a.in);
  const int info_stride = a.info != nullptr ? IB : 0;
  const __amdgpu_buffer_rsrc_t slot = __builtin_amdgcn_make_buffer_rsrc(
      static_cast<unsigned char*>(a.dec) + (size_t)blockIdx.x * NMAIN * n * STEPB, 0, NMAIN * n * STEPB,
      0x00020000);
  const int col = lane * 16;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  constexpr int kSc1 = 16;   // cache policy: agent scope (sc1), the load misses the CU's L1

  uint32_t errors = 0;
  GroupWalk<OPT> walk(a, ngroups, lane, queue_hops(OPT));
  int g = walk.first();
  if (g < ngroups) issue_chunk(g, 0, 0);
  walk.started(g);
  for (int nxt = 0; g < ngroups; g = nxt) {
    const int blk = g * BPG + rblk;
    float M[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) M[r] = (q == 0 && r == 0) ? 0.0f : __builtin_inff();
    uint8_t info[IB];
    auto period_at = [&](int p, auto growth) __attribute__((always_inline)) {
      constexpr bool GROWTH = decltype(growth)::value;
      // this chunk's DMA was issued before the previous period's 8 decision stores (in order)
      if (p >= 2) wait_vmcnt<n>();
      else wait_vmcnt<0>();
      // the next group from the ticket fetched a group ago, read right behind this full drain (see
      // acs_wide.hpp)
      if constexpr (GROWTH) nxt = walk.next(g);
      const int buf = p & 1;
      if (p + 1 < NPER) {
        issue_chunk(g, p + 1, buf ^ 1);
      } else {   // the next group's first chunk (a harmless reload of this one's when there is none)
        issue_chunk(nxt < ngroups ? nxt : g, 0, buf ^ 1);
      }
      // the ticket after nxt: behind the info loads, whose unpacking waits vmcnt(0) right away, and
      // the DMA; waited by period 1's full drain, long back by then
      if constexpr (GROWTH) walk.issued(nxt);
      const uint32_t rd = row + (uint32_t)(buf * BUF);
      f32x4 rowv = lds_read_b128<0>(rd + swz);
      auto phase_at = [&]<int P>() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rowv) :: "memory");
        const float BM[4] = {rowv.x, rowv.y, rowv.z, rowv.w};
        if constexpr (P + 1 < n) rowv = lds_read_b128<0>(rd + (swz ^ (uint32_t)((P + 1) * 16)));
        if constexpr (GROWTH) {
          if constexpr (X::is_lane(P)) multi2_growth_cross_swz<C, P, X>(M, BM, qb);
          else multi2_growth_impl<C, P, X>(M, BM, qb, std::make_index_sequence<NR>{});
        } else {
          uint32_t D[4] = {0u, 0u, 0u, 0u};
          if constexpr (X::is_lane(P)) multi2_cross_swz<C, P, X>(M, BM, qb, D);
          else multi2_step_impl<C, P, X>(M, BM, qb, D, std::make_index_sequence<NR>{});
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{D[0], D[1], D[2], D[3]}, slot, col,
                                                 kMulti2StepOff((p - 1) * n + P, STEPB), 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      [&]<int... Ps>(std::integer_sequence<int, Ps...>) __attribute__((always_inline)) {
        (phase_at.template operator()<Ps>(), ...);
      }(std::make_integer_sequence<int, n>{});
    };
    period_at(0, std::true_type{});
#pragma clang loop unroll(disable)
    for (int p = 1; p < NPER; ++p) period_at(p, std::false_type{});

    // lowest-index minimum (reference :72-79): the trellis ends on phase 0, physical = logical
    // state; lane 0 of the pair holds the lower indices when LB is the top bit, in general the index
    // is phys(q, r) -- per lane the lowest register holding the pair's minimum, then the pair's
    // lowest index
    static_assert(T % n == 0, "the persistent trellis ends on phase 0");
    float mn = tree_min<NR, float>(M);
    mn = vmin(mn, pair_swap(mn));   // the pair's minimum
    uint32_t ne[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      ne[w] = 0;
#pragma unroll
      for (int k = 31; k >= 0; --k) ne[w] = __builtin_amdgcn_alignbit(ne[w], min_minus(mn, M[32 * w + k]), 31);
    }
    const uint64_t eq_lo = ~(((uint64_t)ne[1] << 32) | ne[0]), eq_hi = ~(((uint64_t)ne[3] << 32) | ne[2]);
    // registers map to physical bits in increasing order: the lowest register is the lowest state
    const uint32_t r0 = eq_lo ? (uint32_t)__builtin_ctzll(eq_lo) : (eq_hi ? 64u + (uint32_t)__builtin_ctzll(eq_hi) : 0xFFu);
    uint32_t idx = r0 != 0xFFu ? multi2_phys<LB>((uint32_t)q, r0) : 0xFFFFFFFFu;
    {
      const uint32_t o = pair_swap_u32(idx);
      idx = o < idx ? o : idx;
    }
    const uint32_t st = mn < __builtin_inff() ? idx : 0u;   // nothing below +inf: state 0
    // Traceback in physical coordinates (acs_multi.hpp): the walk keeps the slot's lane part ql and
    // register part rl; each lane of the pair extracts its own word's candidate bit, one DPP swap
    // gives both, and the one of lane ql is the decision.
    uint32_t ql = (st >> LB) & 1u;
    uint32_t rl = compress_bit(st, LB);
    uint64_t h = st;
    const uint32_t qself = (uint32_t)q;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this group's decision stores reached L2
    // the transmitted info bytes, loaded here (round 6) rather than at the growth period, where their
    // unpacking waited vmcnt(0) at once -- for the period's DMA and the queue ticket as well; here
    // they return behind the traceback's loads
    {
      const int bc = blk < nb ? blk : nb - 1;
#pragma unroll
      for (int k = 0; k < IB; ++k) info[k] = info_src[(size_t)bc * info_stride + k];
    }
    u32x4 dw[2][n];
    auto load_period = [&]<int pp>() __attribute__((always_inline)) {   // main period pp (1-based)
#pragma unroll
      for (int P = 0; P < n; ++P)
        dw[pp & 1][P] = __builtin_amdgcn_raw_buffer_load_b128(slot, col, kMulti2StepOff((pp - 1) * n + P, STEPB), kSc1);
    };
    auto walk_period = [&]<int pp>() __attribute__((always_inline)) {
      [&]<int... Ps>(std::integer_sequence<int, Ps...>) __attribute__((always_inline)) {
        ([&]() __attribute__((always_inline)) {
          constexpr int P = n - 1 - Ps;
          uint32_t pos;
          if constexpr (X::is_lane(P)) pos = rl;
          else pos = (((rl >> X::reg_bit(P)) & 1u) << 6) | compress_bit(rl, X::reg_bit(P));
          const u32x4 w = dw[pp & 1][P];
          const uint32_t w01 = (pos & 32u) ? w.y : w.x;
          const uint32_t w23 = (pos & 32u) ? w.w : w.z;
          const uint32_t word = (pos & 64u) ? w23 : w01;
          const uint32_t own = (word >> (pos & 31u)) & 1u;
          uint32_t m = own << qself;
          m |= pair_swap_u32(m);
          const uint32_t d = (m >> ql) & 1u;
          if constexpr (X::is_lane(P)) {
            ql = d;
          } else {
            constexpr uint32_t bit = 1u << X::reg_bit(P);
            rl = (rl & ~bit) | (d << X::reg_bit(P));
          }
          h = (h << 1) | d;
        }(), ...);
      }(std::make_integer_sequence<int, n>{});
    };
    load_period.template operator()<5>();
    load_period.template operator()<4>();
    walk_period.template operator()<5>();
    load_period.template operator()<3>();
    walk_period.template operator()<4>();
    load_period.template operator()<2>();
    walk_period.template operator()<3>();
    load_period.template operator()<1>();
    walk_period.template operator()<2>();
    walk_period.template operator()<1>();
    const uint64_t bits = __builtin_bitreverse64(h);   // bit 63 - t = output of step t
    if (q == 0 && blk < nb) {
      if (a.path_metric) a.path_metric[blk] = (int32_t)mn;   // BSC input through Hamming rows
      uint8_t* o = a.out + (size_t)blk * OB;
#pragma unroll
      for (int k = 0; k < OB; ++k) o[k] = (uint8_t)(bits >> (56 - 8 * k));
      if (a.info != nullptr) {   // consumer AWGN-channel/main.c:118-144
        uint64_t ref = 0;
#pragma unroll
        for (int k = 0; k < IB; ++k) ref |= (uint64_t)info[k] << (56 - 8 * k);
        constexpr uint64_t mask = BLEN >= 64 ? ~0ull : ~(~0ull >> BLEN);
        errors += (uint32_t)__builtin_popcountll((bits ^ ref) & mask);
      }
    }
  }
  wait_vmcnt<0>();   // the look-ahead DMA writes LDS: it must land before the workgroup ends
  walk.done();
  accumulate_errors(a, errors);
}

}  // namespace ccv
