// acs_multi.hpp -- register-trellis Viterbi for K = 8, 9 (128 / 256 states), specialised per code.
//
// L = 2^(K-7) lanes of one wave decode one block; every lane holds 64 path metrics in VGPRs, so the
// register footprint and the ACS instruction stream match the K <= 7 kernel (acs_reg.hpp).
//
// Physical state numbering: phys = (q << 6) | r with q = lane within the block's lane group and
// r = register. The ACS is done in place (the survivors of predecessors s, s|1 overwrite their
// registers), so the logical meaning of the physical bits rotates by one position per step: at
// phase p = t mod (K-1) the logical state held at phys is rotr_{K-1}(phys, p). The logical bit 0 --
// the bit a butterfly pairs on -- is therefore a register bit for 6 of every K-1 steps (ordinary
// in-lane butterflies) and a lane bit for the other K-7 steps. Those cross phases need no data
// exchange: each lane reads its even and odd predecessor from the pair's two lanes with a quad_perm
// DPP move and computes the one new state its position holds (input bit = its own lane bit).
// Branch metrics depend on the lane bits, so each use takes BM[e(q)] where the expected symbol e(q)
// per lane position is a compile-time tuple; the per-lane select is shared by common subexpressions.
//
// Exactness: the same adds, strict compare (sign of odd - even) and min as the reference
// (AWGN-channel/viterbi-decoder.c:108-141); the lowest-index argmin and the traceback
// (:71-90) work on logical state numbers.
//
// Decisions: each lane packs its 64 decision bits per step (bit r = register r), stored to
// [T][P] 64-bit words, P = (nblocks * L) rounded up to 64, column = global lane index. The traceback
// is run by all L lanes of a group in lockstep: each loads its own word (address independent of the
// state) and fetches the word of lane q(state) with ds_bpermute.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "acs_persist.hpp"
#include "acs_reg.hpp"
#include "trellis.hpp"

namespace ccv {

// Physical layout: lane bit b of a block's lane group sits at physical state bit LB<b> (LB1 unused
// for K = 8), the 6 register bits at the remaining positions in increasing order. The default puts
// the lanes on the top bits (phys = q << 6 | r): the cross-lane phases are the last K - 7 of each
// period. LB = {0, 3} (the persistent K = 9 kernel) moves them to phases 0 and 3, which keeps more
// equal-candidate ("twin") states of the x86-idiom trellis inside one lane (tools/
// trellis_value_numbering.py: 100.5 adds / 50.3 mins per lane-step instead of 105.3 / 52.6).
template <CodeSpec C, int LB0 = 6, int LB1 = 7>
struct Multi {
  static constexpr int n = C.K - 1;          // state bits
  static constexpr int QB = C.K - 7;         // lane bits
  static constexpr int L = 1 << QB;          // lanes per block
  static constexpr int S = 1 << n;
  static constexpr int NS = 1 << C.n;
  static_assert(QB == 1 || LB0 != LB1, "distinct lane bits");
  static constexpr bool is_lane(int P) { return P == LB0 || (QB == 2 && P == LB1); }
  static constexpr int lane_of(int P) { return P == LB0 ? 0 : 1; }      // which q bit phys bit P is
  static constexpr int reg_bit(int P) {                                 // which r bit phys bit P is
    int k = 0;
    for (int b = 0; b < P; ++b) k += is_lane(b) ? 0 : 1;
    return k;
  }
  static constexpr uint32_t phys(int q, int r) {
    uint32_t x = 0;
    int k = 0;
    for (int b = 0; b < n; ++b) {
      if (is_lane(b)) x |= (uint32_t)((q >> lane_of(b)) & 1) << b;
      else x |= (uint32_t)((r >> k++) & 1) << b;
    }
    return x;
  }
  static constexpr uint32_t rotr(uint32_t x, int p) {
    p %= n;
    return p == 0 ? x : (((x >> p) | (x << (n - p))) & (S - 1));
  }
  static constexpr uint32_t logical(int q, int r, int p) { return rotr(phys(q, r), p); }
};

__device__ __forceinline__ uint32_t rotl_bits(uint32_t x, int k, int n) {
  return k == 0 ? x : (((x << k) | (x >> (n - k))) & ((1u << n) - 1u));
}
__device__ __forceinline__ uint32_t rotr_bits(uint32_t x, int k, int n) {
  return k == 0 ? x : (((x >> k) | (x << (n - k))) & ((1u << n) - 1u));
}

// Per-lane branch metric BM[e(q)] for a compile-time tuple e(0..L-1); qb0/qb1 = this lane's bits.
template <int L, int E0, int E1, int E2, int E3, typename MT, int NS>
__device__ __forceinline__ MT select_bm(const MT (&BM)[NS], bool qb0, bool qb1) {
  if constexpr (L == 2) {
    if constexpr (E0 == E1) return BM[E0];
    else return qb0 ? BM[E1] : BM[E0];
  } else {
    if constexpr (E0 == E1 && E1 == E2 && E2 == E3) {
      return BM[E0];
    } else {
      const MT lo = (E0 == E1) ? BM[E0] : (qb0 ? BM[E1] : BM[E0]);
      const MT hi = (E2 == E3) ? BM[E2] : (qb0 ? BM[E3] : BM[E2]);
      if constexpr (E0 == E2 && E1 == E3) return lo;
      else return qb1 ? hi : lo;
    }
  }
}

// quad_perm moves with every lane enabled: no "old" value is ever kept, so bound_ctrl and the
// old-operand-free form let the compiler fuse the move into its consumer or skip the v_mov 0
// that an update_dpp(0, ...) needs.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, true);
}
template <int CTRL, typename MT>
__device__ __forceinline__ MT dpp(MT x) {
  if constexpr (sizeof(MT) == 4 && std::is_same<MT, float>::value) return dpp_f32<CTRL>(x);
  else return dpp_u32<CTRL>(x);
}

// One new-state computation (cross phase) or one butterfly (in-lane phase) for register R, in place.
// In-lane phase P: butterfly (R, R | 1 << P); the i = 0 survivor's decision is shifted into `lo`,
// the i = 1 survivor's into `hi`, so bit compress_P(R) of lo / hi belongs to register R / R | 1 << P.
// Cross phase: the decision of register R goes to bit R of (hi:lo).
template <CodeSpec C, int P, int R, bool SAT, typename MT, class X = Multi<C>>
__device__ __forceinline__ void multi_acs(MT (&M)[64], const MT (&BM)[1 << C.n], bool qb0, bool qb1,
                                          uint32_t& lo, uint32_t& hi) {
  constexpr int L = X::L;
  auto sat = [](MT v) {
    if constexpr (SAT) return vmin(v, (MT)0xFF00);   // binary-symmetric-channel/viterbi-decoder.c:127-130
    else return v;
  };
  if constexpr (!X::is_lane(P)) {
    constexpr int k = X::reg_bit(P);
    if constexpr ((R & (1 << k)) == 0) {
      constexpr int R1 = R | (1 << k);
      constexpr auto e = [](int q, int odd, int in) {
        return expected_symbol(C, X::logical(q, R, P) | (uint32_t)odd, in);
      };
      const MT a0 = sat(M[R] + select_bm<L, e(0, 0, 0), e(1 % L, 0, 0), e(2 % L, 0, 0), e(3 % L, 0, 0)>(BM, qb0, qb1));
      const MT a1 = sat(M[R1] + select_bm<L, e(0, 1, 0), e(1 % L, 1, 0), e(2 % L, 1, 0), e(3 % L, 1, 0)>(BM, qb0, qb1));
      const MT b0 = sat(M[R] + select_bm<L, e(0, 0, 1), e(1 % L, 0, 1), e(2 % L, 0, 1), e(3 % L, 0, 1)>(BM, qb0, qb1));
      const MT b1 = sat(M[R1] + select_bm<L, e(0, 1, 1), e(1 % L, 1, 1), e(2 % L, 1, 1), e(3 % L, 1, 1)>(BM, qb0, qb1));
      M[R] = vmin(a0, a1);
      lo = shift_in(lo, a0, a1);
      M[R1] = vmin(b0, b1);
      hi = shift_in(hi, b0, b1);
    }
  } else {
    // cross-lane butterfly on lane bit B: even predecessor in the lane with bit B clear, odd in the
    // lane with it set, same register; this lane's new state has input bit = its own bit B
    constexpr int B = X::lane_of(P);
    constexpr int CE = B == 0 ? 0xA0 : 0x44;   // quad_perm [0,0,2,2] / [0,1,0,1]
    constexpr int CO = B == 0 ? 0xF5 : 0xEE;   // quad_perm [1,1,3,3] / [2,3,2,3]
    constexpr auto e = [](int q, int odd) {
      const int qe = q & ~(1 << B);
      return expected_symbol(C, X::logical(qe, R, P) | (uint32_t)odd, (q >> B) & 1);
    };
    const MT E = dpp<CE, MT>(M[R]);
    const MT O = dpp<CO, MT>(M[R]);
    const MT a0 = sat(E + select_bm<L, e(0, 0), e(1 % L, 0), e(2 % L, 0), e(3 % L, 0)>(BM, qb0, qb1));
    const MT a1 = sat(O + select_bm<L, e(0, 1), e(1 % L, 1), e(2 % L, 1), e(3 % L, 1)>(BM, qb0, qb1));
    M[R] = vmin(a0, a1);
    if constexpr (R >= 32) hi = shift_in(hi, a0, a1);
    else lo = shift_in(lo, a0, a1);
  }
}

// ds_swizzle in quad-permute mode (lane i of each quad reads lane SEL[i] of it): the LDS unit's
// crossbar, not a VALU instruction. On gfx950 a cross-lane VALU instruction (DPP, v_permlane*,
// v_readlane) drops the wave's whole VALU stream to about half rate for the next ~1000 instructions:
// a butterfly stream runs at 0.93-1.04 ns per instruction per SIMD, with 2 DPP adds per 1,605
// instructions at 1.53, with one ds_swizzle or ds_bpermute per 402 at 0.93-0.97
// (tools/raterbench7.hip, profiles/r04c/raterbench7.txt).
template <int Q0, int Q1, int Q2, int Q3>
__device__ __forceinline__ float swz_quad(float x) {
  constexpr int pat = 0x8000 | (Q3 << 6) | (Q2 << 4) | (Q1 << 2) | Q0;
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), pat));
}
template <int Q0, int Q1, int Q2, int Q3>
__device__ __forceinline__ uint32_t swz_quad_u32(uint32_t x) {
  constexpr int pat = 0x8000 | (Q3 << 6) | (Q2 << 4) | (Q1 << 2) | Q0;
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, pat);
}

// Growth step (t = P < K-1, from the reset metrics): the odd predecessor of every state is still
// unreachable (its candidate is +inf / saturated 0xFF00 and never wins the strict compare), so each
// new state is its even predecessor plus the branch metric and its decision is 0 -- the adds only
// (see acs_persist.hpp growth_step; unreachable states stay +inf / 0xFF00 exactly).
template <CodeSpec C, int P, int R, bool SAT, typename MT, class X = Multi<C>>
__device__ __forceinline__ void multi_growth(MT (&M)[64], const MT (&BM)[1 << C.n], bool qb0, bool qb1) {
  constexpr int L = X::L;
  auto sat = [](MT v) {
    if constexpr (SAT) return vmin(v, (MT)0xFF00);   // binary-symmetric-channel/viterbi-decoder.c:127-130
    else return v;
  };
  if constexpr (!X::is_lane(P)) {
    constexpr int k = X::reg_bit(P);
    if constexpr ((R & (1 << k)) == 0) {
      constexpr int R1 = R | (1 << k);
      constexpr auto e = [](int q, int in) { return expected_symbol(C, X::logical(q, R, P), in); };
      const MT even = M[R];
      M[R] = sat(even + select_bm<L, e(0, 0), e(1 % L, 0), e(2 % L, 0), e(3 % L, 0)>(BM, qb0, qb1));
      M[R1] = sat(even + select_bm<L, e(0, 1), e(1 % L, 1), e(2 % L, 1), e(3 % L, 1)>(BM, qb0, qb1));
    }
  } else {
    constexpr int B = X::lane_of(P);
    constexpr int CE = B == 0 ? 0xA0 : 0x44;   // quad_perm [0,0,2,2] / [0,1,0,1]
    constexpr auto e = [](int q) {
      const int qe = q & ~(1 << B);
      return expected_symbol(C, X::logical(qe, R, P), (q >> B) & 1);
    };
    M[R] = sat(dpp<CE, MT>(M[R]) + select_bm<L, e(0), e(1 % L), e(2 % L), e(3 % L)>(BM, qb0, qb1));
  }
}

template <CodeSpec C, int P, bool SAT, typename MT, class X = Multi<C>, size_t... I>
__device__ __forceinline__ void multi_growth_step_impl(MT (&M)[64], const MT (&BM)[1 << C.n], bool qb0,
                                                       bool qb1, std::index_sequence<I...>) {
  (multi_growth<C, P, 63 - (int)I, SAT, MT, X>(M, BM, qb0, qb1), ...);
}

template <CodeSpec C, int P, bool SAT, typename MT, class X = Multi<C>, int GRP = 0, size_t... I>
__device__ __forceinline__ uint64_t multi_step_impl(MT (&M)[64], const MT (&BM)[1 << C.n], bool qb0,
                                                    bool qb1, std::index_sequence<I...>) {
  uint32_t lo = 0, hi = 0;
  // descending registers; GRP > 0: a scheduling barrier after every GRP registers (bounds the live
  // temporaries where the register budget is tight)
  ((multi_acs<C, P, 63 - (int)I, SAT, MT, X>(M, BM, qb0, qb1, lo, hi),
    (GRP && (I + 1) % GRP == 0 ? __builtin_amdgcn_sched_barrier(0) : (void)0)),
   ...);
  return ((uint64_t)hi << 32) | lo;
}

template <CodeSpec C, int P, bool SAT, typename MT, class X = Multi<C>>
__device__ __forceinline__ uint64_t multi_step(MT (&M)[64], const MT (&BM)[1 << C.n], bool qb0, bool qb1) {
  return multi_step_impl<C, P, SAT, MT, X>(M, BM, qb0, qb1, std::make_index_sequence<64>{});
}

// Bit of register r's decision in the word stored at an in-lane phase that pairs on register bit k
// (see multi_acs: bit 5 = r's bit k, below it the other five bits in order); a cross phase stores
// register r's decision at bit r.
__device__ __forceinline__ uint32_t multi_dec_pos_k(uint32_t r, int k) {
  const uint32_t low = r & ((1u << k) - 1u);
  return (((r >> k) & 1u) << 5) | ((r >> (k + 1)) << k) | low;
}
// The same for the default layout (lanes on the top physical bits): phase p < 6 pairs on register
// bit p.
__device__ __forceinline__ uint32_t multi_dec_pos(uint32_t r, int p) {
  if (p >= 6) return r;
  return multi_dec_pos_k(r, p);
}

// One period (phases 0..n-1) of steps t .. t+n-1, each guarded by t + P < T; slot P of the input
// ring is consumed by phase P and refilled with step t + P + n. Each step's decision word goes to
// sink(std::integral_constant<int, P>, t + P, word): an HBM row or a register.
template <CodeSpec C, bool SAT, typename MT, int P, class In, class Load, class Metrics, class Sink>
__device__ __forceinline__ void multi_period(int t, int T, MT (&M)[64], In (&ring)[Multi<C>::n],
                                             Load& load, Metrics& metrics, Sink& sink, bool qb0,
                                             bool qb1) {
  if constexpr (P < Multi<C>::n) {
    constexpr int n = Multi<C>::n;
    if (t + P < T) {
      MT BM[1 << C.n];
      metrics(ring[P], BM);
      sink(std::integral_constant<int, P>{}, t + P, multi_step<C, P, SAT, MT>(M, BM, qb0, qb1));
    }
    const int tn = t + P + n;
    ring[P] = load(tn < T ? tn : T - 1);
    __builtin_amdgcn_sched_barrier(0);
    multi_period<C, SAT, MT, P + 1>(t, T, M, ring, load, metrics, sink, qb0, qb1);
  }
}

// Lowest logical index among the group's minima (reference traceback :72-79).
template <CodeSpec C, typename MT>
__device__ __forceinline__ uint32_t multi_argmin(const MT (&M)[64], int phase, int q, MT sentinel,
                                                 MT& best) {
  using X = Multi<C>;
  best = sentinel;
  uint32_t idx = 0xFFFFFFFFu;
#pragma unroll
  for (int r = 0; r < 64; ++r) {
    const uint32_t li = rotr_bits(((uint32_t)q << 6) | (uint32_t)r, phase, X::n);
    const bool better = M[r] < best || (M[r] == best && idx != 0xFFFFFFFFu && li < idx);
    best = better ? M[r] : best;
    idx = better ? li : idx;
  }
#pragma unroll
  for (int off = 1; off < X::L; off <<= 1) {
    const MT ob = __shfl_xor(best, off, 64);
    const uint32_t oi = (uint32_t)__shfl_xor((int)idx, off, 64);
    const bool better = ob < best || (ob == best && oi < idx);
    best = better ? ob : best;
    idx = better ? oi : idx;
  }
  return idx == 0xFFFFFFFFu ? 0u : idx;   // nothing below the sentinel: state 0 as the reference
}

// Same, for a trellis that ends on phase 0 (T % n == 0: the persistent kernels), without the
// compare/select chain (acs_reg.hpp argmin_state): the logical index is (q << 6) | r, so the answer
// is the lowest lane holding the group's minimum and, in it, the lowest register. v_min3 tree,
// lane minimum, "differs" mask from the sign of min - M[r], lowest clear bit, lane minimum.
// Physical state of (lane q, register r) at run time (Multi::phys).
template <class X>
__device__ __forceinline__ uint32_t multi_phys(uint32_t q, uint32_t r) {
  uint32_t x = 0;
  int k = 0;
#pragma unroll
  for (int b = 0; b < X::n; ++b) {
    if (X::is_lane(b)) x |= ((q >> X::lane_of(b)) & 1u) << b;
    else x |= ((r >> k++) & 1u) << b;
  }
  return x;
}

template <CodeSpec C, class X = Multi<C>>
__device__ __forceinline__ uint32_t multi_argmin_phase0(const float (&M)[64], int q, float sentinel,
                                                        float& best) {
  float mn = tree_min<64, float>(M);
#pragma unroll
  for (int off = 1; off < X::L; off <<= 1) mn = vmin(mn, __shfl_xor(mn, off, 64));
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int r = 31; r >= 0; --r) {
    lo = __builtin_amdgcn_alignbit(lo, min_minus(mn, M[r]), 31);
    hi = __builtin_amdgcn_alignbit(hi, min_minus(mn, M[r + 32]), 31);
  }
  const uint64_t eq = ~(((uint64_t)hi << 32) | lo);
  // registers map to physical bits in increasing order: the lowest register is the lowest state of
  // the lane; across lanes the lowest physical (= logical, phase 0) index wins
  uint32_t idx = eq ? multi_phys<X>((uint32_t)q, (uint32_t)__builtin_ctzll(eq)) : 0xFFFFFFFFu;
#pragma unroll
  for (int off = 1; off < X::L; off <<= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)idx, off, 64);
    idx = o < idx ? o : idx;
  }
  const bool found = mn < sentinel;   // nothing below the sentinel: state 0, as the reference
  best = found ? mn : sentinel;
  return found ? idx : 0u;
}

template <CodeSpec C>
__device__ __forceinline__ uint32_t multi_traceback(const RegArgs& a, int blk, uint32_t st, bool writer) {
  using X = Multi<C>;
  const int T = a.T, OB = (T + 7) >> 3, IB = (a.blen + 7) >> 3;
  const int lane = threadIdx.x & 63;
  const int gbase = lane & ~(X::L - 1);
  const uint64_t* dec = reinterpret_cast<const uint64_t*>(a.dec) + (size_t)blockIdx.x * kRegThreads + lane;
  const size_t stride = (size_t)a.dec_stride;
  uint32_t errors = 0;
  for (int lo = (T - 1) & ~7; lo >= 0; lo -= 8) {
    uint64_t w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = dec[(size_t)(lo + k < T ? lo + k : T - 1) * stride];
    uint32_t acc = 0;
#pragma unroll
    for (int k = 7; k >= 0; --k) {
      const int t = lo + k;
      if (t < T) {
        const int ph = t % X::n;   // survivors of step t sit at the phase-(t+1) positions
        const uint32_t phys = rotl_bits(st, ph + 1 == X::n ? 0 : ph + 1, X::n);
        const int src = (gbase + (int)(phys >> 6)) << 2;
        const uint32_t pos = multi_dec_pos(phys & 63u, ph);
        const uint32_t wl = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)w[k]);
        const uint32_t wh = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(w[k] >> 32));
        const uint32_t bit = ((pos < 32 ? wl : wh) >> (pos & 31)) & 1u;
        acc |= (st >> (C.K - 2)) << (7 - k);
        st = ((st << 1) & (X::S - 1)) | bit;
      }
    }
    if (writer) {
      a.out[(size_t)blk * OB + (lo >> 3)] = (uint8_t)acc;
      if (a.info != nullptr && (lo >> 3) < IB) {
        int valid = a.blen - lo;
        valid = valid > 8 ? 8 : valid;
        const uint32_t mask = (0xFFu << (8 - valid)) & 0xFFu;
        errors += __builtin_popcount((acc ^ a.info[(size_t)blk * IB + (lo >> 3)]) & mask);
      }
    }
  }
  return errors;
}

// HARD = false: soft input float [nb][T][2^n]; HARD = true: symbols uint8 [nb][T].
template <CodeSpec C, bool HARD>
__global__ __launch_bounds__(kRegThreads) void viterbi_multi(RegArgs a) {
  using X = Multi<C>;
  using MT = typename std::conditional<HARD, uint32_t, float>::type;
  constexpr int NS = X::NS;
  const int lane = threadIdx.x;
  const int q = lane & (X::L - 1);
  const bool qb0 = (q & 1) != 0, qb1 = (q & 2) != 0;
  const int blk = (blockIdx.x * kRegThreads + lane) / X::L;
  const int T = a.T, nb = a.nblocks;
  const int bc = blk < nb ? blk : nb - 1;
  uint64_t* dec = reinterpret_cast<uint64_t*>(a.dec) + (size_t)blockIdx.x * kRegThreads + lane;
  const size_t dstride = (size_t)a.dec_stride;
  MT M[64];
#pragma unroll
  for (int r = 0; r < 64; ++r) {
    if constexpr (HARD) M[r] = (q == 0 && r == 0) ? 0u : 0xFF00u;
    else M[r] = (q == 0 && r == 0) ? 0.0f : __builtin_inff();
  }
  constexpr int n = X::n;
  auto sink = [&](auto, int t, uint64_t w) { dec[(size_t)t * dstride] = w; };
  if constexpr (HARD) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(a.in) + (size_t)bc * T;
    auto load = [&](int t) { return (uint32_t)p[t]; };
    auto metrics = [](uint32_t sym, MT (&BM)[NS]) {
#pragma unroll
      for (int k = 0; k < NS; ++k) BM[k] = __builtin_popcount((uint32_t)k ^ (sym & (uint32_t)(NS - 1)));
    };
    uint32_t ring[n];
#pragma unroll
    for (int k = 0; k < n; ++k) ring[k] = load(k < T ? k : T - 1);
    // saturation (reference :127-130) only matters while some states are unreachable: period 0
    multi_period<C, true, MT, 0>(0, T, M, ring, load, metrics, sink, qb0, qb1);
    for (int t = n; t < T; t += n)
      multi_period<C, false, MT, 0>(t, T, M, ring, load, metrics, sink, qb0, qb1);
  } else {
    const float* p = reinterpret_cast<const float*>(a.in) + (size_t)bc * T * NS;
    auto load = [&](int t) { return load_soft_step<NS>(p + (size_t)t * NS); };
    auto metrics = [](const SoftStep<NS>& in, MT (&BM)[NS]) {
#pragma unroll
      for (int k = 0; k < NS; ++k) BM[k] = in.v[k];
    };
    SoftStep<NS> ring[n];
#pragma unroll
    for (int k = 0; k < n; ++k) ring[k] = load(k < T ? k : T - 1);
    for (int t = 0; t < T; t += n)
      multi_period<C, false, MT, 0>(t, T, M, ring, load, metrics, sink, qb0, qb1);
  }
  MT best;
  const MT sentinel = HARD ? (MT)0xFF00u : (MT)__builtin_inff();
  const uint32_t st = multi_argmin<C, MT>(M, T % X::n, q, sentinel, best);
  const bool writer = q == 0 && blk < nb;
  if constexpr (HARD) {
    if (writer && a.path_metric) a.path_metric[blk] = (int32_t)best;
  }
  const uint32_t errors = multi_traceback<C>(a, blk, st, writer);
  accumulate_errors(a, errors);
}

// ---------------------------------------------------------------------------------------------
// Register-resident decisions for the multilane kernel (T <= kMultiRegDecSteps), as
// viterbi_soft_regdec does for K <= 7: each lane keeps its 64-bit decision word of every step in
// VGPRs (2 x T registers), so nothing is written to or read back from a decision scratch array. The
// periods are expanded at compile time (every D[p][P] index is a constant); the traceback walks the
// group's words with one ds_bpermute per step -- every lane of a group holds the same state, so each
// lane pre-selects the half of its own word the state's position needs.
constexpr int kMultiRegDecSteps = 48;

template <CodeSpec C>
inline constexpr int kMultiRegDecPeriods = (kMultiRegDecSteps + Multi<C>::n - 1) / Multi<C>::n;

template <CodeSpec C, bool HARD, int WAVES = 2>
__global__ __launch_bounds__(kRegThreads) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES)))
void viterbi_multi_regdec(RegArgs a) {
  using X = Multi<C>;
  using MT = typename std::conditional<HARD, uint32_t, float>::type;
  constexpr int NS = X::NS;
  constexpr int n = X::n;
  constexpr int NP = kMultiRegDecPeriods<C>;
  const int lane = threadIdx.x;
  const int q = lane & (X::L - 1);
  const bool qb0 = (q & 1) != 0, qb1 = (q & 2) != 0;
  const int blk = (blockIdx.x * kRegThreads + lane) / X::L;
  const int T = a.T, nb = a.nblocks;   // host guarantees T <= NP * n
  const int bc = blk < nb ? blk : nb - 1;
  MT M[64];
#pragma unroll
  for (int r = 0; r < 64; ++r) {
    if constexpr (HARD) M[r] = (q == 0 && r == 0) ? 0u : 0xFF00u;
    else M[r] = (q == 0 && r == 0) ? 0.0f : __builtin_inff();
  }
  uint64_t D[NP][n];
  auto run = [&](auto& ring, auto& load, auto& metrics) {
    auto period_at = [&]<int p>() {
      if (p * n < T) {
        auto sink = [&](auto Pc, int, uint64_t w) { D[p][decltype(Pc)::value] = w; };
        // saturation (reference :127-130) only matters while some states are unreachable: period 0
        multi_period<C, HARD && p == 0, MT, 0>(p * n, T, M, ring, load, metrics, sink, qb0, qb1);
      }
    };
    [&]<int... ps>(std::integer_sequence<int, ps...>) {
      (period_at.template operator()<ps>(), ...);
    }(std::make_integer_sequence<int, NP>{});
  };
  if constexpr (HARD) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(a.in) + (size_t)bc * T;
    auto load = [&](int t) { return (uint32_t)p[t]; };
    auto metrics = [](uint32_t sym, MT (&BM)[NS]) {
#pragma unroll
      for (int k = 0; k < NS; ++k) BM[k] = __builtin_popcount((uint32_t)k ^ (sym & (uint32_t)(NS - 1)));
    };
    uint32_t ring[n];
#pragma unroll
    for (int k = 0; k < n; ++k) ring[k] = load(k < T ? k : T - 1);
    run(ring, load, metrics);
  } else {
    const float* p = reinterpret_cast<const float*>(a.in) + (size_t)bc * T * NS;
    auto load = [&](int t) { return load_soft_step<NS>(p + (size_t)t * NS); };
    auto metrics = [](const SoftStep<NS>& in, MT (&BM)[NS]) {
#pragma unroll
      for (int k = 0; k < NS; ++k) BM[k] = in.v[k];
    };
    SoftStep<NS> ring[n];
#pragma unroll
    for (int k = 0; k < n; ++k) ring[k] = load(k < T ? k : T - 1);
    run(ring, load, metrics);
  }
  MT best;
  const MT sentinel = HARD ? (MT)0xFF00u : (MT)__builtin_inff();
  uint32_t st = multi_argmin<C, MT>(M, T % n, q, sentinel, best);
  const bool writer = q == 0 && blk < nb;
  if constexpr (HARD) {
    if (writer && a.path_metric) a.path_metric[blk] = (int32_t)best;
  }
  // traceback (reference :71-90) over the group's register decisions, steps T-1 ... 0; decoded bits
  // are shifted in from the top, so bit 63 ends up holding step 0 (MSB-first output)
  const int gbase = lane & ~(X::L - 1);
  uint64_t bits = 0;
  auto back_step = [&]<int p, int P>() {
    if (p * n + P < T) {
      // survivors of step t sit at the phase-(t+1) positions (t mod n = P)
      const uint32_t phys = rotl_bits(st, P + 1 == n ? 0 : P + 1, n);
      const uint32_t pos = multi_dec_pos(phys & 63u, P);
      const uint64_t w = D[p][P];
      const uint32_t half = pos < 32 ? (uint32_t)w : (uint32_t)(w >> 32);
      const int src = (gbase + (int)(phys >> 6)) << 2;
      const uint32_t word = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)half);
      const uint32_t bit = (word >> (pos & 31)) & 1u;
      bits = (bits >> 1) | ((uint64_t)(st >> (C.K - 2)) << 63);
      st = ((st << 1) & (X::S - 1)) | bit;
    }
  };
  auto back_period = [&]<int p>() {
    [&]<int... Ps>(std::integer_sequence<int, Ps...>) {
      (back_step.template operator()<p, n - 1 - Ps>(), ...);
    }(std::make_integer_sequence<int, n>{});
  };
  [&]<int... ps>(std::integer_sequence<int, ps...>) {
    (back_period.template operator()<NP - 1 - ps>(), ...);
  }(std::make_integer_sequence<int, NP>{});
  uint32_t errors = 0;
  if (writer) {
    const int OB = (T + 7) >> 3, IB = (a.blen + 7) >> 3;
    uint8_t* o = a.out + (size_t)blk * OB;
    for (int k = 0; k < OB; ++k) o[k] = (uint8_t)(bits >> (56 - 8 * k));
    if (a.info != nullptr) {   // consumer AWGN-channel/main.c:118-144: errors in the first blen bits
      const uint8_t* inf = a.info + (size_t)blk * IB;
      uint64_t ref = 0;
      for (int k = 0; k < IB; ++k) ref |= (uint64_t)inf[k] << (56 - 8 * k);
      const uint64_t mask = a.blen >= 64 ? ~0ull : ~(~0ull >> a.blen);
      errors = (uint32_t)__builtin_popcountll((bits ^ ref) & mask);
    }
  }
  accumulate_errors(a, errors);
}

// ---------------------------------------------------------------------------------------------
// Persistent K = 9 soft kernel at the codebook block length (blen 40: T = 48 = six periods of the
// 8-phase rotation, so a period is exactly one 8-step input chunk), built like the K <= 7
// persistent kernel (acs_persist.hpp): resident waves walk groups of 16 blocks (4 lanes each);
// period 0 is the growth from the reset metrics (adds only, no decisions); the 40 main steps keep
// their decision words in VGPRs; the input is staged by LDS-DMA one chunk ahead (2 KiB per chunk:
// 16 blocks x 8 steps x 16 bytes; the 4 lanes of a block read the same row).
// Ablation switches for timing studies (tools/k9_bench.hip); production kernels use 0.
enum : int { kMultiNoTraceback = 1, kMultiNoMem = 2, kMultiBpermuteTraceback = 4 };

// LDSP: main periods whose decision words go to LDS instead of VGPRs (8 x 8 B x 64 lanes = 4 KiB
// per period per wave): each one frees 16 VGPRs, and with two of them the kernel fits 3 waves per SIMD.
template <CodeSpec C, int BLEN, int ABLATE = 0, int LDSP = 0, int LB0 = 6, int LB1 = 7>
__global__ __launch_bounds__(kRegThreads) __attribute__((amdgpu_waves_per_eu(LDSP >= 2 ? 3 : 2)))
void viterbi_multi_persist(RegArgs a, int ngroups) {
  using X = Multi<C, LB0, LB1>;
  using MT = float;
  static_assert(C.K == 9 && C.n == 2, "K = 9, r = 1/2: the period (8 steps) is the 8-step chunk");
  constexpr int n = X::n;                     // 8 phases per period
  constexpr int T = BLEN + C.K - 1;
  static_assert(T % n == 0 && T / n >= 2 && T / n <= 7, "whole periods");
  constexpr int NPER = T / n;                 // periods = chunks
  constexpr int NMAIN = NPER - 1;             // periods with decisions
  constexpr int BPG = kRegThreads / X::L;     // blocks per group (16)
  constexpr int ROWB = n * 16;                // one chunk of one block: 128 bytes
  constexpr int BUF = BPG * ROWB;             // 2 KiB
  constexpr int UNITS = BUF / 16;             // 16-byte DMA units per chunk (128: 2 instructions)
  constexpr int IB = (BLEN + 7) >> 3, OB = (T + 7) >> 3;
  constexpr uint32_t block_bytes = (uint32_t)T * 16;
  const int lane = threadIdx.x;
  const int q = lane & (X::L - 1);
  const bool qb0 = (q & 1) != 0, qb1 = (q & 2) != 0;
  const int nb = a.nblocks;
  const int stride_groups = gridDim.x;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[BUF];
  __shared__ uint64_t ldsdec[LDSP > 0 ? LDSP * n * kRegThreads : 1];
  const unsigned char* in = reinterpret_cast<const unsigned char*>(a.in);
  // DMA k of a chunk: unit k*64 + lane = block r (of 16), 16-byte step j of its chunk
  auto issue_chunk = [&](int g, int c) __attribute__((always_inline)) {
    if constexpr ((ABLATE & kMultiNoMem) != 0) return;
#pragma unroll
    for (int k = 0; k < UNITS / kRegThreads; ++k) {
      const int unit = k * kRegThreads + lane;
      const int r = unit / n, j = unit % n;
      const int gb = g * BPG + r < nb ? g * BPG + r : nb - 1;
      __builtin_amdgcn_global_load_lds(in + (size_t)gb * block_bytes + (uint32_t)(c * n + j) * 16,
                                       (lds_ptr_t)(lds + k * kRegThreads * 16), 16, 0, 0);
    }
  };
  const uint32_t row = (uint32_t)(uintptr_t)(lds_ptr_t)lds + (uint32_t)((lane / X::L) * ROWB);
  const uint8_t* info_src = a.info != nullptr ? a.info : reinterpret_cast<const uint8_t*>(a.in);
  const int info_stride = a.info != nullptr ? IB : 0;
  const int gbase = lane & ~(X::L - 1);

  uint32_t errors = 0;
  int g = blockIdx.x;
  if (g < ngroups) issue_chunk(g, 0);
  for (; g < ngroups; g += stride_groups) {
    const int blk = g * BPG + lane / X::L;
    const bool has_next = g + stride_groups < ngroups;
    MT M[64];
#pragma unroll
    for (int r = 0; r < 64; ++r) M[r] = (q == 0 && r == 0) ? 0.0f : __builtin_inff();
    uint64_t D[NMAIN - LDSP > 0 ? NMAIN - LDSP : 1][n];
    uint8_t info[IB];
    auto period_at = [&]<int p>() __attribute__((always_inline)) {
      f32x4 chunk[n];
      wait_vmcnt<0>();
      if constexpr ((ABLATE & kMultiNoMem) != 0) {   // full-entropy synthetic rows in [1, 2)
        uint32_t ln = (uint32_t)(lane / X::L + g * 131 + p * 977) * 0x9E3779B9u;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int x = 0; x < n; ++x) {
          const uint32_t r0 = ln ^ (uint32_t)(x * 0x85EBCA6Bu), r1 = r0 * 0xC2B2AE35u;
          chunk[x] = f32x4{__uint_as_float((r0 >> 9) | 0x3F800000u), __uint_as_float((r1 >> 9) | 0x3F800000u),
                           __uint_as_float((r0 & 0x7FFFFFu) | 0x3F800000u), __uint_as_float((r1 & 0x7FFFFFu) | 0x3F800000u)};
        }
      } else
      [&]<int... xs>(std::integer_sequence<int, xs...>) __attribute__((always_inline)) {
        ((chunk[xs] = lds_read_b128<xs * 16>(row)), ...);
      }(std::make_integer_sequence<int, n>{});
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(chunk[0]), "+v"(chunk[1]), "+v"(chunk[2]), "+v"(chunk[3]), "+v"(chunk[4]),
                     "+v"(chunk[5]), "+v"(chunk[6]), "+v"(chunk[7])
                   :
                   : "memory");
      if constexpr (p == 0) {
        const int bc = blk < nb ? blk : nb - 1;
#pragma unroll
        for (int k = 0; k < IB; ++k) info[k] = info_src[(size_t)bc * info_stride + k];
        asm volatile("" ::: "memory");   // info loads before the DMA (vmcnt order)
      }
      if constexpr (p + 1 < NPER) issue_chunk(g, p + 1);
      else issue_chunk(has_next ? g + stride_groups : g, 0);
      auto phase_at = [&]<int P>() __attribute__((always_inline)) {
        const MT BM[4] = {chunk[P].x, chunk[P].y, chunk[P].z, chunk[P].w};
        if constexpr (p == 0) {
          multi_growth_step_impl<C, P, false, MT, X>(M, BM, qb0, qb1, std::make_index_sequence<64>{});
        } else {
          if constexpr (p - 1 < LDSP) {
            ldsdec[((p - 1) * n + P) * kRegThreads + lane] = multi_step<C, P, false, MT, X>(M, BM, qb0, qb1);
          } else {
            D[p - 1 - LDSP][P] = multi_step<C, P, false, MT, X>(M, BM, qb0, qb1);
            pin(D[p - 1 - LDSP][P]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      [&]<int... Ps>(std::integer_sequence<int, Ps...>) __attribute__((always_inline)) {
        (phase_at.template operator()<Ps>(), ...);
      }(std::make_integer_sequence<int, n>{});
    };
    [&]<int... ps>(std::integer_sequence<int, ps...>) __attribute__((always_inline)) {
      (period_at.template operator()<ps>(), ...);
    }(std::make_integer_sequence<int, NPER>{});

    if constexpr ((ABLATE & kMultiNoTraceback) != 0) {
      uint64_t x = 0;
#pragma unroll
      for (int pp = 0; pp < NMAIN - LDSP; ++pp)
#pragma unroll
        for (int P = 0; P < n; ++P) x ^= D[pp][P];
#pragma unroll
      for (int k = 0; k < LDSP * n; ++k) x ^= ldsdec[k * kRegThreads + lane];
#pragma unroll
      for (int r = 0; r < 64; ++r) x += __float_as_uint(M[r]);
      if (blk < nb) reinterpret_cast<uint64_t*>(a.out)[blk * X::L + q] = x;
      continue;
    }
    MT best;
    static_assert(T % n == 0, "the persistent trellis ends on phase 0");
    uint32_t st = multi_argmin_phase0<C, X>(M, q, __builtin_inff(), best);
    uint64_t bits = 0;
    if constexpr ((ABLATE & kMultiBpermuteTraceback) != 0) {   // round-2 traceback (A/B)
      static_assert(LB0 == 6 && LB1 == 7, "the round-2 traceback knows the default layout only");
      auto back_step = [&]<int p, int P>() __attribute__((always_inline)) {
        // survivors of step t sit at the phase-(t+1) positions (t mod n = P)
        const uint32_t phys = rotl_bits(st, P + 1 == n ? 0 : P + 1, n);
        uint32_t bit = 0;
        if constexpr (p > 0) {
          const uint32_t pos = multi_dec_pos(phys & 63u, P);
          const uint64_t w = p - 1 < LDSP ? ldsdec[((p - 1) * n + P) * kRegThreads + lane]
                                          : D[p - 1 - LDSP < 0 ? 0 : p - 1 - LDSP][P];
          const uint32_t half = pos < 32 ? (uint32_t)w : (uint32_t)(w >> 32);
          const int src = (gbase + (int)(phys >> 6)) << 2;
          const uint32_t word = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)half);
          bit = (word >> (pos & 31)) & 1u;
        }
        bits = (bits >> 1) | ((uint64_t)(st >> (C.K - 2)) << 63);
        st = ((st << 1) & (X::S - 1)) | bit;
      };
      auto back_period = [&]<int p>() __attribute__((always_inline)) {
        [&]<int... Ps>(std::integer_sequence<int, Ps...>) __attribute__((always_inline)) {
          (back_step.template operator()<p, n - 1 - Ps>(), ...);
        }(std::make_integer_sequence<int, n>{});
      };
      [&]<int... ps>(std::integer_sequence<int, ps...>) __attribute__((always_inline)) {
        (back_period.template operator()<NPER - 1 - ps>(), ...);
      }(std::make_integer_sequence<int, NPER>{});
    } else {
      // Traceback in physical coordinates, no LDS round trip. The in-place ACS stores the survivor
      // of logical state s at phase P+1 in physical slot rotl(s, P+1); one step back the logical
      // state becomes ((s << 1) | d) mod S, whose physical slot at phase P is the same slot with
      // ONLY bit P replaced by the decision d. So the walk keeps phys (8 bits: lane q = phys >> 6,
      // register r = phys & 63), reads d at bit dec_pos(r, P) of lane q's word and writes it into
      // bit P. The four lanes of a group hold the same phys: each extracts its own candidate bit
      // and two quad DPP ORs give every lane all four, from which it takes lane q's.
      // The decoded bits: the final state's 8 bits are the outputs of the last 8 steps, and the
      // decision read at step t is the output of step t - 8 (it reaches the top state bit 8 steps
      // earlier), so the history h = st, then (h << 1) | d per main step, holds output i at bit i.
      // phase 0: physical = logical; the walk keeps phys split into its lane and register parts
      uint32_t ql = 0, rl = 0;
      {
        int k = 0;
#pragma unroll
        for (int b = 0; b < n; ++b) {
          if (X::is_lane(b)) ql |= ((st >> b) & 1u) << X::lane_of(b);
          else rl |= ((st >> b) & 1u) << k++;
        }
      }
      uint64_t h = st;
      const uint32_t qself = (uint32_t)q;
      auto back_step = [&]<int p, int P>() __attribute__((always_inline)) {
        if constexpr (p > 0) {
          uint32_t pos;
          if constexpr (X::is_lane(P)) pos = rl;
          else pos = multi_dec_pos_k(rl, X::reg_bit(P));
          uint64_t w;
          if constexpr (p - 1 < LDSP) w = ldsdec[((p - 1) * n + P) * kRegThreads + lane];
          else w = D[p - 1 - LDSP][P];
          const uint32_t own = (uint32_t)(w >> pos) & 1u;
          uint32_t m = own << qself;
          m |= dpp_u32<0xB1>(m);   // quad_perm [1,0,3,2]
          m |= dpp_u32<0x4E>(m);   // quad_perm [2,3,0,1]
          const uint32_t d = (m >> ql) & 1u;
          if constexpr (X::is_lane(P)) {
            constexpr uint32_t bit = 1u << X::lane_of(P);
            ql = (ql & ~bit) | (d << X::lane_of(P));
          } else {
            constexpr uint32_t bit = 1u << X::reg_bit(P);
            rl = (rl & ~bit) | (d << X::reg_bit(P));
          }
          h = (h << 1) | d;
        }
      };
      auto back_period = [&]<int p>() __attribute__((always_inline)) {
        [&]<int... Ps>(std::integer_sequence<int, Ps...>) __attribute__((always_inline)) {
          (back_step.template operator()<p, n - 1 - Ps>(), ...);
        }(std::make_integer_sequence<int, n>{});
      };
      [&]<int... ps>(std::integer_sequence<int, ps...>) __attribute__((always_inline)) {
        (back_period.template operator()<NPER - 1 - ps>(), ...);
      }(std::make_integer_sequence<int, NPER>{});
      bits = __builtin_bitreverse64(h);   // bit 63 - t = output of step t
    }
    if (q == 0 && blk < nb) {
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
  accumulate_errors(a, errors);
}

}  // namespace ccv
