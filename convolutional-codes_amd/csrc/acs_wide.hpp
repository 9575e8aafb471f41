// acs_wide.hpp -- persistent one-lane-per-block Viterbi for K = 9 r = 1/2 soft (256 states), gfx950.
//
// The four-lane kernel (acs_multi.hpp) splits a block's 256 metrics over four lanes, which costs the
// x86-idiom trellis its twin sharing: 402 adds / 201 mins per block-step against 300 / 156 when the
// whole trellis sits in one lane (tools/trellis_value_numbering.py, profiles/
// r02e_trellis_value_numbering.txt: only 156 of the 256 metrics are distinct each step). Here one lane
// holds a whole block, as the K <= 7 persistent kernel does (acs_persist.hpp): the 256 metrics are
// SSA values the compiler value-numbers, so only the distinct ones occupy VGPRs. What does not fit is
// the survivor decisions (40 main steps x 256 bits = 320 VGPRs per lane), so each step's eight
// decision words go to a per-wave scratch slot in global memory (80 KiB per wave, rewritten by every
// group the wave decodes, so it stays in the L2 / Infinity Cache working set), and the traceback
// loads them back in two bulk batches once the metrics are dead.
//
// Arithmetic as AWGN-channel/viterbi-decoder.c:108-141 (fp32 adds, strict compare = sign of
// m1 - m0, even predecessor on ties, +inf reset metrics) and traceback :71-90 (lowest-index argmin).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "acs_persist.hpp"
#include "twins.hpp"

namespace ccv {

// Consecutive collapsed butterflies directly below j inside j's 32-bit decision word.
template <CodeSpec C>
constexpr int collapsed_below_word(int j) {
  int h = 0;
  for (int k = j - 1; k >= (j & ~31) && collapsed_butterfly<C>(k); --k) ++h;
  return h;
}
template <CodeSpec C>
constexpr uint32_t collapsed_mask_word(int w) {
  uint32_t m = 0;
  for (int k = 0; k < 32; ++k)
    if (collapsed_butterfly<C>(32 * w + k)) m |= 1u << k;
  return m;
}

// Packed decisions (PACK 1): a collapsed butterfly's upper decision IS its lower one (same
// candidates by construction), so only the lower words and the non-collapsed upper decisions are
// stored, densely: K = 9 idiom 128 + 43 bits = 6 words per step instead of 8.
template <CodeSpec C>
constexpr int noncollapsed_count() {
  int n = 0;
  for (int j = 0; j < (1 << (C.K - 2)); ++j) n += collapsed_butterfly<C>(j) ? 0 : 1;
  return n;
}
template <CodeSpec C>
constexpr int noncollapsed_rank(int j) {   // non-collapsed butterflies above j (descending order)
  int r = 0;
  for (int k = j + 1; k < (1 << (C.K - 2)); ++k) r += collapsed_butterfly<C>(k) ? 0 : 1;
  return r;
}
template <CodeSpec C>
constexpr int packed_words() {
  return (1 << (C.K - 2)) / 32 + (noncollapsed_count<C>() + 31) / 32;
}
// PACK 2: one decision per value-numbering class of the idiom trellis (twins.hpp, generated)
// (twin_code: acs_persist.hpp)
// four 8-bit positions per word, for an LDS copy
template <int K>
struct TwinPosTable {
  uint32_t v[(1 << (K - 1)) / 4];
  constexpr TwinPosTable() : v() {
    for (int s = 0; s < (1 << (K - 1)); ++s) v[s / 4] |= (uint32_t)TwinTable<K>::pos[s] << (8 * (s % 4));
  }
};

template <CodeSpec C>
struct PackedPosTable {
  uint32_t v[(1 << (C.K - 1)) / 4];   // four 8-bit positions (word << 5 | bit) per word
  constexpr PackedPosTable() : v() {
    constexpr int H = 1 << (C.K - 2);
    bool col[H] = {};
    int rank[H] = {};
    int nc = 0;
    for (int j = H - 1; j >= 0; --j) {
      col[j] = collapsed_butterfly<C>(j);
      rank[j] = nc;
      nc += col[j] ? 0 : 1;
    }
    for (int ns = 0; ns < 2 * H; ++ns) {
      uint32_t pos = (uint32_t)(ns < H ? ns : ns - H);
      if (ns >= H && !col[ns - H]) {
        const int r = rank[ns - H], w = r / 32, cnt = nc - 32 * w < 32 ? nc - 32 * w : 32;
        pos = (uint32_t)(((H / 32 + w) << 5) | (cnt - 1 - r % 32));
      }
      v[ns / 4] |= pos << (8 * (ns % 4));
    }
  }
};

// m ? a : b with a VGPR mask (v_bitop3 truth table 0xca, acs_reg.hpp select_bits).
__device__ __forceinline__ uint32_t select_v(uint32_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}

// One trellis step over S = 2^(K-1) > 64 states in one lane: decision word w holds new states
// 32w .. 32w + 31 (bit k = state 32w + k). Butterfly j (old 2j, 2j+1 -> new j, j + S/2) as acs_step;
// a collapsed butterfly's upper decision is the lower one's, filled per word by one v_bitop3.
template <CodeSpec C, int PACK, int NW>
__device__ __forceinline__ void acs_step_wide(float (&M)[1 << (C.K - 1)], const float (&BM)[1 << C.n],
                                              uint32_t (&d)[NW]) {
  constexpr int S = 1 << (C.K - 1);
  constexpr int H = S / 2;
  constexpr int HW = H / 32;
  float N[S];
#pragma unroll
  for (int w = 0; w < NW; ++w) d[w] = 0;
  [&]<int... js>(std::integer_sequence<int, js...>) __attribute__((always_inline)) {
    ([&]() __attribute__((always_inline)) {
      constexpr int j = H - 1 - js;   // descending: state j ends up in bit j % 32 of word j / 32
      const float a0 = M[2 * j] + BM[expected_symbol(C, 2 * j, 0)];
      const float a1 = M[2 * j + 1] + BM[expected_symbol(C, 2 * j + 1, 0)];
      const float b0 = M[2 * j] + BM[expected_symbol(C, 2 * j, 1)];
      const float b1 = M[2 * j + 1] + BM[expected_symbol(C, 2 * j + 1, 1)];
      N[j] = vmin(a0, a1);
      N[j + H] = vmin(b0, b1);
      if constexpr (PACK == 2) {   // the class representatives only, at their packed positions
        using TT = TwinTable<C.K>;
        if constexpr (TT::rep[j] != 0) d[TT::pos[j] >> 5] = shift_in(d[TT::pos[j] >> 5], a0, a1);
        if constexpr (TT::rep[j + H] != 0) d[TT::pos[j + H] >> 5] = shift_in(d[TT::pos[j + H] >> 5], b0, b1);
        return;
      }
      d[j / 32] = shift_in(d[j / 32], a0, a1);
      if constexpr (PACK == 1 && !collapsed_butterfly<C>(j)) {
        constexpr int w = HW + noncollapsed_rank<C>(j) / 32;
        d[w] = shift_in(d[w], b0, b1);
      } else if constexpr (!collapsed_butterfly<C>(j)) {
        d[HW + j / 32] = shift_in_n<collapsed_below_word<C>(j)>(d[HW + j / 32], b0, b1);
      }
    }(), ...);
  }(std::make_integer_sequence<int, H>{});
  if constexpr (!PACK)
    [&]<int... ws>(std::integer_sequence<int, ws...>) __attribute__((always_inline)) {
      ([&]() __attribute__((always_inline)) {
        if constexpr (collapsed_mask_word<C>(ws) != 0)
          d[HW + ws] = select_bits(collapsed_mask_word<C>(ws), d[ws], d[HW + ws]);
      }(), ...);
    }(std::make_integer_sequence<int, HW>{});
#pragma unroll
  for (int s = 0; s < S; ++s) M[s] = N[s];
}

// Growth step t (acs_persist.hpp growth_step) with every state index a template constant: at
// S = 256 the loop form is not fully unrolled and the parities are then computed at run time.
template <CodeSpec C, int t>
__device__ __forceinline__ void growth_step_wide(float (&M)[1 << (C.K - 1)], const float (&BM)[1 << C.n]) {
  constexpr int S = 1 << (C.K - 1);
  constexpr int H = S / 2;
  constexpr int stride = 1 << (C.K - 2 - t);
  float N[S];
  [&]<int... ns>(std::integer_sequence<int, ns...>) __attribute__((always_inline)) {
    ([&]() __attribute__((always_inline)) {
      if constexpr (ns % stride == 0) {
        constexpr int i = ns >> (C.K - 2);
        constexpr int s0 = 2 * (ns & (H - 1));
        N[ns] = M[s0] + BM[expected_symbol(C, s0, i)];
      } else {
        N[ns] = __builtin_inff();
      }
    }(), ...);
  }(std::make_integer_sequence<int, S>{});
#pragma unroll
  for (int s = 0; s < S; ++s) M[s] = N[s];
}

// Lowest-index minimum over S > 64 states (acs_reg.hpp argmin_state: v_min3 tree, per state the sign
// of mn - M[s] into a "differs" mask, lowest clear bit).
template <int S>
__device__ __forceinline__ uint32_t argmin_wide(const float (&M)[S], float& mn) {
  constexpr int W = S / 32;
  mn = tree_min<S, float>(M);
  uint32_t idx = 0;
#pragma unroll
  for (int w = W - 1; w >= 0; --w) {   // the lowest word with a minimum wins
    uint32_t ne = 0;
#pragma unroll
    for (int k = 31; k >= 0; --k) ne = __builtin_amdgcn_alignbit(ne, min_minus(mn, M[32 * w + k]), 31);
    idx = ne != ~0u ? (uint32_t)(32 * w + __builtin_ctz(~ne)) : idx;
  }
  return mn < __builtin_inff() ? idx : 0u;   // nothing below +inf: state 0, as the reference
}

// Scratch: one slot per wave of the grid, [main step][half][lane][4 words] (a store of four words of
// 64 lanes is one contiguous KiB).
template <CodeSpec C, int PACK>
constexpr int wide_words() {
  if constexpr (PACK == 2) return TwinTable<C.K>::words;
  else return PACK == 1 ? packed_words<C>() : (1 << (C.K - 1)) / 32;
}
template <CodeSpec C, int PACK = 0>
constexpr size_t wide_slot_bytes(int main_steps) {
  return (size_t)main_steps * kRegThreads * 4 * wide_words<C, PACK>();
}

// ABLATE (timing studies, tools/k9_bench.hip; production 0): 1 decisions discarded, 2 no traceback
// loads, 4 input with the default cache policy, 16 (round 3: drain the decision stores before the
// traceback; the production default since round 4),
// 32 packed without the position table (wrong output), 64 packed upper words padded to a dwordx4.
// PACK: decision words per step. 0: 8, the collapsed upper bits filled in from the lower words;
// 1: 6, the 128 lower decisions and the 43 non-collapsed upper ones dense (0.91x the time of 0);
// 2 (production): 5, one per value-numbering class of the trellis (156, twins.hpp; 0.87x). With
// 1 and 2 the traceback takes a state's (word, bit) from a 256-byte LDS table
// (profiles/r03_k9_wide_packed_ab.txt, profiles/r03_k9_wide_twin_ab.txt).
template <CodeSpec C, int BLEN, int ABLATE = 0, int PACK = 0>
__global__ __launch_bounds__(kRegThreads) __attribute__((amdgpu_waves_per_eu(2)))
void viterbi_wide_persist(RegArgs a, int ngroups) {
  constexpr int S = 1 << (C.K - 1);
  static_assert(C.n == 2 && S == 256, "K = 9, r = 1/2");
  constexpr int PF = 8;                       // steps per chunk
  constexpr int UPR = PF;                     // 16-byte units per block per chunk = DMAs per chunk
  constexpr int ROWB = UPR * 16;
  constexpr int GRP = 16 / UPR;
  constexpr int BUF = kRegThreads * ROWB;     // one chunk of the group: 8 KiB
  constexpr int G = C.K - 1;                  // growth steps
  constexpr int T = BLEN + G;
  constexpr int NCH = (T + PF - 1) / PF;
  constexpr int IB = (BLEN + 7) >> 3, OB = (T + 7) >> 3;
  constexpr int W = wide_words<C, PACK>();    // decision words per step
  constexpr int WH = W - 4;                   // upper words
  static_assert(WH == 1 || WH == 2 || WH == 4, "upper words stored as one dword / dwordx2 / dwordx4 per lane");
  static_assert(PACK != 2 || twin_code<C>(), "twins.hpp describes the K = 9 (561,753) x86-idiom code");
  constexpr int WS = (ABLATE & 64) ? 4 : WH;  // upper words as stored (AB & 64: padded to a dwordx4)
  constexpr int STEPB = kRegThreads * 4 * (4 + WS);   // slot bytes per main step
  static_assert(T % PF == 0 && G == PF, "K = 9 at blen 40: chunk 0 is the growth, 5 main chunks");
  static_assert(T <= 64, "the history fits 64 bits");
  const int lane = threadIdx.x;
  const int nb = a.nblocks;

  // two chunk buffers: chunk c lives in buffer c % 2 (NCH is even, so the parity carries across
  // groups), and the DMA of chunk c + 1 may start as soon as chunk c's rows are due -- the rows are
  // read from LDS step by step (one step ahead), never held for a whole chunk
  static_assert(NCH % 2 == 0, "buffer = chunk parity across groups");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * BUF];
  const unsigned char* in = reinterpret_cast<const unsigned char*>(a.in);
  constexpr uint32_t block_bytes = (uint32_t)T * 16;
  // DMA k of a chunk: lane l moves 16-byte unit j = l % 8 of block r = 8k + l / 8 of the group from
  // swizzled slot j ^ (r / 2 % 8) (acs_persist.hpp viterbi_soft_persist). r / 2 % 8 = l / 16 + 4 (k % 2)
  // and a block is 768 B (bits 4-6 of r * 768 clear), so the lane's offset is one of two values,
  // off_e (even k) and off_e ^ 64 (odd k), plus 8k blocks, a wave-uniform SGPR offset: the buffer
  // form of the DMA then needs no VALU at all (the global form wanted a 64-bit VGPR address per DMA,
  // recomputed from an opaque lane at every issue to save VGPRs the ACS needs).
  static_assert(UPR == 8 && GRP == 2 && block_bytes % 128 == 0, "the two-offset form of the DMA swizzle");
  const uint32_t off_e = (uint32_t)(lane / UPR) * block_bytes + (uint32_t)((lane % UPR) ^ (lane / 16)) * 16;
  const uint32_t off_o = off_e ^ 64u;
  auto issue_chunk = [&](int g, int c, int buf) __attribute__((always_inline)) {
    int ln = threadIdx.x;
    asm volatile("" : "+v"(ln));
    if (g * kRegThreads + kRegThreads < nb) {
      const __amdgpu_buffer_rsrc_t grp = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<unsigned char*>(in) + (size_t)g * kRegThreads * block_bytes, 0,
          kRegThreads * block_bytes, 0x00020000);
#pragma unroll
      for (int k = 0; k < UPR; ++k)
        // nt (aux 2): the input is read once; 0.976x the time of the default policy (the decision
        // slots keep more of the caches, profiles/r03_k9_wide.txt); AB & 4: default policy
        __builtin_amdgcn_raw_ptr_buffer_load_lds(grp, (lds_ptr_t)(lds + buf * BUF + k * kRegThreads * 16), 16,
                                                 (k & 1) ? off_o : off_e,
                                                 c * PF * 16 + k * (kRegThreads / UPR) * (int)block_bytes, 0,
                                                 (ABLATE & 4) ? 0 : 2);
    } else {
#pragma unroll
      for (int k = 0; k < UPR; ++k) {
        const int r = k * (kRegThreads / UPR) + ln / UPR, j = ln % UPR;
        const int su = j ^ ((r / GRP) % UPR);
        const int gb = g * kRegThreads + r < nb ? g * kRegThreads + r : nb - 1;
        __builtin_amdgcn_global_load_lds(in + (size_t)gb * block_bytes + (uint32_t)(c * PF + su) * 16,
                                         (lds_ptr_t)(lds + buf * BUF + k * kRegThreads * 16), 16, 0, 0);
      }
    }
  };
  const uint32_t rd_base = (uint32_t)(uintptr_t)(lds_ptr_t)lds + (uint32_t)(lane * ROWB) +
                           (uint32_t)(((lane / GRP) % UPR) * 16);
  // this wave's scratch slot, addressed as a buffer: SGPR descriptor, the lane's 16-byte column as
  // the VGPR offset and the [step][half] row as an SGPR / immediate offset (64-bit addresses per
  // step would cost 80 VGPRs)
  const __amdgpu_buffer_rsrc_t slot = __builtin_amdgcn_make_buffer_rsrc(
      static_cast<unsigned char*>(a.dec) + (size_t)blockIdx.x * STEPB * BLEN, 0, STEPB * BLEN, 0x00020000);
  const int col = lane * 16, colh = lane * 4 * WS;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  __shared__ uint32_t ptab[PACK ? S / 4 : 1];
  if constexpr (PACK == 1) {
    static constexpr PackedPosTable<C> kPos{};
    ptab[lane] = kPos.v[lane];
  } else if constexpr (PACK == 2) {
    static constexpr TwinPosTable<C.K> kPos{};
    ptab[lane] = kPos.v[lane];
  }

  uint32_t errors = 0;
  GroupWalk<ABLATE> walk(a, ngroups, lane, queue_hops(ABLATE));
  int g = walk.first();
  if (g < ngroups) issue_chunk(g, 0, 0);
  walk.started(g);
  for (int nxt = 0; g < ngroups; g = nxt) {
    const int b = g * kRegThreads + lane;
    float M[S];
#pragma unroll
    for (int s = 0; s < S; ++s) M[s] = s ? __builtin_inff() : 0.0f;   // viterbi-decoder.c:212-218

    // Chunk c of the group: wait for its DMA, start the next one into the other buffer, run its 8
    // steps reading each step's row one step ahead. The main chunks run as a loop over one 8-step
    // body: fully unrolled, the group is ~175 KB of code, far past the instruction cache, and the
    // waves starve on instruction fetch (2.2x slower).
    auto chunk_at = [&](int c, auto growth) __attribute__((always_inline)) {
      constexpr bool GROWTH = decltype(growth)::value;
      // this chunk's DMA was issued before the previous chunk's 16 decision stores; loads and stores
      // complete in order, so vmcnt(16) is its landing (chunks 0 and 1 follow no stores)
      if ((ABLATE & 1) == 0 && c >= 2) wait_vmcnt<16>();
      else wait_vmcnt<0>();
      // the next group from the ticket fetched a group ago: read right behind this full drain (the
      // growth chunk's), not at the last chunk, where it would drain the previous chunk's decision
      // stores that the counted vmcnt(16) leaves in flight
      if constexpr (GROWTH) {
        nxt = walk.next(g);
        walk.issued(nxt);   // the ticket after it, here too: waited by chunk 1's full drain, long back
      }
      const int buf = c & 1;
      if (c + 1 < NCH) {
        issue_chunk(g, c + 1, buf ^ 1);
      } else {   // the next group's first chunk (a harmless reload of this one's when there is none)
        issue_chunk(nxt < ngroups ? nxt : g, 0, buf ^ 1);
      }
      const uint32_t rd = rd_base + (uint32_t)(buf * BUF);
      f32x4 row = lds_read_b128<0>(rd);
      auto step_at = [&]<int u>() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(row) :: "memory");
        const float bm[4] = {row.x, row.y, row.z, row.w};
        if constexpr (u + 1 < PF) row = lds_read_b128<0>(rd ^ (uint32_t)((u + 1) * 16));
        if constexpr (GROWTH) {
          growth_step_wide<C, u>(M, bm);
        } else {
          uint32_t d[W];
          acs_step_wide<C, PACK, W>(M, bm, d);
          const int m = (c - 1) * PF + u;   // main step
          if constexpr ((ABLATE & 1) != 0) {   // timing ablation: decisions discarded
            uint32_t x = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) x ^= d[w];
            asm volatile("" ::"v"(x));
          } else {
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{d[0], d[1], d[2], d[3]}, slot, col, m * STEPB, 0);
            if constexpr (WS == 1)
              __builtin_amdgcn_raw_buffer_store_b32(d[4], slot, colh, m * STEPB + 1024, 0);
            else if constexpr (WS == 2)
              __builtin_amdgcn_raw_buffer_store_b64(u32x2{d[4], d[W > 5 ? 5 : 4]}, slot, colh, m * STEPB + 1024, 0);
            else
              __builtin_amdgcn_raw_buffer_store_b128(u32x4{d[4], d[W > 5 ? 5 : 4], d[W > 6 ? 6 : 4], d[W > 7 ? 7 : 4]},
                                                     slot, colh, m * STEPB + 1024, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      [&]<int... us>(std::integer_sequence<int, us...>) __attribute__((always_inline)) {
        (step_at.template operator()<us>(), ...);
      }(std::make_integer_sequence<int, PF>{});
    };
    static_assert(G == PF, "chunk 0 = the growth steps");
    chunk_at(0, std::true_type{});
#pragma clang loop unroll(disable)
    for (int c = 1; c < NCH; ++c) chunk_at(c, std::false_type{});

    // Traceback (reference :71-90) from the lowest-index minimum. The history word h starts as the
    // final state (its bits are the outputs of the last K-1 steps) and takes the decision of main
    // step m (the output of step m) at the bottom; its low K-1 bits are always the current state.
    float best;
    uint64_t h = argmin_wide<S>(M, best);
    // BSC input (ccv_decode_device converts its symbols to Hamming-distance rows): the path metric
    // (binary-symmetric-channel/viterbi-decoder.c:95), a small integer, exact in fp32
    if (a.path_metric && b < nb) a.path_metric[b] = (int32_t)best;
    // The decision words come back in quarters of the block, two quarters in flight: a quarter is
    // walked while the next one loads. The group's stores are drained first (vmcnt(0): L2 has
    // acknowledged them) and the loads are agent-scope (sc1), so they miss the CU's L1, which may
    // still hold this slot's lines from the previous group: the words read are the ones just stored,
    // by the memory model rather than by same-address ordering (round 4; the drain measured within
    // 1 % in round 3, profiles/r03_k9_traceback_batches.txt).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    constexpr int Q = BLEN / 4;
    static_assert(BLEN % 4 == 0, "quarters");
    uint32_t dw[2][Q][W];
    auto load_quarter = [&]<int qi>() __attribute__((always_inline)) {   // main steps qi*Q .. qi*Q+Q-1
#pragma unroll
      for (int i = 0; i < Q; ++i) {
        u32x4 lo, hi4 = {};
        u32x2 hi2 = {};
        if constexpr ((ABLATE & 2) != 0) {   // timing ablation: no decision loads
          lo = u32x4{(uint32_t)i, 1u, 2u, 3u};
          hi4 = u32x4{4u, 5u, 6u, (uint32_t)i};
          hi2 = u32x2{4u, (uint32_t)i};
          asm volatile("" : "+v"(lo), "+v"(hi4), "+v"(hi2));
        } else {
          const int m = qi * Q + i;
          constexpr int kSc1 = 16;   // cache policy: agent scope (sc1)
          lo = __builtin_amdgcn_raw_buffer_load_b128(slot, col, m * STEPB, kSc1);
          if constexpr (WS == 1) hi2 = u32x2{__builtin_amdgcn_raw_buffer_load_b32(slot, colh, m * STEPB + 1024, kSc1), 0u};
          else if constexpr (WS == 2) hi2 = __builtin_amdgcn_raw_buffer_load_b64(slot, colh, m * STEPB + 1024, kSc1);
          else hi4 = __builtin_amdgcn_raw_buffer_load_b128(slot, colh, m * STEPB + 1024, kSc1);
          if constexpr (WS == 4 && WH == 2) hi2 = u32x2{hi4.x, hi4.y};
        }
        dw[qi & 1][i][0] = lo.x; dw[qi & 1][i][1] = lo.y; dw[qi & 1][i][2] = lo.z; dw[qi & 1][i][3] = lo.w;
        if constexpr (WH == 1) {
          dw[qi & 1][i][4] = hi2.x;
        } else if constexpr (WH == 2) {
          dw[qi & 1][i][4] = hi2.x; dw[qi & 1][i][W > 5 ? 5 : 4] = hi2.y;
        } else {
          dw[qi & 1][i][4] = hi4.x; dw[qi & 1][i][W > 5 ? 5 : 4] = hi4.y;
          dw[qi & 1][i][W > 6 ? 6 : 4] = hi4.z; dw[qi & 1][i][W > 7 ? 7 : 4] = hi4.w;
        }
      }
    };
    auto walk_quarter = [&]<int qi>() __attribute__((always_inline)) {   // steps qi*Q+Q-1 .. qi*Q
#pragma unroll
      for (int i = Q - 1; i >= 0; --i) {
        const uint32_t* w = dw[qi & 1][i];
        const uint32_t st = (uint32_t)h & (S - 1);
        // where the state's decision sits: (word << 5) | bit (packed: the LDS table; AB & 32: skip it)
        const uint32_t pos = (PACK && (ABLATE & 32) == 0) ? reinterpret_cast<const uint8_t*>(ptab)[st] : st;
        const uint32_t m5 = (uint32_t)__builtin_amdgcn_sbfe((int)pos, 5, 1);   // 0 / -1 per word-index bit
        const uint32_t m6 = (uint32_t)__builtin_amdgcn_sbfe((int)pos, 6, 1);
        const uint32_t m7 = (uint32_t)__builtin_amdgcn_sbfe((int)pos, 7, 1);
        const uint32_t l0 = select_v(m5, w[1], w[0]), l1 = select_v(m5, w[3], w[2]);
        const uint32_t l2 = select_v(m5, w[W > 5 ? 5 : 4], w[4]);
        const uint32_t k0 = select_v(m6, l1, l0);
        uint32_t word;
        if constexpr (W == 5) {
          word = select_v(m7, w[4], k0);   // word 4: bit 7 set, bits 5, 6 clear
        } else if constexpr (W == 6) {
          word = select_v(m7, l2, k0);   // words 4, 5: bit 7 set, bit 6 clear
        } else {
          const uint32_t l3 = select_v(m5, w[W > 7 ? 7 : 4], w[W > 6 ? 6 : 4]);
          word = select_v(m7, select_v(m6, l3, l2), k0);
        }
        const uint32_t dbit = __builtin_amdgcn_ubfe(word, pos & 31u, 1);
        h = (h << 1) | dbit;
      }
    };
    load_quarter.template operator()<3>();
    load_quarter.template operator()<2>();
    walk_quarter.template operator()<3>();
    load_quarter.template operator()<1>();
    walk_quarter.template operator()<2>();
    load_quarter.template operator()<0>();
    walk_quarter.template operator()<1>();
    walk_quarter.template operator()<0>();
    const uint64_t bits = __builtin_bitreverse64(h);   // bit 63 - t = output of step t
    if (b < nb) {
      const uint8_t* info = a.info + (size_t)b * IB;
      uint8_t* o = a.out + (size_t)b * OB;
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
