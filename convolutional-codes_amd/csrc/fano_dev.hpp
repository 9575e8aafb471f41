// fano_dev.hpp -- the reference's Fano decoder on CDNA4, one lane per block.
//
// Reference: AWGN-channel/fano-decoder.c and binary-symmetric-channel/fano-decoder.c (KA9Q-derived
// threshold search: DELTA 17, TIMEOUT 10000 iterations per block bit, :14-15). The search follows ONE
// path through the tree, so the parallelism is across blocks: every lane runs its own search. Searches
// take wildly different numbers of iterations (a noisy block can run into the timeout while its
// neighbours finish after ~T steps), so lanes are persistent: a lane that finishes its block takes
// the next one from a global counter and the wave keeps all 64 lanes busy until the queue drains.
//
// Per lane, the node array of the reference (:17-25) shrinks to what the search reads back: the
// path metric of every node (LDS, [T][64] so same-depth accesses are conflict-free) and a flags byte
// (selected_path, decoded_input). States are re-derived on the way (forward: (s >> 1) | (in << K-2);
// back: the bit that falls out is the decoded input K nodes earlier) and transition metrics are
// recomputed for the node the search lands on -- the same values the reference stored, since a
// node's state and received symbol do not change while it is on the path.
//
// Exactness: same arithmetic (float path metrics and threshold, (float)(1.0 + w * d) branch metrics;
// int32 for BSC), same tie rules (strict < sort, >= threshold tests) and the streaming semantics of
// the oracle (oracle/ccoracle.c fano_block): the block completes when the search passes node T-1, or
// stops at the timeout with the decoded inputs left in the nodes; the BSC path metric is the metric of
// the newest received node at that moment (:195, :269).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "stack_dev.hpp"
#include "trellis.hpp"

namespace ccv {

struct FanoArgs {
  const void* in;            // soft: float [nb][T][2^n]; hard: uint8 [nb][T]
  int n, K, T, blen, gen;
  uint64_t poly[kMaxN];
  float weight;              // soft: code_param.fano_metric_weight (code.h:17)
  int32_t bm0, bm1;          // hard: code_param.fano_bit_metrics (code.h:15)
  int nblocks;
  unsigned int* next_block;  // work counter, zero before the launch
  uint8_t* out;              // [nb][OB]
  int32_t* path_metric;      // hard: may be null
  const uint8_t* info;       // optional: count bit errors
  unsigned long long* err;
  uint32_t* iterations;      // optional [nb]: search iterations used (timeout = 10000 * T)
};

constexpr int kFanoTimeoutPerBit = 10000;   // fano-decoder.c:14
constexpr int kFanoThreads = 64;

// RXL: the block's received symbols are copied into LDS ([t][k][lane]) when a lane takes the block,
// taking global-memory latency off every search step (used when they fit, see launch_fano).
template <bool HARD, int NP, bool W32, bool RXL>
__global__ __launch_bounds__(kFanoThreads) void fano_decode(FanoArgs a) {
  using MT = typename std::conditional<HARD, int32_t, float>::type;
  using ET = typename std::conditional<HARD, uint8_t, float>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int T = a.T, K = a.K, n = a.n;
  const int NS = HARD ? 1 : (1 << n);
  MT* metric = reinterpret_cast<MT*>(smem);                                    // [T][64]
  uint8_t* flags = smem + (size_t)T * kFanoThreads * sizeof(MT);              // [T][64]: sel | dec << 1
  ET* rxl = reinterpret_cast<ET*>(smem + (size_t)T * kFanoThreads * (sizeof(MT) + 1));   // [T][NS][64]
  uint64_t poly[kMaxN];
#pragma unroll
  for (int k = 0; k < kMaxN; ++k) poly[k] = a.poly[k];
  const bool idiom = a.gen == GEN_REF_X86;
  const MT delta = (MT)17;                                                     // fano-decoder.c:15
  const uint64_t smask = (1ull << (K - 1)) - 1ull;   // K <= 64
  const uint8_t symmask = (uint8_t)((1u << n) - 1u);
  const ET* in = reinterpret_cast<const ET*>(a.in);

  for (;;) {
    const unsigned int b = atomicAdd(a.next_block, 1u);
    if (b >= (unsigned int)a.nblocks) break;
    const ET* rx = in + (size_t)b * T * NS;
    if constexpr (RXL) {
      for (int i = 0; i < T * NS; ++i) rxl[i * kFanoThreads + lane] = rx[i];
    }
    // get_transition_metric + sort (:160-181, :213-236) for the node at depth d with state st:
    // tm0 >= tm1 afterwards, swapped = input 1 is the best branch
    auto node_metrics = [&](int d, uint64_t st, MT& tm0, MT& tm1, uint32_t& swapped) {
      const uint32_t es = lane_symbols<NP, W32>(poly, n, K, idiom, st);
      const uint32_t e0 = es >> 8, e1 = es & 0xFFu;
      MT t0, t1;
      if constexpr (HARD) {
        const uint32_t r = (RXL ? rxl[d * kFanoThreads + lane] : rx[d]) & symmask;
        const int32_t d0 = __builtin_popcount(e0 ^ r), d1 = __builtin_popcount(e1 ^ r);
        t0 = d0 * a.bm1 + (n - d0) * a.bm0;
        t1 = d1 * a.bm1 + (n - d1) * a.bm0;
      } else {
        float r0, r1;
        if constexpr (RXL) {
          r0 = rxl[(d * NS + (int)e0) * kFanoThreads + lane];
          r1 = rxl[(d * NS + (int)e1) * kFanoThreads + lane];
        } else {
          r0 = rx[(size_t)d * NS + e0];
          r1 = rx[(size_t)d * NS + e1];
        }
        t0 = (float)(1.0 + (double)(a.weight * r0));
        t1 = (float)(1.0 + (double)(a.weight * r1));
      }
      swapped = t0 < t1 ? 1u : 0u;
      tm0 = swapped ? t1 : t0;
      tm1 = swapped ? t0 : t1;
    };
    for (int d = 0; d < T; ++d) flags[d * kFanoThreads + lane] = 0;   // reset (:108-124)
    metric[lane] = (MT)0;
    int cur = 0, frontier = 0;
    uint64_t st = 0;            // state of node cur
    MT mcur = 0, thr = 0;
    MT tm0, tm1;
    uint32_t swapped;
    node_metrics(0, 0, tm0, tm1, swapped);
    uint32_t sel = 0, dec = swapped;
    flags[lane] = (uint8_t)(dec << 1);
    uint32_t timeout = (uint32_t)kFanoTimeoutPerBit * (uint32_t)T;
    bool done = false;
    while (timeout != 0) {
      --timeout;
      const MT ms = mcur + (sel ? tm1 : tm0);
      if (ms >= thr) {
        if (mcur < thr + delta) {   // tightening (:190-195)
          while (ms >= thr + delta) thr += delta;
        }
        // move forward along the selected branch (input = dec)
        st = (st >> 1) | ((uint64_t)dec << (K - 2));
        ++cur;
        if (cur == T) { done = true; break; }
        mcur = ms;
        metric[cur * kFanoThreads + lane] = ms;
        node_metrics(cur, st, tm0, tm1, swapped);
        sel = 0;
        dec = swapped;
        flags[cur * kFanoThreads + lane] = (uint8_t)(dec << 1);
        frontier = cur > frontier ? cur : frontier;
      } else {
        bool moved = false;
        for (;;) {
          const bool cant = cur == 0 || metric[(cur - 1) * kFanoThreads + lane] < thr;
          if (cant) {   // relax the threshold, restart from the best branch (:241-250)
            thr -= delta;
            if (sel != 0) {
              sel = 0;
              dec ^= 1u;
              flags[cur * kFanoThreads + lane] = (uint8_t)(dec << 1);
            }
            break;
          }
          // move back (:251-261): the state loses the input of node cur-1, regains that of cur-K
          const uint32_t old = cur >= K ? (flags[(cur - K) * kFanoThreads + lane] >> 1) : 0u;
          st = ((st << 1) & smask) | old;
          --cur;
          moved = true;
          const uint32_t f = flags[cur * kFanoThreads + lane];
          sel = f & 1u;
          dec = f >> 1;
          if (sel == 0) {
            sel = 1;
            dec ^= 1u;
            flags[cur * kFanoThreads + lane] = (uint8_t)(1u | (dec << 1));
            break;
          }
        }
        if (moved) {
          mcur = metric[cur * kFanoThreads + lane];
          node_metrics(cur, st, tm0, tm1, swapped);
        }
      }
    }
    // output_data (:315-325): the decoded input of every node, MSB-first
    const int OB = (T + 7) >> 3, IB = (a.blen + 7) >> 3;
    uint32_t errors = 0;
    for (int j = 0; j < OB; ++j) {
      uint32_t byte = 0;
      for (int k = 0; k < 8; ++k) {
        const int d = 8 * j + k;
        if (d < T) byte |= (uint32_t)(flags[d * kFanoThreads + lane] >> 1) << (7 - k);
      }
      a.out[(size_t)b * OB + j] = (uint8_t)byte;
      if (a.info && j < IB) {
        int valid = a.blen - 8 * j;
        valid = valid > 8 ? 8 : valid;
        const uint32_t mask = (0xFFu << (8 - valid)) & 0xFFu;
        errors += __builtin_popcount((byte ^ a.info[(size_t)b * IB + j]) & mask);
      }
    }
    if (a.err && errors) atomicAdd(a.err, (unsigned long long)errors);
    if constexpr (HARD) {
      if (a.path_metric)
        a.path_metric[b] = done ? metric[(T - 1) * kFanoThreads + lane] : metric[frontier * kFanoThreads + lane];
    }
    if (a.iterations) a.iterations[b] = (uint32_t)kFanoTimeoutPerBit * (uint32_t)T - timeout;
  }
}

}  // namespace ccv
