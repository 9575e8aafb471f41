// fano_dev.hpp -- the reference's Fano decoder on CDNA4, one lane per block.
//
// Reference: AWGN-channel/fano-decoder.c and binary-symmetric-channel/fano-decoder.c (KA9Q-derived
// threshold search: DELTA 17, TIMEOUT 10000 iterations per block bit, :14-15). The search follows ONE
// path through the tree, so the parallelism is across blocks: every lane runs its own search. Searches
// take wildly different numbers of iterations (a noisy block can run into the timeout while its
// neighbours finish after ~T steps), so lanes are persistent: a lane that finishes its block takes
// the next one from a global counter and the wave keeps all 64 lanes busy until the queue drains.
//
// Two passes. Lanes pull blocks one at a time, and search lengths are heavy-tailed (K = 15 at 4 dB:
// median 15,000 outer ticks, mean 59,000, 2.7 % run into the 10000 x T = 540,000 timeout): a lane
// commits to whatever it draws, so the kernel ends with a few lanes finishing long searches in
// nearly empty waves. Pass 1 therefore parks a search after `cap` moves -- its node path metrics and
// flags up to the frontier and its registers go to global memory -- and takes the next block; pass 2
// resumes the parked searches, one per lane, so the long tail runs side by side. A parked search
// continues from exactly the state it left, so the result is the one-pass result, bit for bit.
//
// Loop shape matters more than anything in the pass: the block switch (finish, take, start) must stay
// a branch INSIDE the one pass loop. Written as a `continue` after the switch only, the AMDGPU
// control-flow structurizer turned the round-2 kernel into a per-block inner loop in which a lane
// whose search had ended waited, exec-masked, for every other lane of its wave to end theirs (2.3x
// the time at 4 dB). With the park branch at the top of the pass the compiler keeps
// one loop.
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

#include "channel_dev.hpp"
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
  int count_moves;           // diagnostics (option "fano_count_moves"): `iterations` gets the number of
                             // moves (forward, back, threshold relaxations) instead
  unsigned long long* stats; // diagnostics (CCV_DEBUG): [0] sum over waves of loop passes,
                             // [1] sum over lanes of passes in which the lane had a search to advance
  const uint16_t* symtab;    // TAB: [2^(K-1)] expected symbols (stack_symtab_init), K <= kSymtabMaxK
  const uint32_t* order;     // optional [nb]: the queue hands out block order[q] (noisiest first)
  // Two-pass schedule (see fano_decode): pass 1 parks a search after `cap` moves (0 = never) in
  // slot atomicAdd(park_count); pass 2 (resume = 1, next_block reset) resumes the parked searches.
  uint32_t cap;
  int resume;
  unsigned int park_capacity;   // slots; a search that finds them full keeps running in pass 1
  unsigned int* park_count;
  uint32_t* park_hdr;        // [nb][kFanoParkWords]: block, cur, frontier, state, metrics, flags
  void* park_metric;         // [nb][T + 1] path metrics of the nodes 0..frontier
  uint8_t* park_flags;       // [nb][T + 1] sel | dec << 1 of the nodes 0..frontier
  int rows_mode;             // host only (ccv_plan_set_option "fano_rows"): -1 auto, else kRows*
  int iq;                    // host only (option "fano_input" 1): `in` holds the received points, float
                             // [nb][T][2] (ccv_simulate_device CCV_CHANNEL_IQ), demapped in the kernel
};

constexpr int kFanoParkWords = 12;

// Queue order for soft input (launch_fano_order): a search's length is set by the noise in its
// block, and a few blocks run into the 10000 x T timeout; handed out last, such a block holds its
// lane (and its wave) long after the queue has drained. Score = sum over steps of the distance to
// the nearest constellation point (the demapper output's minimum), sorted descending so the noisy
// blocks start first and the short ones fill in around them. Output is per block index, so the order
// changes nothing but the schedule.
template <int NS>
__global__ void fano_score(const float* in, int T, int nblocks, float* key, uint32_t* idx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const float* p = in + (size_t)b * T * NS;
  float s = 0.0f;
  for (int t = 0; t < T; ++t) {
    float m = p[t * NS];
#pragma unroll
    for (int k = 1; k < NS; ++k) m = fminf(m, p[t * NS + k]);
    s += m;
  }
  key[b] = s;
  idx[b] = (uint32_t)b;
}

// distance of the received point (x, y) to QPSK point e, as the demapper computes it (the points
// (+-a, +-a): x negative for symbol bit 1, y for bit 0 -- channel_dev.hpp's sign flips; no contraction:
// the translation unit is built with -ffp-contract=off)
__device__ __forceinline__ float qpsk_distance(float x, float y, uint32_t e) {
  constexpr const float* pts = Constellation<2>::pts;
  static_assert(pts[0] == pts[1] && pts[4] == -pts[0] && pts[3] == -pts[1], "QPSK signs");
  constexpr float ndx = pts[0] - pts[2], ndy = pts[1] - pts[3];
  constexpr float nd = (ndx * ndx) + (ndy * ndy);
  const uint32_t a = __builtin_bit_cast(uint32_t, pts[0]);
  const float px = __builtin_bit_cast(float, a ^ ((e & 2u) << 30)), py = __builtin_bit_cast(float, a ^ ((e & 1u) << 31));
  return div_const<nd>(((x - px) * (x - px)) + ((y - py) * (y - py)));
}

// The same score from received points (option "fano_input" 1): the nearest point's distance, the
// demapper's arithmetic -- the order, and so the schedule, of the distance-row input.
template <int NP = 2>   // a template: the header is in two translation units
__global__ void fano_score_iq(const float* in, int T, int nblocks, float* key, uint32_t* idx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const float2* p = reinterpret_cast<const float2*>(in) + (size_t)b * T;
  float s = 0.0f;
  for (int t = 0; t < T; ++t) {
    const float2 v = p[t];
    float m = qpsk_distance(v.x, v.y, 0u);
#pragma unroll
    for (uint32_t k = 1; k < 4; ++k) m = fminf(m, qpsk_distance(v.x, v.y, k));
    s += m;
  }
  key[b] = s;
  idx[b] = (uint32_t)b;
}

constexpr int kFanoTimeoutPerBit = 10000;   // fano-decoder.c:14

// (Round 5 measured and removed a node-flag form with two 64-bit masks per lane instead of a byte
// per node in LDS: 9 -> 11 waves per CU at K = 15, but the mask updates cost more than the occupancy
// gained -- 67 -> 60 Mbit/s soft, 222 -> 218 BSC, profiles/r05c/ab/fanoreg*.)
constexpr int kFanoThreads = 64;
// LDS bytes of the node arrays (metrics [T + 1][64] + a flags byte per node), 16-byte aligned; the
// rows follow. (Round 5 measured 2-bit packed flags -- 9 -> 10 waves per CU, updates by two LDS
// atomics: 67.3 -> 64.5 Mbit/s soft, 217 -> 209 BSC, profiles/r05_fano/.)
__host__ __device__ constexpr size_t fano_node_bytes(int T, size_t metric_bytes) {
  return ((size_t)(T + 1) * kFanoThreads * (metric_bytes + 1) + 15) & ~(size_t)15;
}

// Received-symbol access per lane (RM):
//   kRowsDirect: the branch metrics of the node a move lands on read r[e] from global memory after
//     the move is decided (any code).
//   kRowsGlobal: each pass first issues the loads of the two rows a move can land on (cur - 1,
//     cur + 1) and the lane keeps its own node's row in registers, so the load latency overlaps the
//     pass instead of following it (hard input or rate 1/2: a row is a byte or a float4).
//   kRowsLds: as kRowsGlobal, the block's rows copied into LDS when the lane takes the block; the two
//     rows are read as soon as the previous pass has decided its move (round 6).
// (Round 5 measured and removed a register window of rows cur - 1, cur, cur + 1 with one load per
// move issued a pass ahead: 67 -> 48 Mbit/s soft, 222 -> 156 BSC, profiles/r05b/.)
//   kRowsIQ / kRowsIQLds (round 6, soft rate 1/2, option "fano_input" 1): the rows are the received
//     points (x, y) -- 8 instead of 16 bytes per node -- from global memory as kRowsGlobal, or in LDS;
//     the two branch metrics are the demapper's distances recomputed with its exact fp32 operations
//     (common/demapper.c:66-70 as channel_dev.hpp ChannelSource::compute): the same decoder input bit
//     for bit, for frames the on-device channel produced (a drop-in caller's input IS the distances).
constexpr int kRowsDirect = 0, kRowsGlobal = 2, kRowsLds = 1, kRowsIQ = 3, kRowsIQLds = 4;
constexpr bool rows_iq(int rm) { return rm == kRowsIQ || rm == kRowsIQLds; }
template <bool HARD, int NP, bool IQ = false>
struct FanoRow;
template <int NP>
struct FanoRow<true, NP> {
  uint32_t v;
  // component-wise select: a select of whole structs becomes a private-memory copy
  __device__ void pick(bool a, const FanoRow& ra, bool b, const FanoRow& rb) {
    v = a ? ra.v : (b ? rb.v : v);
  }
};
template <int NP>
struct FanoRow<false, NP, true> {
  float2 v;
  __device__ void pick(bool a, const FanoRow& ra, bool b, const FanoRow& rb) {
    v.x = a ? ra.v.x : (b ? rb.v.x : v.x);
    v.y = a ? ra.v.y : (b ? rb.v.y : v.y);
  }
};
template <int NP>
struct FanoRow<false, NP, false> {
  float4 v;
  __device__ void pick(bool a, const FanoRow& ra, bool b, const FanoRow& rb) {
    v.x = a ? ra.v.x : (b ? rb.v.x : v.x);
    v.y = a ? ra.v.y : (b ? rb.v.y : v.y);
    v.z = a ? ra.v.z : (b ? rb.v.z : v.z);
    v.w = a ? ra.v.w : (b ? rb.v.w : v.w);
  }
};

// One lane, one search. The reference's loop (:183-263) is an outer iteration (one timeout tick:
// try the selected branch, move forward or start looking back) with an inner loop of backward moves.
// Here every pass of the kernel loop is ONE move -- forward, one step back, or a threshold
// relaxation -- so all lanes of a wave stay in the same code whatever phase their searches are in,
// and the branch metrics of the node a lane lands on are computed by one shared piece of code.
// TAB: the node's expected symbols are one cached load from the per-plan table (stack_dev.hpp,
// stack_symtab_init) instead of ~25 VALU of parities per pass.
template <bool HARD, int NP, bool W32, int RM, bool TAB = false>
__global__ __launch_bounds__(kFanoThreads) void fano_decode(FanoArgs a) {
  static_assert(!TAB || (W32 && NP != 0), "the table covers specialised K <= 32 codes");
  using MT = typename std::conditional<HARD, int32_t, float>::type;
  using ET = typename std::conditional<HARD, uint8_t, float>::type;
  using ST = typename std::conditional<W32, uint32_t, uint64_t>::type;
  static_assert(RM == kRowsDirect || HARD || NP == 2, "rows of received symbols are a byte or a float4");
  static_assert(!rows_iq(RM) || (!HARD && NP == 2), "received points: soft rate 1/2");
  constexpr bool ROWS = RM != kRowsDirect;
  constexpr bool IQ = rows_iq(RM);
  constexpr bool LDSROWS = RM == kRowsLds || RM == kRowsIQLds;
  using Row = FanoRow<HARD, NP, IQ>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int T = a.T, K = a.K, n = a.n;
  const int NS = HARD ? 1 : (IQ ? 2 : (1 << n));   // input floats per node
  // node arrays [T + 1][64]; row T takes the stores a lane does not need
  MT* metric = reinterpret_cast<MT*>(smem);
  uint8_t* flags = smem + (size_t)(T + 1) * kFanoThreads * sizeof(MT);   // sel | dec << 1
  // rows: [T][64] float4 / float2 (soft) or bytes (hard), after the flags (16-byte aligned)
  unsigned char* rows = smem + fano_node_bytes(T, sizeof(MT));
  // a node's flags byte (sel | dec << 1)
  auto flag_get = [&](int d) -> uint32_t { return flags[d * kFanoThreads + lane]; };
  // store v at node d when `write`; otherwise into the spare row T (branch-free)
  auto flag_put = [&](bool write, int d, uint32_t v) { flags[(write ? d : T) * kFanoThreads + lane] = (uint8_t)v; };
  uint64_t poly[kMaxN];
#pragma unroll
  for (int k = 0; k < kMaxN; ++k) poly[k] = a.poly[k];
  const bool idiom = a.gen == GEN_REF_X86;
  const MT delta = (MT)17;                                                     // fano-decoder.c:15
  const ST smask = (ST)((1ull << (K - 1)) - 1ull);   // K <= 64
  const uint32_t symmask = (1u << n) - 1u;
  const ET* in = reinterpret_cast<const ET*>(a.in);
  const int OB = (T + 7) >> 3, IB = (a.blen + 7) >> 3;
  const uint32_t budget = (uint32_t)kFanoTimeoutPerBit * (uint32_t)T;

  const ET* rx = nullptr;
  auto row_at = [&](int d) {
    Row r;
    if constexpr (LDSROWS) {
      if constexpr (HARD) r.v = rows[d * kFanoThreads + lane];
      else if constexpr (IQ) r.v = reinterpret_cast<const float2*>(rows)[d * kFanoThreads + lane];
      else r.v = reinterpret_cast<const float4*>(rows)[d * kFanoThreads + lane];
    } else {
      if constexpr (HARD) r.v = rx[d];
      else if constexpr (IQ) r.v = reinterpret_cast<const float2*>(rx)[d];
      else r.v = reinterpret_cast<const float4*>(rx)[d];
    }
    return r;
  };
  // get_transition_metric + sort (:160-181, :213-236) for the node at depth d with state st, whose
  // received row is `row` (ROWS): tm0 >= tm1 afterwards, swapped = input 1 is the best branch
  auto node_metrics = [&](const ET* rx, int d, ST st, const Row& row, MT& tm0, MT& tm1,
                          uint32_t& swapped) {
    uint32_t es;
    if constexpr (TAB) es = a.symtab[(uint32_t)st];
    else es = lane_symbols<NP, W32>(poly, n, K, idiom, (uint64_t)st);
    const uint32_t e0 = es >> 8, e1 = es & 0xFFu;
    MT t0, t1;
    if constexpr (HARD) {
      const uint32_t r = (ROWS ? row.v : (uint32_t)rx[d]) & symmask;
      const int32_t d0 = __builtin_popcount(e0 ^ r), d1 = __builtin_popcount(e1 ^ r);
      t0 = d0 * a.bm1 + (n - d0) * a.bm0;
      t1 = d1 * a.bm1 + (n - d1) * a.bm0;
    } else {
      float r0, r1;
      if constexpr (IQ) {   // the demapper's two distances from the received point
        r0 = qpsk_distance(row.v.x, row.v.y, e0);
        r1 = qpsk_distance(row.v.x, row.v.y, e1);
      } else if constexpr (ROWS || NP == 2) {   // rate 1/2: the node's whole row is one 16-byte load
        const float4 v = ROWS ? row.v : reinterpret_cast<const float4*>(rx)[d];
        r0 = (e0 & 2u) ? ((e0 & 1u) ? v.w : v.z) : ((e0 & 1u) ? v.y : v.x);
        r1 = (e1 & 2u) ? ((e1 & 1u) ? v.w : v.z) : ((e1 & 1u) ? v.y : v.x);
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

  // per-lane search state
  // the next block from the queue (through the noisiest-first order when there is one), or in the
  // resume pass the next parked search
  unsigned int b = 0, slot = 0;
  unsigned int parked = 0;   // final: pass 1 has completed
  if (a.resume) parked = *a.park_count < a.park_capacity ? *a.park_count : a.park_capacity;
  auto take = [&]() -> bool {
    const unsigned int q = atomicAdd(a.next_block, 1u);
    if (a.resume) {
      if (q >= parked) return false;
      slot = q;
      b = a.park_hdr[(size_t)q * kFanoParkWords];
      return true;
    }
    if (q >= (unsigned int)a.nblocks) return false;
    b = a.order ? a.order[q] : q;
    return true;
  };
  const bool first = take();
  int cur = 0, frontier = 0;
  ST st = 0;
  MT mcur = 0, thr = 0, tm0 = 0, tm1 = 0;
  uint32_t sel = 0, dec = 0, timeout = 0;
  bool inback = false, moved = false;
  uint32_t moves = 0, spass = 0;
  Row row0{};   // received row of node cur
  // the rows of nodes cur - 1 and cur + 1, where this pass's move can land. Rows in LDS: read as soon
  // as the previous pass has decided its move, so their latency overlaps the rest of that pass too
  // (round 6, BSC 212 -> 232 Mbit/s); rows in global memory: at the top of the pass (the early form
  // measured 1-1.6 % slower there, profiles/r06_fano_early/)
  constexpr bool EARLY = LDSROWS;
  Row rowm{}, rowp{};
  auto prefetch_rows = [&](int c) {
    if constexpr (ROWS && EARLY) {
      rowm = row_at(c > 0 ? c - 1 : 0);
      rowp = row_at(c + 1 < T ? c + 1 : T - 1);
    }
  };
  auto as_bits = [](MT v) -> uint32_t {
    if constexpr (HARD) return (uint32_t)v;
    else return __float_as_uint(v);
  };
  auto from_bits = [](uint32_t v) -> MT {
    if constexpr (HARD) return (MT)(int32_t)v;
    else return __uint_as_float(v);
  };
  // the search at the queue head parks its whole state (the node path metrics and flags up to the
  // frontier -- the nodes it can read back -- and the registers) for the resume pass
  auto park = [&]() -> bool {
    const unsigned int k = atomicAdd(a.park_count, 1u);
    if (k >= a.park_capacity) return false;
    uint32_t* h = a.park_hdr + (size_t)k * kFanoParkWords;
    MT* pm = static_cast<MT*>(a.park_metric) + (size_t)k * (T + 1);
    uint8_t* pf = a.park_flags + (size_t)k * (T + 1);
    for (int d = 0; d <= frontier; ++d) {
      pm[d] = metric[d * kFanoThreads + lane];
      pf[d] = (uint8_t)flag_get(d);
    }
    h[0] = b;
    h[1] = (uint32_t)cur;
    h[2] = (uint32_t)frontier;
    h[3] = (uint32_t)(uint64_t)st;
    h[4] = (uint32_t)((uint64_t)st >> 32);
    h[5] = as_bits(mcur);
    h[6] = as_bits(thr);
    h[7] = as_bits(tm0);
    h[8] = as_bits(tm1);
    h[9] = sel | (dec << 1) | ((inback ? 1u : 0u) << 2) | ((moved ? 1u : 0u) << 3);
    h[10] = timeout;
    h[11] = moves;
    return true;
  };
  auto load_rows = [&]() {
    rx = in + (size_t)b * T * NS;
    if constexpr (LDSROWS) {
      if constexpr (HARD) {
        for (int d = 0; d < T; ++d) rows[d * kFanoThreads + lane] = rx[d];
      } else if constexpr (IQ) {
        const float2* src = reinterpret_cast<const float2*>(rx);
        float2* dst = reinterpret_cast<float2*>(rows);
        for (int d = 0; d < T; ++d) dst[d * kFanoThreads + lane] = src[d];
      } else {
        const float4* src = reinterpret_cast<const float4*>(rx);
        float4* dst = reinterpret_cast<float4*>(rows);
        for (int d = 0; d < T; ++d) dst[d * kFanoThreads + lane] = src[d];
      }
    }
  };
  // resume a parked search exactly where pass 1 left it
  auto restore = [&]() {
    load_rows();
    const uint32_t* h = a.park_hdr + (size_t)slot * kFanoParkWords;
    cur = (int)h[1];
    frontier = (int)h[2];
    const MT* pm = static_cast<const MT*>(a.park_metric) + (size_t)slot * (T + 1);
    const uint8_t* pf = a.park_flags + (size_t)slot * (T + 1);
    for (int d = 0; d <= frontier; ++d) {
      metric[d * kFanoThreads + lane] = pm[d];
      flag_put(true, d, pf[d]);
    }
    st = (ST)((uint64_t)h[3] | ((uint64_t)h[4] << 32));
    mcur = from_bits(h[5]);
    thr = from_bits(h[6]);
    tm0 = from_bits(h[7]);
    tm1 = from_bits(h[8]);
    sel = h[9] & 1u;
    dec = (h[9] >> 1) & 1u;
    inback = (h[9] & 4u) != 0;
    moved = (h[9] & 8u) != 0;
    timeout = h[10];
    moves = h[11];
    spass = 0;
    if constexpr (ROWS) row0 = row_at(cur);
    prefetch_rows(cur);
  };
  // start a search (:108-124 reset, then the root's branch metrics)
  auto start = [&]() {
#ifndef CCV_FANO_NO_PARK
    if (a.resume) {
      restore();
      return;
    }
#endif
    load_rows();
    spass = 0;
    if constexpr (ROWS) row0 = row_at(0);
    prefetch_rows(0);
    metric[lane] = (MT)0;
    cur = 0;
    frontier = 0;
    st = 0;
    mcur = 0;
    thr = 0;
    uint32_t sw;
    node_metrics(rx, 0, 0, row0, tm0, tm1, sw);
    sel = 0;
    dec = sw;
    flag_put(true, 0, dec << 1);
    timeout = budget;
    inback = false;
    moves = 0;
  };
  // output_data (:315-325): the decoded input of every node, MSB-first; nodes past the frontier
  // were never visited and still hold the reset value 0
  auto finish = [&](bool done) {
    uint32_t errors = 0;
    for (int j = 0; j < OB; ++j) {
      uint32_t byte = 0;
      for (int k = 0; k < 8; ++k) {
        const int d = 8 * j + k;
        if (d <= frontier && d < T) byte |= (flag_get(d) >> 1) << (7 - k);
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
      // the metric of the newest received node (:195, :269): the last node when done
      if (a.path_metric) a.path_metric[b] = metric[(done ? T - 1 : frontier) * kFanoThreads + lane];
    }
    if (a.iterations) a.iterations[b] = a.count_moves ? moves : budget - timeout;
  };

  uint32_t lane_passes = 0;
  if (first) {
  start();
  // One move per pass, computed without branches (a lone lane's search is latency-bound and every
  // taken branch costs the wave an instruction-fetch bubble); stores that a lane does not need go
  // to the spare node row T.
  for (;;) {
    ++lane_passes;
#ifndef CCV_FANO_NO_PARK
    if (__builtin_expect(a.cap != 0 && spass == a.cap, 0)) {   // a long search: resumed in pass 2
      if (park()) {
        if (!take()) break;
        start();
        continue;
      }
    }
#endif
    ++spass;
    // everything a backward move can read, fetched before the move is decided
    const int cm = cur > 0 ? cur - 1 : 0;
    const MT mprev = metric[cm * kFanoThreads + lane];
    const uint32_t fprev = flag_get(cm);
    const uint32_t fold = flag_get(cur >= K ? cur - K : 0);
    if constexpr (ROWS && !EARLY) {
      rowm = row_at(cm);
      rowp = row_at(cur + 1 < T ? cur + 1 : T - 1);
    }
    // outer iteration (:183-196): one timeout tick, try the selected branch
    const bool outer = !inback;
    const bool expired = outer && timeout == 0;
    const bool tick = outer && timeout != 0;
    timeout -= tick ? 1u : 0u;
    const MT ms = mcur + (sel ? tm1 : tm0);
    const bool fwd = tick && ms >= thr;
    if (fwd && mcur < thr + delta) {   // tightening (:190-195)
      while (ms >= thr + delta) thr += delta;
    }
    // look back (:237-263): one step per pass
    const bool entering = tick && !fwd;
    const bool was_moved = entering ? false : moved;
    const bool looking = entering || inback;
    const bool cant = cur == 0 || mprev < thr;
    const bool relax = looking && cant;   // relax the threshold, restart from the best branch
    const bool bstep = looking && !cant;  // move back to node cur-1
    const bool untried = (fprev & 1u) == 0u;   // node cur-1 has not tried its second branch yet
    thr = relax ? thr - delta : thr;
    const ST st_f = (ST)((st >> 1) | ((ST)dec << (K - 2)));
    const ST st_b = (ST)(((st << 1) & smask) | (ST)(cur >= K ? (fold >> 1) : 0u));
    st = fwd ? st_f : (bstep ? st_b : st);
    const int ncur = cur + (fwd ? 1 : 0) - (bstep ? 1 : 0);
    const bool flip = relax && sel != 0;
    // sel/dec of the node the lane is on afterwards (forward: dec set from its branch metrics below)
    dec = bstep ? ((fprev >> 1) ^ (untried ? 1u : 0u)) : (dec ^ (flip ? 1u : 0u));
    sel = bstep ? 1u : ((fwd || relax) ? 0u : sel);
    mcur = fwd ? ms : (bstep ? mprev : mcur);
    inback = bstep && !untried;
    moved = bstep || was_moved;
    const bool need = fwd || (relax && was_moved) || (bstep && untried);
    moves += (fwd || relax || bstep) ? 1u : 0u;
    frontier = fwd && ncur > frontier ? ncur : frontier;
    cur = ncur;
    if (__builtin_expect(expired || (fwd && ncur == T), 0)) {
      finish(!expired);
      if (!take()) break;
      start();
      continue;
    }
    Row nextm{}, nextp{};   // the next pass's candidate rows, issued right away (EARLY)
    if constexpr (ROWS && EARLY) {
      nextm = row_at(ncur > 0 ? ncur - 1 : 0);
      nextp = row_at(ncur + 1 < T ? ncur + 1 : T - 1);
    }
    metric[(fwd ? ncur : T) * kFanoThreads + lane] = ms;
    if constexpr (ROWS) row0.pick(fwd, rowp, bstep, rowm);
    MT n0, n1;
    uint32_t sw;
    node_metrics(rx, ncur, st, row0, n0, n1, sw);
    if constexpr (ROWS && EARLY) {
      rowm = nextm;
      rowp = nextp;
    }
    tm0 = need ? n0 : tm0;
    tm1 = need ? n1 : tm1;
    dec = fwd ? sw : dec;
    const bool wflag = fwd || flip || (bstep && untried);
    flag_put(wflag, ncur, (bstep ? 1u : 0u) | (dec << 1));
  }
  }
  if (a.stats) {   // all lanes again (those without a block skipped the loop)
    const int32_t wave_passes = wave_max((int32_t)lane_passes);
    if (lane == 0) atomicAdd(&a.stats[0], (unsigned long long)wave_passes);
    atomicAdd(&a.stats[1], (unsigned long long)lane_passes);
  }
}

}  // namespace ccv
