// acs_persist.hpp -- persistent register-trellis Viterbi kernels for K <= 7 (gfx950).
//
// Same trellis arithmetic as acs_reg.hpp (one lane = one block, all 2^(K-1) metrics in VGPRs, the ACS
// of AWGN-channel/viterbi-decoder.c:108-141 / binary-symmetric-channel/viterbi-decoder.c:114-150 in
// closed form), restructured around three measured costs of viterbi_soft_regdec
// (profiles/r02_pmc_icache_baseline.txt: its waves issue VALU in only 67 % of their lifetime):
//
//  * Growth steps. Every block starts from the reset metrics (0 for state 0, +inf / 0xFF00 elsewhere,
//    viterbi-decoder.c:212-218 / :222-232), so during the first K-1 steps only the multiples of
//    2^(K-2-t) are reachable after step t, and each of them has exactly one finite candidate -- the
//    even predecessor s0 -- because the odd one is still unreachable. The reference keeps s0 on that
//    compare (m1 = inf is not < m0), so those steps are ONE add per reachable state with decision 0:
//    126 adds instead of 6 x 64 full ACS at K=7, no decision registers, and the unreachable metrics
//    are compile-time constants. (Finite inputs; with +-inf or NaN in the input the reference itself
//    traces back through stale state-matrix entries.)
//  * No padding, no guards. The kernels are specialised on the block length (the codebook's 40 for
//    every Viterbi code, common/codebook.c:66-68): chunks are aligned to the block start and every
//    step, chunk and decision register is static. Other lengths use viterbi_soft_regdec /
//    viterbi_hard_reg.
//  * Persistent waves. The grid holds exactly the resident waves; each walks groups of 64 blocks
//    g, g + grid, ... and the LDS-DMA of the NEXT group's first chunk is issued at the start of the
//    current group's last chunk, so no wave ever waits for a cold first load and no SIMD idles
//    between short-lived waves.
//
// Survivor decisions of the main steps stay in VGPRs (two 32-bit words per step at K=7), the
// traceback (reference :71-90 / :75-96) walks them back from the lowest-index minimum, then the
// growth steps (decision 0), and writes the reference's MSB-first output buffer (tail included).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <mutex>
#include <utility>
#include <vector>

#include "acs_reg.hpp"
#include "twins.hpp"

namespace ccv {

constexpr int kPersistMaxMain = 48;   // main (post-growth) steps with register-resident decisions

// Materialise a decision word where it is produced. Its only use is the traceback, so without this
// the compiler sinks the whole decision packing there and keeps every raw m1 - m0 alive across the
// block (hundreds of VGPRs, thousands of spills).
template <typename DW>
__device__ __forceinline__ void pin(DW& d) {
  asm volatile("" : "+v"(d));
}

// ACS step in full-rate instructions only (soft decision): per new state d = m1 - m0 (v_sub),
// mask = d >> 31 arithmetic (v_ashrrev), survivor = mask ? m1 : m0 (v_bitop3 select), and the
// decision bit OR-ed into its fixed position of the word (mask & bit, merged by the compiler for
// states whose masks are the same value). Same decisions and metrics as acs_step: mask = sign of
// m1 - m0, the survivor is m1 exactly when m1 < m0 (metrics are never -0; see acs_step).
__device__ __forceinline__ uint32_t sign_mask(float a0, float a1) {
  float d;
  asm("v_sub_f32 %0, %1, %2" : "=v"(d) : "v"(a1), "v"(a0));
  uint32_t m;
  asm("v_ashrrev_i32 %0, 31, %1" : "=v"(m) : "v"(d));
  return m;
}
__device__ __forceinline__ float select_mask(uint32_t m, float a0, float a1) {
  float n;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(n) : "v"(m), "v"(a1), "v"(a0));   // m ? a1 : a0
  return n;
}

template <CodeSpec C>
__device__ __forceinline__ DecWord<(1 << (C.K - 1))> acs_step_select(float (&M)[1 << (C.K - 1)],
                                                                     const float (&BM)[1 << C.n]) {
  constexpr int S = 1 << (C.K - 1);
  constexpr int H = S / 2;
  constexpr int W = S > 32 ? 2 : 1;
  float N[S];
  uint32_t dw[W] = {};
#pragma unroll
  for (int j = 0; j < H; ++j) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float m0 = M[2 * j] + BM[expected_symbol(C, 2 * j, i)];
      const float m1 = M[2 * j + 1] + BM[expected_symbol(C, 2 * j + 1, i)];
      const uint32_t mask = sign_mask(m0, m1);
      const int ns = j + i * H;
      N[ns] = select_mask(mask, m0, m1);
      dw[ns / 32] |= mask & (1u << (ns % 32));
    }
  }
#pragma unroll
  for (int s = 0; s < S; ++s) M[s] = N[s];
  if constexpr (S > 32) return ((uint64_t)dw[1] << 32) | dw[0];
  else return dw[0];
}

// Growth step t (0 <= t < K-1) from the reset metrics: new state ns is reachable iff it is a
// multiple of 2^(K-2-t); its only finite candidate is M[s0] + bm(s0, i).
template <CodeSpec C, int t, typename MT>
__device__ __forceinline__ void growth_step(MT (&M)[1 << (C.K - 1)], const MT (&BM)[1 << C.n],
                                            MT unreachable) {
  constexpr int S = 1 << (C.K - 1);
  constexpr int H = S / 2;
  constexpr int stride = 1 << (C.K - 2 - t);
  MT N[S];
#pragma unroll
  for (int ns = 0; ns < S; ++ns) {
    if (ns % stride == 0) {
      const int i = ns >> (C.K - 2);
      const int s0 = 2 * (ns & (H - 1));
      N[ns] = M[s0] + BM[expected_symbol(C, s0, i)];
    } else {
      N[ns] = unreachable;
    }
  }
#pragma unroll
  for (int s = 0; s < S; ++s) M[s] = N[s];
}

// Traceback over register decisions D[0 .. F-1] (main steps, F = blen), then the K-1 growth steps (decision
// 0 on every path through them). Returns the T decoded bits MSB-aligned: bit 63 = step 0.
// F_rt == F at run time: the per-8-step guards only cut the code into basic blocks (a fully
// straight-line kernel makes the register allocator spill thousands of VGPRs; see acs_persist notes).
// The output bit of step t is the top bit of the state there, and walking back shifts each decision in
// at the bottom of the state: so the output bits of steps T-1 .. 0 are the final state's K-1 bits
// followed by the decisions read at main steps F-1 .. 0, and one history word h (low K-1 bits = the
// current state) carries the whole traceback: d = D[m] >> (h mod S) (for K = 6, 7 the mask is the
// shifter's own), h = (h << 1) | (d & 1) -- three VALU ops per step. The history
// outgrows 32 bits after 33 - K steps: the word is saved then and the walk continues in the low bits.
template <int K, typename DW, int F>
__device__ __forceinline__ uint64_t traceback_regs(const DW (&D)[F], uint32_t st, int F_rt) {
  constexpr int S = 1 << (K - 1);
  constexpr int T = F + K - 1;
  static_assert(T <= 64, "history fits two words");
  constexpr int SPLIT = 33 - K;   // main steps after which h holds 32 bits
  uint32_t h = st, hi = 0;
#pragma unroll
  for (int j = 0; j < F; ++j) {
    const int m = F - 1 - j;
    if (m % 8 == 7 || m == F - 1) {
      if (m >= F_rt) continue;
    }
    const uint32_t d = (uint32_t)(D[m] >> (h & (S - 1)));   // the mask folds into the shifter
    h = (h << 1) | (d & 1u);
    if (j + 1 == SPLIT) hi = h;
  }
  // bit i of H = output of step i
  uint64_t H;
  if constexpr (F <= SPLIT) H = h;
  else H = ((uint64_t)hi << (F - SPLIT)) | (h & ((1u << (F - SPLIT)) - 1u));
  return __builtin_bitreverse64(H);   // bit 63 - t = output of step t
}

// One stored decision per value-numbering class (twins.hpp, generated by tools/gen_twins.py) for the
// x86-idiom K = 7 / K = 9 codes: states whose candidate pairs are the same expressions share their
// decision at every main step, so only each class's first state in processing order (butterfly j
// descending, state j then j + S/2) shifts its decision in, at the class's position.
template <CodeSpec C>
constexpr bool twin_code() {
  if constexpr (C.K == 7 || C.K == 9)
    return C.n == 2 && C.gen == GEN_REF_X86 && C.poly[0] == TwinTable<C.K>::polys[0] &&
           C.poly[1] == TwinTable<C.K>::polys[1];
  else
    return false;
}

// Output bytes (MSB-first, reference traceback :88) and the bit errors of the first blen bits
// against the transmitted info bytes (consumer AWGN-channel/main.c:118-144). Static sizes: runtime
// byte loops here cost the persistent kernels their register allocation (spills).
template <int T>
__device__ __forceinline__ void store_block(const RegArgs& a, int b, uint64_t bits) {
  constexpr int OB = (T + 7) >> 3;
  uint8_t* o = a.out + (size_t)b * OB;
#pragma unroll
  for (int k = 0; k < OB; ++k) o[k] = (uint8_t)(bits >> (56 - 8 * k));
}
template <int BLEN>
__device__ __forceinline__ uint32_t block_errors(const RegArgs& a, uint64_t bits, uint64_t ref) {
  if (a.info == nullptr) return 0;
  constexpr uint64_t mask = BLEN >= 64 ? ~0ull : ~(~0ull >> BLEN);
  return (uint32_t)__builtin_popcountll((bits ^ ref) & mask);
}
template <int T, int BLEN>
__device__ __forceinline__ uint32_t emit_block(const RegArgs& a, int b, uint64_t bits, uint64_t ref) {
  store_block<T>(a, b, bits);
  return block_errors<BLEN>(a, bits, ref);
}

// The block's transmitted info bytes, MSB-aligned (bit 63 = info bit 0), or 0 without error counting.
template <int BLEN>
__device__ __forceinline__ uint64_t load_info(const RegArgs& a, int b) {
  constexpr int IB = (BLEN + 7) >> 3;
  if (a.info == nullptr) return 0;
  const uint8_t* p = a.info + (size_t)b * IB;
  uint64_t ref = 0;
#pragma unroll
  for (int k = 0; k < IB; ++k) ref |= (uint64_t)p[k] << (56 - 8 * k);
  return ref;
}

// ------------------------------------------------------------------------------------------------
// Group schedule. Round 1-5 kernels walked g, g + grid, ... (a static share per wave). The waves of a
// SIMD do not progress alike: VALU issue is arbitrated by age, so the oldest wave runs nearly
// unimpeded and the youngest gets the leftover slots; with equal static shares the youngest sets the
// kernel length (round-5 PMC: waves resident 0.87 of the headline kernel's cycles, 0.69 of the BSC
// K = 7 kernel's at 3 waves per SIMD). With the queue (kPersistQueue) every wave starts on one static
// group and then takes the next free group: a wave that progresses faster simply decodes more groups.
//
// One head per XCD label (blockIdx.x % 8: the workgroups of a label share an XCD under the
// round-robin placement; speed only, never correctness) over a contiguous eighth of the groups, on
// 128-byte lines of their own: 40,625 groups per 0.5 ms would be ~81 dequeues/us on one word, at its
// measured ceiling (~88/us, MI355X_MICROARCH.md "dequeue"); eight heads take ~10/us each. A label whose
// range is exhausted steals from the next labels in turn. Tickets are agent-scope atomics (performed
// at the memory side, coherent across XCDs) from lane 0, fetched one group AHEAD so their latency
// (~1-3 us) hides behind a whole group's work; only the steals at the very end are synchronous.
// The queue is self-resetting: every wave adds 1 to the exit word after its last ticket, and the wave
// that adds last (it has seen grid - 1) zeroes the heads and the exit word, so the next launch on the
// stream starts from zeros (graph replays included). A plan's launches are stream-ordered, as for
// its other scratch.
constexpr int kQueueLabels = 8;
constexpr int kQueueStride = 32;                                  // u32 words per head: 128 B
constexpr int kQueueWords = (kQueueLabels + 1) * kQueueStride;   // heads + the exit word
constexpr int kStampWords = 8;                                    // diagnostic stamps per wave

struct GroupQueue {
  uint32_t* q;
  int ngroups, grid, label;
  __device__ __forceinline__ int lo(int x) const {
    return (int)((long long)x * ngroups / kQueueLabels);
  }
  // statically assigned groups of label x: its waves' first groups (blocks x, x + 8, ...)
  __device__ __forceinline__ int nstatic(int x) const {
    const int waves = grid > x ? (grid - x + kQueueLabels - 1) / kQueueLabels : 0;
    const int range = lo(x + 1) - lo(x);
    return waves < range ? waves : range;
  }
  // ticket from head x: lane 0 draws it, the caller reads it with read_lane(t, 0). The address carries
  // an opaque zero VGPR: on a uniform address the compiler's atomic optimizer rewrites the fetch into
  // its per-lane form (mbcnt + readfirstlane of the result), which waits for the atomic right there.
  // (A snapshot of the other heads in the same instruction -- lanes 1..7 adding 0 -- multiplies the
  // atomic traffic per head by 8, past one word's ~88/us ceiling: 1.27-1.46x the static walk's time,
  // profiles/r06b.)
  // (Leaving the other lanes' t undefined instead of 0 -- the zero's v_mov into the register the
  // previous fetch returned into makes hipCC drain the stores in flight first, inside the K = 9
  // kernels' chunk loop -- let the optimizer break the kernels: wrong outputs, profiles/r06_tail/r06j.)
  __device__ __forceinline__ uint32_t fetch(int x, int lane) const {
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    uint32_t t = 0;
    if (lane == 0)
      t = __hip_atomic_fetch_add(q + x * kQueueStride + z, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return t;
  }
  // ticket t of head qx -> group (wave-uniform). Every label's own waves drain its head (the queue is
  // only used with a wave on every label, grid >= 8); an exhausted head sends the wave to the next
  // label's head for at most `hops` synchronous tickets (balancing between XCDs, the tail only).
  // ngroups when done. `syncs` counts the synchronous tickets.
  __device__ __forceinline__ int resolve(uint32_t t, int& qx, int lane, uint32_t& syncs, int hops) const {
    int grp = lo(qx) + nstatic(qx) + (int)read_lane(t, 0);
    while (grp >= lo(qx + 1)) {
      if ((qx - label + kQueueLabels) % kQueueLabels >= hops) return ngroups;
      qx = (qx + 1) % kQueueLabels;
      ++syncs;
      grp = lo(qx) + nstatic(qx) + (int)read_lane(fetch(qx, lane), 0);
    }
    return grp;
  }
  __device__ __forceinline__ int first(int lane, int& qx, uint32_t& syncs, int hops) const {
    const int j = blockIdx.x / kQueueLabels;
    if (j < lo(label + 1) - lo(label)) return lo(label) + j;
    return resolve(fetch(qx, lane), qx, lane, syncs, hops);
  }
  // lane i of a fetch as a wave-uniform value. Inline asm: the builtin readfirstlane of a loop-carried
  // ticket is pushed into the predecessors by the compiler, i.e. right behind the fetch, with a
  // vmcnt(0) wait for the atomic there -- the latency the look-ahead exists to hide.
  __device__ __forceinline__ static uint32_t read_lane(uint32_t t, int i) {
    uint32_t r;
    asm volatile("v_readlane_b32 %0, %1, %2" : "=s"(r) : "v"(t), "s"(i));
    return r;
  }
  // after the wave's last ticket: the last wave out zeroes the queue for the next launch
  __device__ __forceinline__ void exit(int lane) const {
    if (lane == 0) {
      uint32_t* done = q + kQueueLabels * kQueueStride;
      const uint32_t d = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == (uint32_t)grid - 1) {
#pragma unroll
        for (int x = 0; x <= kQueueLabels; ++x)
          __hip_atomic_exchange(q + x * kQueueStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
};

// The group walk of a persistent kernel as one object (the K = 9 kernels, acs_wide.hpp /
// acs_multi2.hpp): static (g, g + grid, ...) or, with OPT & kPersistQueue, the queue. first() before
// the first group's DMA, started() after it; next(g) where the next group's first DMA is issued (the
// queue resolves the ticket fetched a group ago), issued(nxt) right after that DMA; done() at exit.
template <int OPT>
struct GroupWalk {
  static constexpr bool QUEUE = (OPT & 1024) != 0;   // kPersistQueue (declared below)
  GroupQueue Q;
  int lane, qx, hops;
  uint32_t syncs = 0, ticket = 0;
  __device__ __forceinline__ GroupWalk(const RegArgs& a, int ngroups, int lane_, int max_hops)
      : Q{a.queue, ngroups, (int)gridDim.x, (int)(blockIdx.x % kQueueLabels)}, lane(lane_), qx(Q.label),
        hops((int)gridDim.x < kQueueLabels ? kQueueLabels - 1 : max_hops) {}
  __device__ __forceinline__ int first() { return QUEUE ? Q.first(lane, qx, syncs, hops) : (int)blockIdx.x; }
  __device__ __forceinline__ void started(int g) {
    if (QUEUE && g < Q.ngroups) ticket = Q.fetch(qx, lane);
  }
  __device__ __forceinline__ int next(int g) {
    return QUEUE ? Q.resolve(ticket, qx, lane, syncs, hops) : g + (int)gridDim.x;
  }
  __device__ __forceinline__ void issued(int nxt) {
    if (QUEUE && nxt < Q.ngroups) ticket = Q.fetch(qx, lane);
  }
  __device__ __forceinline__ void done() {
    if constexpr (QUEUE) Q.exit(lane);
  }
};

// Diagnostic stamps (kPersistStamp builds only; production never stamps): per wave, lane 0 writes
// {start lo, start hi, end lo, end hi (s_memrealtime, 100 MHz), HW_ID, XCC_ID, groups decoded, steals}
// with vector stores to a buffer of their own (tools/persist_bench.hip "tail").
__device__ __forceinline__ uint32_t hw_id_reg() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
  return v;
}
__device__ __forceinline__ uint32_t xcc_id_reg() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v;
}
__device__ __forceinline__ void write_stamps(uint32_t* stamps, int lane, uint64_t t0, uint32_t groups,
                                             uint32_t steals) {
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) {
    uint4* p = reinterpret_cast<uint4*>(stamps + (size_t)blockIdx.x * kStampWords);
    p[0] = make_uint4((uint32_t)t0, (uint32_t)(t0 >> 32), (uint32_t)t1, (uint32_t)(t1 >> 32));
    p[1] = make_uint4(hw_id_reg(), xcc_id_reg(), groups, steals);
  }
}

// ------------------------------------------------------------------------------------------------
// Soft decision, r = 1/2 (16-byte steps), block-major input [nb][T][4] staged by LDS-DMA in 8-step
// (128-byte) chunks per block, XOR-swizzled rows as in viterbi_soft_reg, one chunk in flight: the DMA
// of chunk c+1 (of this group, or chunk 0 of the next) is issued as soon as chunk c has been read
// into registers. The LDS reads are inline asm and the waits explicit vmcnt, so the compiler adds
// none of its own. Issue order per group:
//   chunk 0: wait | read | info loads | DMA(g,1)
//   chunk c: wait | read | DMA(g,c+1), or at the last chunk DMA(g',0) (g' = next group, or a
//            harmless reload when there is none: the op count never depends on the group)
//   end    : argmin, traceback, output stores
// Two chunks in flight in two buffers (kPersistDepth2: DMA of chunk c+2 at chunk c, vmcnt(8), which
// is exact because loads complete in order and at most OB < 8 stores sit between) is no faster:
// 1.005x the time in paired ABBA runs (tools/persist_bench ab, profiles/r02_persist_ab.txt). The
// kernel is power-bound (the clock falls from 2.4 GHz without input traffic to 1.9-2.1 GHz with
// it, profiles/r02_persist_bench.txt), not latency-bound.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int OFF>
__device__ __forceinline__ f32x4 lds_read_b128(uint32_t addr) {
  f32x4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

// Ablation switches for timing studies (tools/persist_bench.hip); production kernels use 0.
// Measured and removed in round 5 (A/B recorded in DESIGN.md 4.1b / 4.1c): line-aligned DMA staging
// (10 % less fetch, 17 % slower), one decision per value-numbering class (1.02x), staged loads +
// ds_write instead of LDS-DMA (1.5 % slower).
enum : int { kPersistNoMem = 1, kPersistNoTraceback = 2, kPersistSelectAcs = 4, kPersistCachedInput = 8,
             kPersistDepth2 = 16, kPersistNoMemRandom = 64, kPersistNoDma = 128, kPersistNoLdsRead = 256,
             kPersistInputNt = 512, kPersistQueue = 1024, kPersistStamp = 2048,
             kPersistInfoFirst = 4096, kPersistQueueHop1 = 8192, kPersistQueueHop7 = 16384,
             kPersistDeferOut = 32768 };
// kPersistDeferOut: a group's output stores (and the BSC path metric) are issued at the NEXT group's
// start, behind its first DMA, instead of at the group's end: every vmcnt wait also waits for the
// stores issued before it, and at the end of a group the next wait follows at once (the soft kernel's
// chunk 0, the hard kernel's group start), so each group began with a store round trip.
// Production schedules (round 6, tools/tail_bench.hip, profiles/r06c): the group queue with full
// stealing -- soft 0.982x the static walk's time, hard 0.869x (+ the info loads ahead of the DMA, 0.997x
// alone); 0, 1 or 7 steal hops measured alike.
// K = 7 only: a group of a smaller code is over in a few microseconds, about a ticket's round trip,
// and its dequeue rate exceeds the heads' (code 0, K = 3, BSC: 40,625 groups in 0.104 ms = 390
// dequeues/us; on the queue 0.104 -> 0.167 ms per launch, profiles/r06_bench) -- those keep the
// static walk.
// Deferred output stores for every code (tools/defer_bench.hip, profiles/r06_defer: ABBA time ratio
// 0.993 headline, 0.998 BSC K = 7, 0.995 code 0 BSC, 0.985 soft code 0; bit-identical).
constexpr int kPersistSoftProd = kPersistQueue | kPersistQueueHop7 | kPersistDeferOut;
constexpr int kPersistHardProd = kPersistQueue | kPersistQueueHop7 | kPersistInfoFirst | kPersistDeferOut;
template <CodeSpec C>
constexpr int persist_soft_opt() { return C.K >= 7 ? kPersistSoftProd : kPersistDeferOut; }
template <CodeSpec C>
constexpr int persist_hard_opt() { return C.K >= 7 ? kPersistHardProd : kPersistDeferOut; }
static_assert(kPersistQueue == 1024, "GroupWalk::QUEUE");
// steal hops of the queue schedule (GroupQueue::resolve): 0, or the OPT bits above
constexpr int queue_hops(int opt) {
  return (opt & kPersistQueueHop7) ? kQueueLabels - 1 : (opt & kPersistQueueHop1) ? 1 : 0;
}

// CCV_PERSIST_SOFT_WAVES (A/B builds only): the soft kernel's minimum waves per SIMD (2 in production:
// 195 VGPRs; 3 caps it at 168 and spills, 4.5 % slower on the static walk in round 5)
#ifndef CCV_PERSIST_SOFT_WAVES
#define CCV_PERSIST_SOFT_WAVES 2
#endif
template <CodeSpec C, int BLEN, int ABLATE = 0>
__global__ __launch_bounds__(kRegThreads) __attribute__((amdgpu_waves_per_eu(CCV_PERSIST_SOFT_WAVES)))
void viterbi_soft_persist(RegArgs a, int ngroups) {
  constexpr int S = 1 << (C.K - 1);
  static_assert(C.n == 2, "16-byte trellis steps");
  constexpr int PF = 8;                       // steps per chunk
  constexpr int UPR = PF;                     // 16-byte units per block per chunk = DMAs per chunk
  constexpr int ROWB = UPR * 16;
  constexpr int GRP = 16 / UPR;
  constexpr int BUF = kRegThreads * ROWB;     // one chunk of the group: 8 KiB
  constexpr int G = C.K - 1;                  // growth steps
  constexpr int T = BLEN + G;                 // trellis steps per block
  constexpr int NCH = (T + PF - 1) / PF;
  constexpr int IB = (BLEN + 7) >> 3;
  static_assert(BLEN >= 1 && BLEN <= kPersistMaxMain, "decisions of the main steps live in VGPRs");
  static_assert(NCH >= 4 && NCH % 2 == 0, "buffer = chunk parity across groups");
  constexpr bool DEPTH2 = (ABLATE & kPersistDepth2) != 0;   // two chunks in flight
  using DW = DecWord<S>;
  const int lane = threadIdx.x;
  const int nb = a.nblocks;
  const int stride_groups = gridDim.x;

  __shared__ __attribute__((aligned(1024))) unsigned char lds[DEPTH2 ? 2 * BUF : BUF];
  const unsigned char* in = reinterpret_cast<const unsigned char*>(a.in);
  constexpr uint32_t block_bytes = (uint32_t)T * 16;
  // DMA k of a chunk: lane l moves 16-byte unit j = l % 8 of block r = 8k + l / 8 of the group, from
  // swizzled slot su = j ^ (r / 2 % 8) of the block's chunk. The per-lane byte offsets inside a
  // group are the same for every group and chunk (+ c * 128): computed once, 8 VGPRs; the group
  // base is wave-uniform (SGPRs) and the chunk offset an immediate, so an issue costs no VALU.
  uint32_t dma_off[UPR];
#pragma unroll
  for (int k = 0; k < UPR; ++k) {
    const int r = k * (kRegThreads / UPR) + lane / UPR, j = lane % UPR;
    const int su = j ^ ((r / GRP) % UPR);
    dma_off[k] = (uint32_t)r * block_bytes + (uint32_t)su * 16;
  }
  // Groups holding the batch's last block clamp every unit into the buffer (a lane past the batch
  // replays block nb-1; a unit past the block end re-reads its last step; neither is ever read).
  auto issue_chunk = [&](int g, int c, int buf) __attribute__((always_inline)) {
    if constexpr ((ABLATE & kPersistNoDma) != 0) return;   // ablation: LDS reads of stale rows
    if constexpr ((ABLATE & kPersistCachedInput) != 0) g = blockIdx.x & 7;   // L2-resident input
    if (g * kRegThreads + kRegThreads < nb) {
      // buffer form: the group's base in an SGPR descriptor, the lane's offset as the VGPR offset
      // and the chunk's as the SGPR offset -- the global form wants a 64-bit VGPR address, one
      // v_lshl_add_u64 ahead of every DMA, which the DMA then waits for
      const __amdgpu_buffer_rsrc_t grp = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<unsigned char*>(in) + (size_t)g * kRegThreads * block_bytes, 0,
          kRegThreads * block_bytes, 0x00020000);
#pragma unroll
      for (int k = 0; k < UPR; ++k)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(grp, (lds_ptr_t)(lds + buf * BUF + k * kRegThreads * 16), 16,
                                                 dma_off[k], c * PF * 16, 0, (ABLATE & kPersistInputNt) ? 2 : 0);
    } else {
#pragma unroll
      for (int k = 0; k < UPR; ++k) {
        const int r = k * (kRegThreads / UPR) + lane / UPR, j = lane % UPR;
        const int su = j ^ ((r / GRP) % UPR);
        const int gb = g * kRegThreads + r < nb ? g * kRegThreads + r : nb - 1;
        uint32_t off = (uint32_t)(c * PF + su) * 16;
        off = off < block_bytes ? off : block_bytes - 16;
        __builtin_amdgcn_global_load_lds(in + (size_t)gb * block_bytes + off,
                                         (lds_ptr_t)(lds + buf * BUF + k * kRegThreads * 16), 16, 0, 0);
      }
    }
  };
  // without error counting the info loads still run (from the input): one instruction stream
  const uint8_t* info_src = a.info != nullptr ? a.info : reinterpret_cast<const uint8_t*>(a.in);
  const int info_stride = a.info != nullptr ? IB : 0;
  const uint32_t rd_base = (uint32_t)(uintptr_t)(lds_ptr_t)lds + (uint32_t)(lane * ROWB) +
                           (uint32_t)(((lane / GRP) % UPR) * 16);

  uint32_t errors = 0;
  constexpr bool QUEUE = (ABLATE & kPersistQueue) != 0, STAMP = (ABLATE & kPersistStamp) != 0;
  constexpr int HOPS = queue_hops(ABLATE);
  static_assert(!(QUEUE && DEPTH2), "the queue resolves one group ahead");
  static_assert(!(QUEUE && (ABLATE & kPersistNoMem)), "the next group is resolved with the DMA");
  const uint64_t t_start = STAMP ? __builtin_amdgcn_s_memrealtime() : 0;
  if constexpr (STAMP) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const GroupQueue Q{a.queue, ngroups, (int)gridDim.x, (int)(blockIdx.x % kQueueLabels)};
  int qx = Q.label;
  uint32_t steals = 0, ndone = 0, ticket = 0;
  // fewer waves than labels (a batch of < 8 groups): every head must be reachable
  const int hops = (int)gridDim.x < kQueueLabels ? kQueueLabels - 1 : HOPS;
  int g = QUEUE ? Q.first(lane, qx, steals, hops) : (int)blockIdx.x;
  if (!(ABLATE & kPersistNoMem) && g < ngroups) {
    issue_chunk(g, 0, 0);
    if constexpr (DEPTH2) issue_chunk(g, 1, 1);
  }
  if (QUEUE && g < ngroups) ticket = Q.fetch(qx, lane);
  constexpr bool DEFER = (ABLATE & kPersistDeferOut) != 0;
  uint64_t pend_bits = 0;   // DEFER: the previous group's output, stored behind this group's first DMA
  int pend_b = -1;
  for (int nxt = 0; g < ngroups; g = QUEUE ? nxt : g + stride_groups) {
    const int b = g * kRegThreads + lane;
    const bool has_next = g + stride_groups < ngroups;
    ++ndone;
    float M[S];
#pragma unroll
    for (int s = 0; s < S; ++s) M[s] = s ? __builtin_inff() : 0.0f;   // viterbi-decoder.c:212-218
    DW D[BLEN];
    uint8_t info[IB];

    // one chunk: wait for its DMA, read its rows, hand the buffer to the DMA two chunks ahead, run
    // its steps
    auto chunk_at = [&]<int c>() __attribute__((always_inline)) {
      f32x4 chunk[UPR];
      // ablations: full-entropy synthetic rows in [1, 2) instead of LDS reads
      auto synth_rows = [&]() __attribute__((always_inline)) {
        uint32_t ln = (uint32_t)(lane + g) * 0x9E3779B9u;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int x = 0; x < UPR; ++x) {
          const uint32_t r0 = ln ^ (uint32_t)(x * 0x85EBCA6Bu), r1 = r0 * 0xC2B2AE35u;
          chunk[x] = f32x4{__uint_as_float((r0 >> 9) | 0x3F800000u), __uint_as_float((r1 >> 9) | 0x3F800000u),
                           __uint_as_float((r0 & 0x7FFFFFu) | 0x3F800000u), __uint_as_float((r1 & 0x7FFFFFu) | 0x3F800000u)};
        }
      };
      if constexpr ((ABLATE & kPersistNoMemRandom) != 0) {   // no memory, full-entropy values
        synth_rows();
      } else if constexpr ((ABLATE & kPersistNoMem) != 0) {
        int ln = lane + g;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int x = 0; x < UPR; ++x)
          chunk[x] = f32x4{(float)((ln + x) & 3), (float)((ln + x + 1) & 3), (float)((ln + 2 * x) & 3),
                           (float)((ln ^ x) & 3)};
      } else {
        if constexpr (DEPTH2) wait_vmcnt<UPR>();   // the next chunk's may be in flight
        else wait_vmcnt<0>();
        // row x of this lane's block sits at slot x ^ sw: (row base | sw * 16) ^ (x * 16), the array
        // being 1 KiB aligned
        if constexpr ((ABLATE & kPersistNoLdsRead) != 0) synth_rows();
        else [&]<int... xs>(std::integer_sequence<int, xs...>) __attribute__((always_inline)) {
          ((chunk[xs] = lds_read_b128<(DEPTH2 ? c % 2 : 0) * BUF>(rd_base ^ (uint32_t)(xs * 16))), ...);
        }(std::make_integer_sequence<int, UPR>{});
        // the rows are in registers once these reads return; only then may the DMA overwrite them
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(chunk[0]), "+v"(chunk[1]), "+v"(chunk[2]), "+v"(chunk[3]), "+v"(chunk[4]),
                       "+v"(chunk[5]), "+v"(chunk[6]), "+v"(chunk[7])
                     :
                     : "memory");
        if constexpr (c == 0) {
          const int bc = b < nb ? b : nb - 1;
#pragma unroll
          for (int k = 0; k < IB; ++k) info[k] = info_src[(size_t)bc * info_stride + k];
          asm volatile("" ::: "memory");   // keep the info loads before the DMA (issue order above)
        }
        if constexpr (!DEPTH2) {
          if constexpr (c + 1 < NCH) {
            issue_chunk(g, c + 1, 0);
          } else if constexpr (QUEUE) {
            // the next group from the ticket fetched a group ago, its first chunk's DMA, then the
            // ticket of the group after it (returns long before it is read, at that group's last chunk)
            nxt = Q.resolve(ticket, qx, lane, steals, hops);
            issue_chunk(nxt < ngroups ? nxt : g, 0, 0);
            if (nxt < ngroups) ticket = Q.fetch(qx, lane);
          } else {
            issue_chunk(has_next ? g + stride_groups : g, 0, 0);
          }
        } else if constexpr (c + 2 < NCH) {
          issue_chunk(g, c + 2, c % 2);
        } else {
          issue_chunk(has_next ? g + stride_groups : g, c + 2 - NCH, c % 2);
        }
        if constexpr (DEFER && c == 0) {
          asm volatile("" ::: "memory");   // behind the DMA: the next chunk's wait finds them done
          if (pend_b >= 0) store_block<T>(a, pend_b, pend_bits);
        }
      }
      auto step_at = [&]<int u>() __attribute__((always_inline)) {
        constexpr int t = c * PF + u;
        const float bm[4] = {chunk[u].x, chunk[u].y, chunk[u].z, chunk[u].w};
        if constexpr (t < G) growth_step<C, t, float>(M, bm, __builtin_inff());
        else if constexpr (t < T) {
          if constexpr ((ABLATE & kPersistSelectAcs) != 0) D[t - G] = acs_step_select<C>(M, bm);
          else D[t - G] = acs_step<C, false, float>(M, bm);
          pin(D[t - G]);
        }
        __builtin_amdgcn_sched_barrier(0);   // schedule step by step: interleaving steps only adds VGPRs
      };
      [&]<int... us>(std::integer_sequence<int, us...>) __attribute__((always_inline)) {
        (step_at.template operator()<us>(), ...);
      }(std::make_integer_sequence<int, PF>{});
    };
    [&]<int... cs>(std::integer_sequence<int, cs...>) __attribute__((always_inline)) {
      (chunk_at.template operator()<cs>(), ...);
    }(std::make_integer_sequence<int, NCH>{});

    if constexpr ((ABLATE & kPersistNoTraceback) != 0) {
      uint64_t x = 0;
#pragma unroll
      for (int m = 0; m < BLEN; ++m) x ^= D[m];
#pragma unroll
      for (int s = 0; s < S; ++s) x += __float_as_uint(M[s]);
      if (b < nb) reinterpret_cast<uint64_t*>(a.out)[b] = x;
    } else {
      float best;
      const uint32_t st = (uint32_t)argmin_state<S, float>(M, __builtin_inff(), best);
      const uint64_t bits = traceback_regs<C.K, DW, BLEN>(D, st, a.blen);
      uint64_t ref = 0;
#pragma unroll
      for (int k = 0; k < IB; ++k) ref |= (uint64_t)info[k] << (56 - 8 * k);
      // lanes past the batch store nothing (exec-masked)
      if constexpr (DEFER) {
        if (b < nb) errors += block_errors<BLEN>(a, bits, ref);
        pend_b = b < nb ? b : -1;
        pend_bits = bits;
      } else if (b < nb) {
        store_block<T>(a, b, bits);
        errors += block_errors<BLEN>(a, bits, ref);
      }
    }
  }
  if (DEFER && pend_b >= 0) store_block<T>(a, pend_b, pend_bits);
  // the last group's look-ahead DMAs write LDS: they must land before the workgroup (and its LDS
  // allocation) ends
  wait_vmcnt<0>();
  if constexpr (QUEUE) Q.exit(lane);
  accumulate_errors(a, errors);
  if constexpr (STAMP) write_stamps(a.stamps, lane, t_start, ndone, steals);
}

// ------------------------------------------------------------------------------------------------
// Hard decision (BSC), block-major uint8 [nb][T], whole groups only (the host sends a partial last
// group to viterbi_hard_reg). A group's 64*T input bytes are contiguous and 4-byte aligned: one
// LDS-DMA of dwords stages them (double-buffered across groups), each lane reads its step bytes.
// The ACS runs on 16-bit metrics from the first step: reachable metrics are <= n*T < 0xFF00, so the
// reference's saturation (binary-symmetric-channel/viterbi-decoder.c:127-130) never binds outside
// the growth steps, whose unreachable states are the constant 0xFF00.
constexpr int kHardPersistMaxT = 64;   // staged bytes per block (LDS: 2 x 64 x 64 B)

template <int OFF>
__device__ __forceinline__ uint32_t lds_read_u8(uint32_t addr) {
  uint32_t r;
  asm volatile("ds_read_u8 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

// Metric type of the BSC persistent kernel (MMODE): 3 = fp32 (production since round 5), 2 = uint16_t
// (v_add_u16 / v_min_u16, rounds 2-4), 1 = u32, 0 = inline-asm u16 (ablations, tools/persist_bench).
// Every metric of this kernel is a small integer (<= n * T after the growth steps, whose unreachable
// states hold the constant 0xFF00), so fp32 adds, mins and the sign of m1 - m0 are exact and give the
// u16 decisions and path metrics bit for bit -- and the instruction stream is the soft kernel's
// (v_add_f32 / v_min_f32 / v_sub_f32 / v_alignbit). The u16 stream's waves were issue-stalled 0.33 of
// their lifetime (round-4 PMC) against 0.12 for the soft kernel: fp32 runs 0.428 instead of 0.456 ms per
// 104-frame launch, 239 instead of 225 Gbit/s (profiles/r05c/ab/bsc2_*). Also measured in round 5
// (profiles/r05a/ab/bsc_*, u16): no scheduling barrier between steps, the next chunk's symbols read a
// chunk ahead, two popcounts for the four branch metrics -- all within +-0.8 %.
template <CodeSpec C, int BLEN, int MMODE = 3, int OPT = 0>
__global__ __launch_bounds__(kRegThreads) __attribute__((amdgpu_waves_per_eu(2)))
void viterbi_hard_persist(RegArgs a, int ngroups) {
  constexpr int S = 1 << (C.K - 1);
  constexpr int NS = 1 << C.n;
  constexpr int PF = 8;
  constexpr int G = C.K - 1;
  constexpr int T = BLEN + G;
  constexpr int NCH = (T + PF - 1) / PF;
  static_assert(BLEN >= 1 && BLEN <= kPersistMaxMain && T <= kHardPersistMaxT, "register decisions");
  constexpr uint32_t kMask = NS - 1;   // decoder_input masks to n bits (viterbi-decoder.c:235-237)
  using DW = DecWord<S>;
  const int lane = threadIdx.x;
  const int stride_groups = gridDim.x;
  // sized for T = 64 (buffers sized by T, whole 1 KiB DMA instructions, give code 0 six waves per
  // SIMD instead of five: 1.019x the time, tools/defer_bench.hip round 6, profiles/r06_defer)
  constexpr int kBuf = kRegThreads * kHardPersistMaxT;
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * kBuf];
  const unsigned char* in = reinterpret_cast<const unsigned char*>(a.in);
  // 16-byte DMA units (round 4; dword units before): an LDS-DMA instruction holds the SIMD's VALU
  // issue whatever its width (tools/raterbench7.hip), so the group moves in 3
  // instructions instead of 12 at T = 46. The LDS image is the same: the group's bytes, contiguous.
  constexpr int units = (kRegThreads * T + 15) >> 4;   // 16-byte units per group
  auto issue_group = [&](int g, int buf) __attribute__((always_inline)) {
    const unsigned char* src = in + (size_t)g * kRegThreads * T;
    if constexpr ((kRegThreads * T) % 16 == 0) {
#pragma unroll
      for (int k = 0; k * kRegThreads < units; ++k) {
        int u = k * kRegThreads + lane;
        u = u < units ? u : units - 1;   // past the group: clamped (LDS slot never read)
        __builtin_amdgcn_global_load_lds(src + (size_t)u * 16, (lds_ptr_t)(lds + buf * kBuf + k * kRegThreads * 16),
                                         16, 0, 0);
      }
    } else {   // 64 * T not a multiple of 16: dword units
      constexpr int dunits = (kRegThreads * T) >> 2;
#pragma unroll
      for (int k = 0; k * kRegThreads < dunits; ++k) {
        int u = k * kRegThreads + lane;
        u = u < dunits ? u : dunits - 1;
        __builtin_amdgcn_global_load_lds(src + (size_t)u * 4, (lds_ptr_t)(lds + buf * kBuf + k * kRegThreads * 4),
                                         4, 0, 0);
      }
    }
  };

  uint32_t errors = 0;
  // group schedule (see GroupQueue): OPT & kPersistQueue takes groups from the queue, kPersistStamp
  // writes the diagnostic stamps
  constexpr bool QUEUE = (OPT & kPersistQueue) != 0, STAMP = (OPT & kPersistStamp) != 0;
  constexpr int HOPS = queue_hops(OPT);
  const uint64_t t_start = STAMP ? __builtin_amdgcn_s_memrealtime() : 0;
  if constexpr (STAMP) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const GroupQueue Q{a.queue, ngroups, (int)gridDim.x, (int)(blockIdx.x % kQueueLabels)};
  int qx = Q.label;
  uint32_t steals = 0, ndone = 0, ticket = 0;
  // fewer waves than labels (a batch of < 8 groups): every head must be reachable
  const int hops = (int)gridDim.x < kQueueLabels ? kQueueLabels - 1 : HOPS;
  int g = QUEUE ? Q.first(lane, qx, steals, hops) : (int)blockIdx.x;
  int buf = 0;
  if (g < ngroups) issue_group(g, 0);
  if (QUEUE && g < ngroups) ticket = Q.fetch(qx, lane);
  constexpr bool DEFER = (OPT & kPersistDeferOut) != 0;
  uint64_t pend_bits = 0;   // DEFER: the previous group's output and path metric
  uint32_t pend_pm = 0;
  int pend_b = -1;
  for (int nxt = 0; g < ngroups; g = QUEUE ? nxt : g + stride_groups, buf ^= 1) {
    const int b = g * kRegThreads + lane;
    ++ndone;
    // this group's bytes must have landed before the first read (vmcnt also covers the previous
    // group's output stores, long retired by now, and the queue ticket fetched a group ago)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // kPersistInfoFirst: the info loads ahead of the next group's DMA, so that their wait (at the
    // error count) is a counted vmcnt; behind it, as in rounds 2-5, the compiler waits vmcnt(0) for
    // them right here -- i.e. for the next group's DMA (and the queue ticket) at every group start
    uint64_t info = 0;
    if constexpr ((OPT & kPersistInfoFirst) != 0) {
      info = load_info<BLEN>(a, b);
      asm volatile("" ::: "memory");
    }
    if constexpr (QUEUE) {
      nxt = Q.resolve(ticket, qx, lane, steals, hops);
      if (nxt < ngroups) {
        issue_group(nxt, buf ^ 1);
        ticket = Q.fetch(qx, lane);
      }
    } else if (g + stride_groups < ngroups) {
      issue_group(g + stride_groups, buf ^ 1);
    }
    if constexpr (DEFER) {   // behind the next group's DMA: the next group start finds them done
      asm volatile("" ::: "memory");
      if (pend_b >= 0) {
        if (a.path_metric) a.path_metric[pend_b] = (int32_t)pend_pm;
        store_block<T>(a, pend_b, pend_bits);
      }
    }
    const uint32_t row_addr = (uint32_t)(uintptr_t)(lds_ptr_t)(lds + buf * kBuf + lane * T);
    if constexpr ((OPT & kPersistInfoFirst) == 0) info = load_info<BLEN>(a, b);
    // metric type (see above): 3 = fp32 (production); 2 = plain uint16_t (v_add_u16 / v_min_u16,
    // rounds 2-4); 0 = H16 inline-asm ops (round 2 first cut: hipcc puts an s_nop 0 after every
    // inline-asm VALU whose result is read next, 6 % slower than 2); 1 = u32 (v_bcnt-folded adds and
    // v_min_u32, half rate: 25 % slower than 2). tools/persist_bench abh.
    using MT = typename std::conditional<
        MMODE == 3, float,
        typename std::conditional<MMODE == 1, uint32_t,
                                  typename std::conditional<MMODE >= 2, uint16_t, H16>::type>::type>::type;
    MT M[S];
#pragma unroll
    for (int s = 0; s < S; ++s) M[s] = MT{(MT)(s ? 0xFF00u : 0u)};   // viterbi-decoder.c:225-228
    DW D[BLEN];
    auto chunk_at = [&]<int c>() __attribute__((always_inline)) {
      if (c * PF >= a.T) return;   // always true: per-chunk basic blocks (see the soft kernel)
      // inline-asm LDS reads: the compiler would otherwise wait for the NEXT group's DMA (into the
      // other buffer) before every read, since it cannot tell the buffers apart
      uint32_t sym[PF];
      [&]<int... us>(std::integer_sequence<int, us...>) __attribute__((always_inline)) {
        ((sym[us] = lds_read_u8<c * PF + us>(row_addr)), ...);
      }(std::make_integer_sequence<int, PF>{});
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(sym[0]), "+v"(sym[1]), "+v"(sym[2]), "+v"(sym[3]), "+v"(sym[4]), "+v"(sym[5]),
                     "+v"(sym[6]), "+v"(sym[7]));
      auto step_at = [&]<int u>() __attribute__((always_inline)) {
        constexpr int t = c * PF + u;
        if constexpr (t < T) {
          MT BM[NS];
          if constexpr (MMODE == 3 && NS == 4) {
            // popcount(k ^ s) over n = 2 bits as floats: k and k ^ 3 sum to 2
            const float p0 = (float)__builtin_popcount(sym[u] & kMask);
            const float p1 = (float)__builtin_popcount((sym[u] ^ 1u) & kMask);
            BM[0] = p0;
            BM[1] = p1;
            BM[2] = 2.0f - p1;
            BM[3] = 2.0f - p0;
          } else {
#pragma unroll
            for (int k = 0; k < NS; ++k) BM[k] = MT{(MT)__builtin_popcount((uint32_t)k ^ (sym[u] & kMask))};
          }
          if constexpr (MMODE == 2) {
#pragma unroll
            for (int k = 0; k < NS; ++k) asm volatile("" : "+v"(BM[k]));   // else hipcc folds the popcounts into every add (v_bcnt)
          }
          if constexpr (t < G) growth_step<C, t, MT>(M, BM, MT{(MT)0xFF00u});
          else {
            D[t - G] = acs_step<C, false, MT>(M, BM);
            pin(D[t - G]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      [&]<int... us>(std::integer_sequence<int, us...>) __attribute__((always_inline)) {
        (step_at.template operator()<us>(), ...);
      }(std::make_integer_sequence<int, PF>{});
    };
    [&]<int... cs>(std::integer_sequence<int, cs...>) __attribute__((always_inline)) {
      (chunk_at.template operator()<cs>(), ...);
    }(std::make_integer_sequence<int, NCH>{});

    uint32_t best, st;
    if constexpr (MMODE == 3) {
      float bf;
      st = (uint32_t)argmin_state<S, float>(M, 65280.0f, bf);
      best = (uint32_t)bf;
    } else {
      uint32_t Mu[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if constexpr (MMODE >= 1) Mu[s] = M[s];
        else Mu[s] = M[s].v & 0xFFFFu;
      }
      st = (uint32_t)argmin_state<S, uint32_t>(Mu, 0xFF00u, best);
    }
    const uint64_t bits = traceback_regs<C.K, DW, BLEN>(D, st, a.blen);
    if constexpr (DEFER) {
      errors += block_errors<BLEN>(a, bits, info);
      pend_b = b;
      pend_bits = bits;
      pend_pm = best;
    } else {
      if (a.path_metric) a.path_metric[b] = (int32_t)best;
      errors += emit_block<T, BLEN>(a, b, bits, info);
    }
  }
  if (DEFER && pend_b >= 0) {
    if (a.path_metric) a.path_metric[pend_b] = (int32_t)pend_pm;
    store_block<T>(a, pend_b, pend_bits);
  }
  if constexpr (QUEUE) Q.exit(lane);
  accumulate_errors(a, errors);
  if constexpr (STAMP) write_stamps(a.stamps, lane, t_start, ndone, steals);
}

// ------------------------------------------------------------------------------------------------
// Host side: persistent grids hold exactly the resident waves.
// Resident waves of a one-wave-per-workgroup kernel on the current device (occupancy x CUs), cached
// per (kernel, device): every persistent kernel has the type void(*)(RegArgs, int), so the key is the
// kernel's address, not its type. The table is process-wide (one definition across translation
// units) and guarded for plans driven from several host threads.
struct ResidentCache {
  std::mutex mu;
  struct Entry { const void* kernel; int dev; int waves; };
  std::vector<Entry> entries;
};
inline ResidentCache& resident_cache() {
  static ResidentCache c;
  return c;
}

// Introspection (ccv_plan_persistent_waves): while `active`, launch_persistent launches nothing and
// reports the grid it would use -- the cached value, or with `fresh` a new occupancy query.
struct PersistQuery {
  bool active = false;
  bool fresh = false;
  int waves = 0;
};
inline thread_local PersistQuery g_persist_query;

template <class Kern>
inline int resident_groups(Kern kernel, bool fresh = false) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  const void* key = reinterpret_cast<const void*>(kernel);
  ResidentCache& cache = resident_cache();
  std::lock_guard<std::mutex> lock(cache.mu);
  if (!fresh)
    for (const auto& e : cache.entries)
      if (e.kernel == key && e.dev == dev) return e.waves;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kRegThreads, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  // every wave walks the same number of groups: the same number of waves on each of a CU's four
  // SIMDs, or the SIMDs holding one more wave finish a third later (10 per CU: 0.50 vs 0.39 ms)
  if (per_cu >= 4) per_cu -= per_cu % 4;
  // CCV_PERSIST_WAVES_PER_CU caps the resident waves per CU exactly (occupancy / L2 working-set
  // studies, tools/waves_sweep.sh); read per kernel
  if (const char* env = std::getenv("CCV_PERSIST_WAVES_PER_CU")) {
    const int cap = std::atoi(env);
    if (cap > 0 && cap < per_cu) per_cu = cap;
  }
  if (!fresh) cache.entries.push_back({key, dev, per_cu * cus});
  return per_cu * cus;
}

template <class Kern>
inline hipError_t launch_persistent(Kern kernel, const RegArgs& a, int ngroups, hipStream_t stream) {
  if (g_persist_query.active) {
    g_persist_query.waves = resident_groups(kernel, g_persist_query.fresh);
    return hipSuccess;
  }
  if (ngroups <= 0) return hipSuccess;
  int resident = resident_groups(kernel);
  if (resident <= 0) return hipErrorInvalidDeviceFunction;
  const int grid = ngroups < resident ? ngroups : resident;
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(kRegThreads), 0, stream, a, ngroups);
  return hipGetLastError();
}

}  // namespace ccv
