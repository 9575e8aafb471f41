// stack_dev.hpp -- the reference's stack (sequential) decoder on CDNA4, one wave per block.
//
// Reference: AWGN-channel/stack-decoder.c and binary-symmetric-channel/stack-decoder.c. A block is
// decoded by repeatedly extending the most probable path of a 64-entry path stack (STACK_DEPTH,
// :12) by both inputs until it spans the received frontier (:132-197); when the stack is full the
// least probable path is overwritten (duplicate_path, :227-241).
//
// MI355X mapping: the stack depth equals the wave width, so lane i of the wave IS stack entry i --
// its next-input index, encoder state, metric and decoded-path bits live in that lane's VGPRs. The
// reference's linear scans become wave reductions (row DPP + 4 readlanes) and a ballot + find-first
// for the lowest index among equal metrics (strict > / < from -inf / +inf, :199-225); the per-
// iteration bookkeeping is wave-uniform scalar code. There is no divergence at all: the whole wave
// follows one block's search. The block's received symbols (and the previous block's, see below)
// are staged once in LDS.
//
// Exactness: same float arithmetic as the reference -- the branch metric is
// (float)(1.0 + (double)(weight * d[sym])) (:274, float product, double sum) and path metrics
// accumulate in fp32 -- and the reference's streaming loop is kept: after step t arrives the most
// probable path is extended until it ends exactly at the frontier. That matters when the stack fills
// with equal metrics (idiom codes emit one symbol for both inputs): then the most and the least
// probable path are the same entry, duplicate_path copies it onto itself and both extensions land on
// it, so it skips a symbol and runs ahead of the frontier, where the reference's input buffer still
// holds the PREVIOUS block's symbols. The kernel reads exactly that: block b-1 of the batch (block 0:
// the caller's previous block, or zeros for a fresh decoder). A search that would read past the
// buffer (the reference then reads unrelated heap memory) is reported in the per-block status.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "trellis.hpp"

namespace ccv {

struct StackArgs {
  const void* in;          // soft: float [nb][T][2^n]; hard: uint8 [nb][T]
  const void* prev;        // the block decoded before block 0 (same layout, one block), or null
  int n, K, T, blen, gen;
  uint64_t poly[kMaxN];
  float weight;            // soft: code_param.metric_weight (code.h:16)
  int32_t bm0, bm1;        // hard: code_param.bit_metrics[0..1] (code.h:14)
  int nblocks;
  uint8_t* out;            // [nb][OB]
  int32_t* path_metric;    // hard: final path metric, may be null
  const uint8_t* info;     // optional [nb][IB]: count bit errors
  unsigned long long* err;
  int32_t* status;         // optional [nb]: 0 ok, 1 = the reference would read past its buffers
  unsigned int* next_block;  // stack_decode_rows: work counter, zero before the launch
  const uint16_t* symtab;    // stack_decode_rows, K <= kSymtabMaxK: [2^(K-1)] expected symbols
  int opt_row_lanes;         // host only (ccv_plan_set_option): 0 auto, 8, 16 lanes per search
  int opt_keys;              // host only: packed metric / index keys for hard input where they fit
};

constexpr int kStackDepth = 64;   // stack-decoder.c:12 == wave64

// Wave-wide max / min, result in every lane's register and returned as a uniform value. Row-level
// butterflies, then row_bcast:15 / row_bcast:31 carry rows 0-2 upward so lane 63 holds the result.
// Inline asm (explicit s_nop for the VALU-write -> DPP-read hazard): the compiler would wrap each
// step in canonicalising v_max x,x and a v_mov of the DPP "old" operand. Non-finite inputs: IEEE
// max/min skip NaN, as the reference's strict compares do.
#define CCV_DPP_STEP(op, ctrl) "s_nop 1\n" op "_dpp %0, %0, %0 " ctrl " row_mask:0xf bank_mask:0xf\n"
#define CCV_WAVE_REDUCE(op)                                                                      \
  CCV_DPP_STEP(op, "quad_perm:[1,0,3,2]") CCV_DPP_STEP(op, "quad_perm:[2,3,0,1]")                \
  CCV_DPP_STEP(op, "row_half_mirror") CCV_DPP_STEP(op, "row_mirror")                              \
  "s_nop 1\n" op "_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n"                     \
  "s_nop 1\n" op "_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
__device__ __forceinline__ float wave_max(float v) {
  asm volatile(CCV_WAVE_REDUCE("v_max_f32") : "+v"(v));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_min(float v) {
  asm volatile(CCV_WAVE_REDUCE("v_min_f32") : "+v"(v));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ int32_t wave_max(int32_t v) {
  asm volatile(CCV_WAVE_REDUCE("v_max_i32") : "+v"(v));
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int32_t wave_min(int32_t v) {
  asm volatile(CCV_WAVE_REDUCE("v_min_i32") : "+v"(v));
  return __builtin_amdgcn_readlane(v, 63);
}
#undef CCV_WAVE_REDUCE
#undef CCV_DPP_STEP

__device__ __forceinline__ uint32_t bcast(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ float bcast(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ int32_t bcast(int32_t v, int lane) { return __builtin_amdgcn_readlane(v, lane); }

// get_transition_metric's expected symbols (stack-decoder.c:249-272) for both inputs of a state,
// packed (e0 << 8) | e1. The register (state << (64-K)) | (input << 63) differs between the inputs
// only in bit 63, which the idiom's mask 0x1010..10 does not cover, so per polynomial one parity p
// and one masked parity q serve both: bit(in) = (p ^ (in & poly bit 63)) & (idiom ? !q : 1).
// Evaluated per lane in VALU for the lane's own entry (the scalar unit, shared by the CU's four
// SIMDs, is the stack search's bottleneck). NP = n when specialised (0: runtime n); W32: K <= 32,
// so the register lives in the upper 32 bits.
template <int NP, bool W32>
__device__ __forceinline__ uint32_t lane_symbols(const uint64_t (&poly)[kMaxN], int n, int K, bool idiom,
                                                 uint64_t state) {
  const uint64_t sr = state << (64 - K);
  uint32_t e0 = 0, e1 = 0;
#pragma unroll
  for (int k = 0; k < (NP ? NP : kMaxN); ++k) {
    if (NP || k < n) {
      uint32_t par, q;
      if constexpr (W32) {
        const uint32_t v = (uint32_t)(sr >> 32) & (uint32_t)(poly[k] >> 32);
        par = (uint32_t)__builtin_popcount(v);
        q = (uint32_t)__builtin_popcount(v & 0x10101010u);
      } else {
        const uint64_t v = sr & poly[k];
        par = (uint32_t)__popcll(v);
        q = (uint32_t)__popcll(v & 0x1010101010101010ull);
      }
      const uint32_t keep = idiom ? (~q & 1u) : 1u;
      const uint32_t b0 = par & keep;
      const uint32_t b1 = (par ^ (uint32_t)(poly[k] >> 63)) & keep;
      e0 = (e0 << 1) | (b0 & 1u);
      e1 = (e1 << 1) | (b1 & 1u);
    }
  }
  return (e0 << 8) | e1;
}

// PW = 32-bit words of decoded path per entry (T <= 32 * PW). Word w holds path bits 32w..32w+31,
// first bit in the MSB, i.e. output bytes 4w..4w+3 big-endian.
template <bool HARD, int PW, int NP, bool W32>
__global__ __launch_bounds__(kStackDepth) void stack_decode(StackArgs a) {
  using MT = typename std::conditional<HARD, int32_t, float>::type;
  using ET = typename std::conditional<HARD, uint8_t, float>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int b = blockIdx.x;
  const int T = a.T;
  const int NS = HARD ? 1 : (1 << a.n);
  const int per = T * NS;
  ET* cur_in = reinterpret_cast<ET*>(smem);
  ET* prev_in = cur_in + per;
  const ET* in = reinterpret_cast<const ET*>(a.in);
  const ET* prev = b > 0 ? in + (size_t)(b - 1) * per : reinterpret_cast<const ET*>(a.prev);
  for (int i = lane; i < per; i += kStackDepth) {
    ET v = in[(size_t)b * per + i];
    ET pv = prev ? prev[i] : (ET)0;
    if constexpr (HARD) {   // binary-symmetric-channel/stack-decoder.c:116-118 masks each symbol
      v = (ET)(v & ((1u << a.n) - 1u));
      pv = (ET)(pv & ((1u << a.n) - 1u));
    }
    cur_in[i] = v;
    prev_in[i] = pv;
  }
  __syncthreads();

  // stack entry = this lane
  uint32_t nxt = 0;      // next_input_index in trellis steps
  uint64_t st = 0;       // encoder_state
  MT met = 0;            // metric
  uint32_t path[PW];
#pragma unroll
  for (int w = 0; w < PW; ++w) path[w] = 0;
  int size = 1;          // next_stack_idx
  int cur = 0;
  int status = 0;
  uint64_t poly[kMaxN];
#pragma unroll
  for (int k = 0; k < kMaxN; ++k) poly[k] = a.poly[k];
  const int n = a.n, K = a.K;
  const bool idiom = a.gen == GEN_REF_X86;
  uint32_t esym = lane_symbols<NP, W32>(poly, n, K, idiom, 0);   // this entry's next symbols
  const MT lo_sent = HARD ? (MT)INT32_MIN : (MT)-__builtin_inff();
  const MT hi_sent = HARD ? (MT)INT32_MAX : (MT)__builtin_inff();

  for (int t = 1; t <= T && !status; ++t) {
    for (;;) {
      // get_most_probable_path (:213-225): strict > from the lowest value, first index wins
      const bool live = lane < size;
      const MT mx = wave_max(live ? met : lo_sent);
      const uint64_t hit = __ballot(live && met == mx && mx > lo_sent);
      if (hit == 0) { status = 1; break; }
      cur = __builtin_ctzll(hit);
      const uint32_t c_next = bcast(nxt, cur);
      if (c_next == (uint32_t)t) break;                 // the path ends at the frontier
      if (c_next >= (uint32_t)T) { status = 1; break; } // would read past the input buffer
      const uint64_t c_st = ((uint64_t)bcast((uint32_t)(st >> 32), cur) << 32) | bcast((uint32_t)st, cur);
      const MT c_met = bcast(met, cur);
      const uint32_t c_e = bcast(esym, cur);
      const uint32_t e0 = c_e >> 8, e1 = c_e & 0xFFu;
      const uint64_t ns0 = c_st >> 1;                          // successors (stack-decoder.c:272)
      const uint64_t ns1 = ns0 | ((uint64_t)1 << (K - 2));
      // symbols at or beyond the frontier are still the previous block's (see header)
      const ET* row = (c_next < (uint32_t)t ? cur_in : prev_in) + (size_t)c_next * NS;
      MT tm0, tm1;
      if constexpr (HARD) {
        const int32_t d0 = __builtin_popcount(e0 ^ row[0]), d1 = __builtin_popcount(e1 ^ row[0]);
        tm0 = d0 * a.bm1 + (n - d0) * a.bm0;   // binary-symmetric-channel/stack-decoder.c:266-272
        tm1 = d1 * a.bm1 + (n - d1) * a.bm0;
      } else {
        tm0 = (float)(1.0 + (double)(a.weight * row[e0]));   // AWGN-channel/stack-decoder.c:274
        tm1 = (float)(1.0 + (double)(a.weight * row[e1]));
      }
      // duplicate_path (:227-241)
      int lhs;
      if (size == kStackDepth) {
        const MT mn = wave_min(met);
        const uint64_t low = __ballot(met == mn && mn < hi_sent);
        if (low == 0) { status = 1; break; }
        lhs = __builtin_ctzll(low);
      } else {
        lhs = size++;
      }
      // extend the current path by input 0 and the duplicate by input 1 (:154-167); when lhs == cur
      // both extensions apply to the same entry, one after the other
      const uint32_t n0 = c_next + 1;
      const MT m0 = c_met + tm0;
      const bool same = lhs == cur;
      const uint32_t bn = same ? n0 : c_next;
      const uint64_t bs = same ? ns0 : c_st;
      const MT bm = same ? m0 : c_met;
      const uint32_t w1 = bn & 0xFF;                     // outbuf_widx is uint8_t
      if (lane == cur) { nxt = n0; st = ns0; met = m0; }
      // lhs: copy of the current path (before its extension unless it IS the current path)
      uint32_t cp[PW];
#pragma unroll
      for (int w = 0; w < PW; ++w) cp[w] = bcast(path[w], cur);
      if (lane == lhs) {
        nxt = bn + 1;
        st = ns1;
        met = bm + tm1;
#pragma unroll
        for (int w = 0; w < PW; ++w)
          path[w] = cp[w] | ((uint32_t)(w1 >> 5) == (uint32_t)w ? (0x80000000u >> (w1 & 31)) : 0u);
      }
      (void)bs;
      if (lane == cur || lane == lhs) esym = lane_symbols<NP, W32>(poly, n, K, idiom, st);
    }
  }
  // the most probable path at the end (or entry 0 if the search stopped)
  uint32_t res[PW];
#pragma unroll
  for (int w = 0; w < PW; ++w) res[w] = bcast(path[w], status ? 0 : cur);
  const int OB = (T + 7) >> 3, IB = (a.blen + 7) >> 3;
  uint32_t errors = 0;
  if (lane < OB) {
    uint32_t word = 0;
#pragma unroll
    for (int w = 0; w < PW; ++w) word = (lane >> 2) == w ? res[w] : word;
    const uint32_t byte = (word >> (24 - 8 * (lane & 3))) & 0xFFu;
    a.out[(size_t)b * OB + lane] = (uint8_t)byte;
    if (a.info && lane < IB) {
      int valid = a.blen - 8 * lane;
      valid = valid > 8 ? 8 : valid;
      const uint32_t mask = (0xFFu << (8 - valid)) & 0xFFu;
      errors = __builtin_popcount((byte ^ a.info[(size_t)b * IB + lane]) & mask);
    }
  }
  if constexpr (HARD) {
    if (lane == 0 && a.path_metric) a.path_metric[b] = bcast(met, status ? 0 : cur);
  }
  if (lane == 0 && a.status) a.status[b] = status;
  if (a.err) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) errors += __shfl_xor(errors, off, 64);
    if (lane == 0 && errors) atomicAdd(a.err, (unsigned long long)errors);
  }
}

// ---------------------------------------------------------------------------------------------
// Four searches per wave (round 2). The one-search-per-wave kernel above is bound by the CU's one
// scalar unit: every search iteration is ~50 SALU plus the branches of its wave-uniform control
// flow (profiles/r01_pmc_stack.txt: ~78 CU cycles per iteration). Here each 16-lane DPP row runs
// its own search and keeps a whole 64-entry stack, entry e in lane e % 16, slot e / 16, so:
//   * the scans are row reductions (quad_perm, row_half_mirror, row_mirror: every lane of the row
//     ends with the result, no readlane) -- max / min, then the lowest index among the equal ones
//     as a second u32 min reduction over per-lane candidates;
//   * all bookkeeping (frontier t, stack size, status) is row-uniform VALU state, so the four
//     searches share one instruction stream and the scalar unit only runs the loop;
//   * the 64 path metrics live in LDS next to the records (lane l reads its kRowSlots entries as one
//     ds_read_b128 at the top of each iteration, for the scans); the rest of an entry -- next index
//     and expected symbols packed, 32-bit encoder state, 64 path bits -- is one 16-byte LDS record
//     per entry, so the current path's record is one broadcast ds_read_b128 and an update one
//     ds_write_b128 by the row's lane 0 (current path) and lane 1 (duplicate);
//   * the most- and least-probable scans read the same metrics, so they run as ONE interleaved pair
//     of row reductions (values, then indices): each fills the other's DPP hazard slots (round 4);
//   * rows are persistent: a row that finishes its block writes the output and takes the next
//     block from a global counter, so a long search holds up only its own row.
// Same arithmetic, tie rules and streaming quirks as stack_decode (the previous block's symbols
// are read from global memory when a path runs ahead of the frontier). K <= 32 (32-bit state),
// n = NP in {2, 3}, T <= 64 (two path words); other codes use stack_decode.
constexpr int kRowsMaxT = 64;

// row-wide reductions over RL = 16 or 8 lanes (every lane of the row gets the result); explicit
// s_nop for the VALU-write -> DPP-read hazard, as CCV_WAVE_REDUCE
#define CCV_ROW_STEP(op, ctrl) "s_nop 1\n" op "_dpp %0, %0, %0 " ctrl " row_mask:0xf bank_mask:0xf\n"
#define CCV_ROW_REDUCE8(op)                                                                    \
  CCV_ROW_STEP(op, "quad_perm:[1,0,3,2]") CCV_ROW_STEP(op, "quad_perm:[2,3,0,1]")             \
  CCV_ROW_STEP(op, "row_half_mirror")
#define CCV_ROW_REDUCE(op) CCV_ROW_REDUCE8(op) CCV_ROW_STEP(op, "row_mirror")
#define CCV_ROW_FN(name, T, op)                                                                 \
  template <int RL>                                                                             \
  __device__ __forceinline__ T name(T v) {                                                      \
    if constexpr (RL == 16) asm volatile(CCV_ROW_REDUCE(op) : "+v"(v));                        \
    else asm volatile(CCV_ROW_REDUCE8(op) : "+v"(v));                                          \
    return v;                                                                                   \
  }
CCV_ROW_FN(row_max, float, "v_max_f32")
CCV_ROW_FN(row_min, float, "v_min_f32")
CCV_ROW_FN(row_max, int32_t, "v_max_i32")
CCV_ROW_FN(row_min, int32_t, "v_min_i32")
CCV_ROW_FN(row_min_u32, uint32_t, "v_min_u32")
#undef CCV_ROW_FN
#undef CCV_ROW_REDUCE8
#undef CCV_ROW_REDUCE
#undef CCV_ROW_STEP

// Two independent row reductions in ONE asm block, their DPP steps interleaved: a DPP read needs two
// wait states after the VALU write of its source, and the other chain's step fills one of them, so
// each step pair costs one s_nop 0 instead of the two s_nop 1 of two separate reductions (the
// most- and least-probable scans of a search iteration read the same metrics and are independent).
#define CCV_ROW_STEP2(opa, opb, ctrl)                                                          \
  opa "_dpp %0, %0, %0 " ctrl " row_mask:0xf bank_mask:0xf\n" opb "_dpp %1, %1, %1 " ctrl      \
      " row_mask:0xf bank_mask:0xf\n"
#define CCV_ROW_REDUCE2_8(opa, opb)                                                            \
  "s_nop 1\n" CCV_ROW_STEP2(opa, opb, "quad_perm:[1,0,3,2]") "s_nop 0\n"                       \
      CCV_ROW_STEP2(opa, opb, "quad_perm:[2,3,0,1]") "s_nop 0\n"                               \
      CCV_ROW_STEP2(opa, opb, "row_half_mirror")
#define CCV_ROW_REDUCE2(opa, opb) CCV_ROW_REDUCE2_8(opa, opb) "s_nop 0\n" CCV_ROW_STEP2(opa, opb, "row_mirror")
#define CCV_ROW_FN2(name, TA, TB, opa, opb)                                                    \
  template <int RL>                                                                            \
  __device__ __forceinline__ void name(TA& a, TB& b) {                                         \
    if constexpr (RL == 16) asm volatile(CCV_ROW_REDUCE2(opa, opb) : "+v"(a), "+v"(b));        \
    else asm volatile(CCV_ROW_REDUCE2_8(opa, opb) : "+v"(a), "+v"(b));                         \
  }
CCV_ROW_FN2(row_max_min, float, float, "v_max_f32", "v_min_f32")
CCV_ROW_FN2(row_max_min, int32_t, int32_t, "v_max_i32", "v_min_i32")
CCV_ROW_FN2(row_min_min_u32, uint32_t, uint32_t, "v_min_u32", "v_min_u32")
#undef CCV_ROW_FN2
#undef CCV_ROW_REDUCE2_8
#undef CCV_ROW_REDUCE2
#undef CCV_ROW_STEP2



// max / min without the canonicalising v_max x,x hipcc wraps around fmaxf (IEEE max/min skip NaN,
// as the reference's strict compares do)
__device__ __forceinline__ float vmax2(float a, float b) { float r; asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ __forceinline__ float vmin2(float a, float b) { float r; asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ __forceinline__ int32_t vmax2(int32_t a, int32_t b) { return a > b ? a : b; }
__device__ __forceinline__ int32_t vmin2(int32_t a, int32_t b) { return a < b ? a : b; }

// LDS bytes per row: the block's symbols (16-byte aligned), 65 entry records (64 + a dummy), then
// the 64 path metrics + the dummy (padded to 68)
__host__ __device__ constexpr size_t stack_rows_sym_bytes(int T, int ns, bool hard) {
  return (((size_t)T * (size_t)ns * (hard ? 1 : 4)) + 15) & ~(size_t)15;
}
__host__ __device__ constexpr size_t stack_rows_row_bytes(int T, int ns, bool hard) {
  return stack_rows_sym_bytes(T, ns, hard) + (size_t)(kStackDepth + 1) * 16 + 68 * 4;
}

// Expected-symbol table for the rows kernel: entry s = lane_symbols(s) (e0 << 8 | e1), so a new
// path's symbols are one cached 2-byte load instead of ~25 VALU of parities per search iteration.
constexpr int kSymtabMaxK = 16;   // 2^15 entries, 64 KiB
template <int NP>
__global__ void stack_symtab_init(uint16_t* tab, StackArgs a) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= (1u << (a.K - 1))) return;
  uint64_t poly[kMaxN];
#pragma unroll
  for (int k = 0; k < kMaxN; ++k) poly[k] = a.poly[k];
  tab[s] = (uint16_t)lane_symbols<NP, true>(poly, NP, a.K, a.gen == GEN_REF_X86, (uint64_t)s);
}

// KEY (hard input whose path metrics provably stay below 2^24 in magnitude: T * n * max|bit metric|
// < 2^24, stack_rows_keyed): metric and entry index share one 32-bit key, metric * 64 + index, so
// each scan is ONE row reduction -- max of metric * 64 + (63 - e) gives the largest metric and, among
// equal ones, the lowest index; min of metric * 64 + e the smallest and the lowest index. Entries not
// on the stack then hold -2^25 (a key below every live one).
__host__ __device__ constexpr bool stack_rows_keyed(int T, int n, int32_t bm0, int32_t bm1) {
  const long long b0 = bm0 < 0 ? -(long long)bm0 : bm0, b1 = bm1 < 0 ? -(long long)bm1 : bm1;
  return (long long)T * n * (b0 > b1 ? b0 : b1) < (1ll << 24);
}

template <bool HARD, int NP, bool TAB, int RL, bool KEY = false>
__global__ __launch_bounds__(kStackDepth) void stack_decode_rows(StackArgs a) {
  static_assert(RL == 16 || RL == 8, "a search is one DPP row or half-row");
  static_assert(HARD || !KEY, "keys pack integer metrics");
  constexpr int kRowLanes = RL;                        // lanes per search
  constexpr int kRowSlots = kStackDepth / RL;          // stack entries per lane
  using MT = typename std::conditional<HARD, int32_t, float>::type;
  using ET = typename std::conditional<HARD, uint8_t, float>::type;
  constexpr int NS = HARD ? 1 : (1 << NP);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x;
  const int l = lane & (kRowLanes - 1);
  const int rbase = lane & ~(kRowLanes - 1);
  const int T = a.T, K = a.K, nb = a.nblocks;
  const int per = T * NS;
  const size_t sym_bytes = stack_rows_sym_bytes(T, NS, HARD);
  unsigned char* rowp = smem + (size_t)(lane / kRowLanes) * stack_rows_row_bytes(T, NS, HARD);
  ET* syms = reinterpret_cast<ET*>(rowp);
  uint4* ent = reinterpret_cast<uint4*>(rowp + sym_bytes);   // [65] records
  // [68] path metrics; entry e = l * kRowSlots + k, so lane l reads its kRowSlots entries as 16-byte
  // rows; entries not on the stack hold the low sentinel (never a hit, so the scan needs no liveness
  // test; the least-probable scan only matters once all 64 are live)
  MT* metl = reinterpret_cast<MT*>(rowp + sym_bytes + (kStackDepth + 1) * 16);
  const ET* in = reinterpret_cast<const ET*>(a.in);
  const ET* prev_caller = reinterpret_cast<const ET*>(a.prev);
  uint64_t poly[kMaxN];
#pragma unroll
  for (int k = 0; k < kMaxN; ++k) poly[k] = a.poly[k];
  const bool idiom = a.gen == GEN_REF_X86;
  const uint32_t symmask = (1u << NP) - 1u;
  const MT lo_sent = HARD ? (MT)INT32_MIN : (MT)-__builtin_inff();
  const MT hi_sent = HARD ? (MT)INT32_MAX : (MT)__builtin_inff();
  const MT dead = KEY ? (MT)-(1 << 25) : lo_sent;   // metric of an entry not on the stack
  const int OB = (T + 7) >> 3, IB = (a.blen + 7) >> 3;
  // record: x = next index | expected symbols (e0 << 8 | e1) << 8, y = encoder state, z/w = path
  auto symbols_of = [&](uint32_t st) -> uint32_t {
    // a 32-bit byte offset from the table's SGPR base: one global_load_ushort, no 64-bit add
    if constexpr (TAB) return *reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(a.symtab) + (st << 1));
    else return lane_symbols<NP, true>(poly, NP, K, idiom, (uint64_t)st);
  };
  const uint32_t esym_root = symbols_of(0);

  // the next block from the work counter
  auto fetch = [&]() -> int {
    uint32_t b = 0;
    if (l == 0) b = atomicAdd(a.next_block, 1u);
    return __shfl((int)b, rbase, 64);
  };
  // stage a block's symbols and the root entry; the row's LDS is private to its 16 lanes
  auto stage = [&](int b) {
    const ET* src = in + (size_t)b * per;
    for (int i = l; i < per; i += kRowLanes) {
      ET v = src[i];
      if constexpr (HARD) v = (ET)(v & symmask);   // binary-symmetric-channel/stack-decoder.c:116-118
      syms[i] = v;
    }
    if (l == 0) ent[0] = make_uint4(esym_root << 8, 0u, 0u, 0u);
#pragma unroll
    for (int k = 0; k < kRowSlots; ++k) metl[l * kRowSlots + k] = (k == 0 && l == 0) ? (MT)0 : dead;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  };

  int blk = fetch();
  bool live_row = blk < nb;
  int t = 1, size = 1, status = 0;
  if (live_row) stage(blk);
  uint32_t errors = 0;

  while (__ballot(live_row) != 0) {
    if (live_row) {
      // get_most_probable_path (stack-decoder.c:213-225): strict > from -inf, first index wins
      MT met[kRowSlots];
#pragma unroll
      for (int k = 0; k < kRowSlots; ++k) met[k] = metl[l * kRowSlots + k];
      // ... and duplicate_path's least probable entry (:227-241, strict < from +inf, first index
      // wins) from the same metrics: both scans run as one interleaved pair of row reductions
      MT mx, mn;
      uint32_t cur, c2;
      bool ok;
      if constexpr (KEY) {
        int32_t kx = INT32_MIN, kn = INT32_MAX;
#pragma unroll
        for (int k = 0; k < kRowSlots; ++k) {
          kx = vmax2(kx, (int32_t)((uint32_t)met[k] * 64u) + (63 - (l * kRowSlots + k)));
          kn = vmin2(kn, (int32_t)((uint32_t)met[k] * 64u) + (l * kRowSlots + k));
        }
        row_max_min<RL>(kx, kn);
        mx = (MT)(kx >> 6);
        cur = 63u - ((uint32_t)kx & 63u);
        ok = kx > -(1 << 30);
        mn = (MT)(kn >> 6);
        c2 = (uint32_t)kn & 63u;
      } else {
        mx = met[0];
        mn = met[0];
#pragma unroll
        for (int k = 1; k < kRowSlots; ++k) {
          mx = vmax2(mx, met[k]);
          mn = vmin2(mn, met[k]);
        }
        row_max_min<RL>(mx, mn);
        uint32_t cand = kStackDepth;
        c2 = kStackDepth;
        if constexpr (!HARD && kRowSlots == 4) {
          // the lane's lowest slot holding the max / min without a VCC compare-select chain: the
          // sign of met[k] - mx (of mn - met[k]) is clear exactly on equality (+0: no metric is
          // ever -0), shifted into a 4-bit "differs" mask whose lowest clear bit is the slot;
          // v_ffbl gives -1 for a lane without one, above every index. -inf - -inf (a NaN, either
          // sign) only arises with entries not on the stack: then mx = -inf (no live entry, !ok,
          // cur unused) or mn = -inf (stack not full, c2 unused)
          uint32_t dx = 0, dn = 0;
#pragma unroll
          for (int k = kRowSlots - 1; k >= 0; --k) {
            dx = __builtin_amdgcn_alignbit(dx, __float_as_uint(met[k] - mx), 31);
            dn = __builtin_amdgcn_alignbit(dn, __float_as_uint(mn - met[k]), 31);
          }
          uint32_t fx, fn;
          asm("v_ffbl_b32 %0, %1" : "=v"(fx) : "v"(dx ^ 0xFu));
          asm("v_ffbl_b32 %0, %1" : "=v"(fn) : "v"(dn ^ 0xFu));
          cand = fx | (uint32_t)(l * kRowSlots);
          c2 = fn | (uint32_t)(l * kRowSlots);
        } else {
#pragma unroll
          for (int k = kRowSlots - 1; k >= 0; --k) {
            cand = met[k] == mx ? (uint32_t)(l * kRowSlots + k) : cand;
            c2 = met[k] == mn ? (uint32_t)(l * kRowSlots + k) : c2;
          }
        }
        row_min_min_u32<RL>(cand, c2);
        cur = cand;
        ok = mx > lo_sent;
      }
      // the common path is branch-free: every quantity is computed, the outcome selected
      const uint4 rec = ent[ok ? cur : (uint32_t)kStackDepth];
      const uint32_t c_next = rec.x & 0xFFu;
      // the path ends at the frontier: the next symbol arrives (t + 1). The reference then scans
      // again and finds the same path (no metric changed), now one step behind the frontier, and
      // extends it -- done here in the same iteration, so an arrival costs no scan of its own.
      const bool adv = ok && c_next == (uint32_t)t;
      const int tn = t + (adv ? 1 : 0);
      bool bad = !ok || (!adv && c_next >= (uint32_t)T);     // would read past the input buffer
      bool ext = !bad && tn <= T;
      const uint32_t e0 = (rec.x >> 16) & 0xFFu, e1 = (rec.x >> 8) & 0xFFu;
      const uint32_t ci = c_next < (uint32_t)T ? c_next : (uint32_t)T - 1u;
      // the new paths' expected symbols (lane 0: input 0 of the current path, lane 1: its duplicate
      // by input 1), loaded here so the latency hides behind the least-probable scan
      const bool dup = l == 1;
      const uint32_t ns0 = rec.y >> 1, ns1 = ns0 | (1u << (K - 2));
      const uint32_t est = dup ? ns1 : ns0;
      uint32_t es = symbols_of(est);
      ET r0, r1;
      if constexpr (HARD) { r0 = r1 = syms[ci]; }
      else { r0 = syms[ci * NS + e0]; r1 = syms[ci * NS + e1]; }
      if (ext && c_next >= (uint32_t)tn) {
        // symbols at or beyond the frontier are still the previous block's (header of stack_decode)
        const ET* pv = blk > 0 ? in + (size_t)(blk - 1) * per : prev_caller;
        if constexpr (HARD) {
          r0 = r1 = pv ? (ET)(pv[c_next] & symmask) : (ET)0;
        } else {
          r0 = pv ? pv[c_next * NS + e0] : 0.0f;
          r1 = pv ? pv[c_next * NS + e1] : 0.0f;
        }
      }
      MT tm0, tm1;
      if constexpr (HARD) {
        const int32_t d0 = __builtin_popcount(e0 ^ r0), d1 = __builtin_popcount(e1 ^ r1);
        tm0 = d0 * a.bm1 + (NP - d0) * a.bm0;   // binary-symmetric-channel/stack-decoder.c:266-272
        tm1 = d1 * a.bm1 + (NP - d1) * a.bm0;
      } else {
        tm0 = (float)(1.0 + (double)(a.weight * r0));   // AWGN-channel/stack-decoder.c:274
        tm1 = (float)(1.0 + (double)(a.weight * r1));
      }
      // duplicate_path (:227-241): a free entry, or the least probable one (mn / c2 above)
      const bool full = size == kStackDepth;
      const bool dbad = ext && full && !(mn < hi_sent);
      bad = bad || dbad;
      ext = ext && !dbad;
      const uint32_t lhs = full ? c2 : (uint32_t)size;
      size += (ext && !full) ? 1 : 0;
      // extend the current path by input 0 and the duplicate by input 1 (:154-167); when lhs == cur
      // both extensions apply to the same entry, one after the other
      const uint32_t n0 = c_next + 1;
      const MT m0 = mx + tm0;
      const bool same = lhs == cur;
      const uint32_t bn = same ? n0 : c_next;
      const MT lhs_met = (same ? m0 : mx) + tm1;
      const uint32_t w1 = bn & 0xFFu;   // outbuf_widx is uint8_t
      // lane 0 of the row writes the current path's record and metric, lane 1 the duplicate's
      const uint32_t nx = dup ? bn + 1 : n0;
      const uint32_t bit = dup ? 0x80000000u >> (w1 & 31u) : 0u;
      const uint32_t p0 = rec.z | (w1 < 32u ? bit : 0u);
      const uint32_t p1 = rec.w | (w1 >= 32u && w1 < 64u ? bit : 0u);
      const uint32_t slot = dup ? lhs : (same ? (uint32_t)kStackDepth : cur);
      asm volatile("" : "+v"(es));   // keeps the table load ahead of the branch below
      if (ext && l < 2) {
        ent[slot] = make_uint4((nx & 0xFFu) | (es << 8), est, p0, p1);
        // the metric's address from its own base: otherwise hipCC derives it from the record's
        // (ent + 16 slot - 12 slot) with a 64-bit v_mad_u64_u32
        uint32_t mslot = slot;
        asm volatile("" : "+v"(mslot));
        metl[mslot] = dup ? lhs_met : m0;
      }
      t = tn;
      const bool finish = bad || t > T;
      status = bad ? 1 : status;
      if (finish) {
        // the most probable path at the end, or entry 0 if the search stopped
        const uint4 res = status ? ent[0] : rec;
        const MT m_entry0 = metl[0];
        if (l < OB) {
          const uint32_t word = l < 4 ? res.z : res.w;
          const uint32_t byte = (word >> (24 - 8 * (l & 3))) & 0xFFu;
          a.out[(size_t)blk * OB + l] = (uint8_t)byte;
          if (a.info && l < IB) {
            int valid = a.blen - 8 * l;
            valid = valid > 8 ? 8 : valid;
            const uint32_t mask = (0xFFu << (8 - valid)) & 0xFFu;
            errors += __builtin_popcount((byte ^ a.info[(size_t)blk * IB + l]) & mask);
          }
        }
        if constexpr (HARD) {
          if (l == 0 && a.path_metric) a.path_metric[blk] = status ? m_entry0 : mx;
        }
        if (l == 0 && a.status) a.status[blk] = status;
        blk = fetch();
        live_row = blk < nb;
        if (live_row) {
          stage(blk);
          t = 1;
          size = 1;
          status = 0;
        }
      }
    }
  }
  if (a.err) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) errors += __shfl_xor(errors, off, 64);
    if (lane == 0 && errors) atomicAdd(a.err, (unsigned long long)errors);
  }
}

}  // namespace ccv
