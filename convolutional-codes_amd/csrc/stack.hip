// stack.hip -- launches of the sequential decoders: the wave-per-block stack decoder (stack_dev.hpp)
// and the lane-per-block Fano decoder (fano_dev.hpp). Built with -ffp-contract=off: the branch
// metrics' float product and double sum must not fuse.
#include <cstdio>
#include <cstdlib>

#include <hipcub/hipcub.hpp>

#include "fano_dev.hpp"
#include "stack_dev.hpp"

namespace ccv {

template <bool HARD, int PW, int NP, bool W32>
static hipError_t launch_v(const StackArgs& a, size_t lds, hipStream_t s) {
  hipLaunchKernelGGL((stack_decode<HARD, PW, NP, W32>), dim3(a.nblocks), dim3(kStackDepth), lds, s, a);
  return hipGetLastError();
}

// rate 1/2 and 1/3 codes with K <= 32 (the codebook, K=15) get specialised symbol code
template <bool HARD, int PW>
static hipError_t launch_pw(const StackArgs& a, size_t lds, hipStream_t s) {
  if (a.K <= 32) {
    if (a.n == 2) return launch_v<HARD, PW, 2, true>(a, lds, s);
    if (a.n == 3) return launch_v<HARD, PW, 3, true>(a, lds, s);
  }
  return launch_v<HARD, PW, 0, false>(a, lds, s);
}

bool stack_rows_eligible(int n, int K, int T);

// Four searches per wave (stack_decode_rows) as persistent rows: as many waves as the chip holds
// at once, capped by the blocks (4 per wave).
template <bool HARD, int NP, bool TAB, int RL, bool KEY = false>
static hipError_t launch_rows(const StackArgs& a, hipStream_t s) {
  constexpr int kStackRows = kStackDepth / RL;   // searches per wave
  const void* fn = reinterpret_cast<const void*>(&stack_decode_rows<HARD, NP, TAB, RL, KEY>);
  const size_t lds = (size_t)kStackRows * stack_rows_row_bytes(a.T, HARD ? 1 : 1 << NP, HARD);
  int dev = 0, cus = 0, per_cu = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kStackDepth, lds);
  if (e != hipSuccess) return e;
  const long resident = (long)(cus > 0 ? cus : 1) * (per_cu > 0 ? per_cu : 1);
  const long waves_needed = ((long)a.nblocks + kStackRows - 1) / kStackRows;
  const int grid = (int)(waves_needed < resident ? waves_needed : resident);
  if (std::getenv("CCV_DEBUG"))
    std::fprintf(stderr, "stack rows: %d lanes per search, table %d, keys %d, lds %zu B/wave, %d waves/CU x %d CUs, grid %d\n",
                 RL, (int)TAB, (int)KEY, lds, per_cu, cus, grid);
  hipLaunchKernelGGL((stack_decode_rows<HARD, NP, TAB, RL, KEY>), dim3(grid), dim3(kStackDepth), lds, s, a);
  return hipGetLastError();
}

template <bool HARD, int NP>
static hipError_t launch_rows_t(const StackArgs& a, hipStream_t s) {
  // Hard input whose metrics fit a 32-bit key with the entry index (stack_dev.hpp) runs one reduction
  // per scan. Lanes per search: 16, except hard input without keys: 8 (8 entries per lane, 8 searches
  // per wave -- fewer DPP steps, but twice the LDS per wave, which for soft input caps a CU at 9 waves).
  // Measured (profiles/r02c_stack_ab.txt): soft 16 lanes 546 vs 8 lanes 519 Mbit/s; hard keyed
  // 16 lanes 1275, 8 lanes 1259, unkeyed 8 lanes 1104-1152, 16 lanes 1073. The plan options
  // "stack_row_lanes" and "stack_keys" override.
  bool keyed = false;
  if constexpr (HARD) keyed = a.opt_keys && a.symtab != nullptr && stack_rows_keyed(a.T, a.n, a.bm0, a.bm1);
  const int rl = a.opt_row_lanes ? a.opt_row_lanes : (HARD && !keyed ? 8 : 16);
  if (keyed) {
    if (rl == 8) return launch_rows<HARD, NP, true, 8, HARD>(a, s);
    return launch_rows<HARD, NP, true, 16, HARD>(a, s);
  }
  if (rl == 8) return a.symtab ? launch_rows<HARD, NP, true, 8>(a, s) : launch_rows<HARD, NP, false, 8>(a, s);
  return a.symtab ? launch_rows<HARD, NP, true, 16>(a, s) : launch_rows<HARD, NP, false, 16>(a, s);
}

bool stack_symtab_eligible(int n, int K, int T) { return stack_rows_eligible(n, K, T) && K <= kSymtabMaxK; }

hipError_t launch_stack_symtab(uint16_t* tab, const StackArgs& a, hipStream_t s) {
  const unsigned S = 1u << (a.K - 1);
  const dim3 grid((S + 255) / 256), block(256);
  if (a.n == 2) hipLaunchKernelGGL((stack_symtab_init<2>), grid, block, 0, s, tab, a);
  else hipLaunchKernelGGL((stack_symtab_init<3>), grid, block, 0, s, tab, a);
  return hipGetLastError();
}

bool stack_rows_eligible(int n, int K, int T) { return K <= 32 && (n == 2 || n == 3) && T <= kRowsMaxT; }

hipError_t launch_stack(const StackArgs& a, bool hard, hipStream_t s) {
  if (stack_rows_eligible(a.n, a.K, a.T) && a.next_block != nullptr) {
    if (hard) return a.n == 2 ? launch_rows_t<true, 2>(a, s) : launch_rows_t<true, 3>(a, s);
    return a.n == 2 ? launch_rows_t<false, 2>(a, s) : launch_rows_t<false, 3>(a, s);
  }
  const size_t per = (size_t)a.T * (hard ? 1 : ((size_t)1 << a.n));
  const size_t lds = 2 * per * (hard ? 1 : sizeof(float));
  const int pw = (a.T + 31) / 32;
  if (hard) {
    if (pw <= 2) return launch_pw<true, 2>(a, lds, s);
    if (pw <= 4) return launch_pw<true, 4>(a, lds, s);
    if (pw <= 8) return launch_pw<true, 8>(a, lds, s);
    return launch_pw<true, 10>(a, lds, s);
  }
  if (pw <= 2) return launch_pw<false, 2>(a, lds, s);
  if (pw <= 4) return launch_pw<false, 4>(a, lds, s);
  if (pw <= 8) return launch_pw<false, 8>(a, lds, s);
  return launch_pw<false, 10>(a, lds, s);
}

// Persistent lanes: exactly as many waves as the chip holds at once (occupancy query: a wave that
// is not resident from the start would only begin after a resident one has finished its whole
// share, doubling the launch), each lane pulling blocks from the queue.
template <bool HARD, int NP, bool W32, int RM>
static hipError_t launch_fano_v(const FanoArgs& a, size_t lds, hipStream_t s) {
  if constexpr (W32 && NP != 0) {   // the expected-symbol table variant, where the plan built one
    if (a.symtab) {
      const void* fnt = reinterpret_cast<const void*>(&fano_decode<HARD, NP, W32, RM, true>);
      if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(fnt, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
      }
      int dev = 0, cus = 0, per_cu = 0;
      hipError_t e = hipGetDevice(&dev);
      if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fnt, kFanoThreads, lds);
      if (e != hipSuccess) return e;
      const int resident = (cus > 0 ? cus : 1) * (per_cu > 0 ? per_cu : 1);
      const int waves_needed = (a.nblocks + kFanoThreads - 1) / kFanoThreads;
      const int grid = waves_needed < resident ? waves_needed : resident;
      hipLaunchKernelGGL((fano_decode<HARD, NP, W32, RM, true>), dim3(grid), dim3(kFanoThreads), lds, s, a);
      return hipGetLastError();
    }
  }
  const void* fn = reinterpret_cast<const void*>(&fano_decode<HARD, NP, W32, RM>);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  int dev = 0, cus = 0, per_cu = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kFanoThreads, lds);
  if (e != hipSuccess) return e;
  const int resident = (cus > 0 ? cus : 1) * (per_cu > 0 ? per_cu : 1);
  const int waves_needed = (a.nblocks + kFanoThreads - 1) / kFanoThreads;
  const int grid = waves_needed < resident ? waves_needed : resident;
  if (std::getenv("CCV_DEBUG"))
    std::fprintf(stderr, "fano: lds %zu B/wave, %d waves/CU x %d CUs, grid %d\n", lds, per_cu, cus, grid);
  hipLaunchKernelGGL((fano_decode<HARD, NP, W32, RM>), dim3(grid), dim3(kFanoThreads), lds, s, a);
  return hipGetLastError();
}

template <bool HARD>
static hipError_t launch_fano_h(const FanoArgs& a, int rm, size_t lds, hipStream_t s) {
  if (a.K <= 32 && a.n == 2) {
    if constexpr (!HARD) {
      if (rm == kRowsIQ) return launch_fano_v<false, 2, true, kRowsIQ>(a, lds, s);
      if (rm == kRowsIQLds) return launch_fano_v<false, 2, true, kRowsIQLds>(a, lds, s);
    }
    if (rm == kRowsLds) return launch_fano_v<HARD, 2, true, kRowsLds>(a, lds, s);
    if (rm == kRowsGlobal) return launch_fano_v<HARD, 2, true, kRowsGlobal>(a, lds, s);
    return launch_fano_v<HARD, 2, true, kRowsDirect>(a, lds, s);
  }
  if (a.K <= 32 && a.n == 3) {
    if (HARD && rm == kRowsLds) return launch_fano_v<HARD, 3, true, HARD ? kRowsLds : kRowsDirect>(a, lds, s);
    if (HARD && rm == kRowsGlobal) return launch_fano_v<HARD, 3, true, HARD ? kRowsGlobal : kRowsDirect>(a, lds, s);
    return launch_fano_v<HARD, 3, true, kRowsDirect>(a, lds, s);
  }
  if (HARD && rm == kRowsLds) return launch_fano_v<HARD, 0, false, HARD ? kRowsLds : kRowsDirect>(a, lds, s);
  if (HARD && rm == kRowsGlobal) return launch_fano_v<HARD, 0, false, HARD ? kRowsGlobal : kRowsDirect>(a, lds, s);
  return launch_fano_v<HARD, 0, false, kRowsDirect>(a, lds, s);
}

// Received rows (fano_dev.hpp, RM): in LDS for hard input (one byte per node, the footprint stays
// small); for soft rate-1/2 input the two rows a move can land on are loaded from global memory at the
// top of each pass (kRowsGlobal), so their latency overlaps the pass. Round 1 measured the prefetch
// ~10 % slower (profiles/r01_fano.txt), but the round-3 one-loop kernel waits on memory (PMC, round 4:
// wait 0.66, valu_frac 0.17) and the prefetch now wins: 4 dB 49.6 -> 55.7 Mbit/s, 67.2 with the
// parities computed instead of the table load (profiles/r04c/fano_ab.txt). Soft K=15 rows in LDS
// (16 B per node) cut the chip from 9 to 2 waves per CU and run 4x slower. The plan option
// "fano_rows" (FanoArgs::rows_mode) overrides.
// Received points (option "fano_input" 1, soft rate 1/2, K <= 32): half-size rows prefetched from
// global memory (kRowsIQ), or in LDS with "fano_rows" 1 (kRowsIQLds).
hipError_t launch_fano(const FanoArgs& a, bool hard, hipStream_t s) {
  const size_t node_bytes = fano_node_bytes(a.T, hard ? sizeof(int32_t) : sizeof(float));
  if (a.iq) {
    if (hard || a.n != 2 || a.K > 32) return hipErrorInvalidValue;
    const bool lds_rows = a.rows_mode == kRowsLds || a.rows_mode == kRowsIQLds;
    const size_t lds = node_bytes + (lds_rows ? (size_t)a.T * kFanoThreads * 8 : 0);
    return launch_fano_h<false>(a, lds_rows ? kRowsIQLds : kRowsIQ, lds, s);
  }
  const size_t row_bytes = (size_t)a.T * kFanoThreads * (hard ? 1 : 16);
  const bool rowable = hard || (a.n == 2 && a.K <= 32);
  int rm = hard ? kRowsLds : (rowable ? kRowsGlobal : kRowsDirect);
  if (a.rows_mode >= 0) rm = rowable ? a.rows_mode : kRowsDirect;
  if (rm == kRowsLds && node_bytes + row_bytes > 80 * 1024) rm = kRowsGlobal;
  if (rm < 0 || rm > 2) rm = kRowsDirect;
  const size_t lds = node_bytes + (rm == kRowsLds ? row_bytes : 0);
  return hard ? launch_fano_h<true>(a, rm, lds, s) : launch_fano_h<false>(a, rm, lds, s);
}

// Noisiest-first queue order for the soft Fano decoder (fano_dev.hpp, fano_score): scores, then a
// descending radix sort of (score, block) pairs. Scratch layout: keys in/out, indices in/out, the
// sort's temporary storage. A null scratch returns the bytes needed.
size_t fano_order_bytes(int nblocks) {
  size_t tmp = 0;
  (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp, (const float*)nullptr, (float*)nullptr,
                                                     (const uint32_t*)nullptr, (uint32_t*)nullptr, nblocks);
  return 16 * (size_t)nblocks + tmp + 256;
}

static hipError_t noise_order(const void* in_v, int n_out, int T, int nblocks, void* scratch, size_t bytes,
                              const uint32_t** order, hipStream_t s, bool iq = false) {
  const size_t n = (size_t)nblocks;
  float* k_in = static_cast<float*>(scratch);
  float* k_out = k_in + n;
  uint32_t* i_in = reinterpret_cast<uint32_t*>(k_out + n);
  uint32_t* i_out = i_in + n;
  void* tmp = reinterpret_cast<void*>(((uintptr_t)(i_out + n) + 255) & ~(uintptr_t)255);
  size_t tmp_bytes = bytes - (size_t)(static_cast<char*>(tmp) - static_cast<char*>(scratch));
  const float* in = static_cast<const float*>(in_v);
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  if (iq && n_out == 2) hipLaunchKernelGGL(fano_score_iq<2>, grid, block, 0, s, in, T, nblocks, k_in, i_in);
  else if (iq) return hipErrorInvalidValue;
  else if (n_out == 2) hipLaunchKernelGGL((fano_score<4>), grid, block, 0, s, in, T, nblocks, k_in, i_in);
  else if (n_out == 3) hipLaunchKernelGGL((fano_score<8>), grid, block, 0, s, in, T, nblocks, k_in, i_in);
  else return hipErrorInvalidValue;
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = hipcub::DeviceRadixSort::SortPairsDescending(tmp, tmp_bytes, k_in, k_out, i_in, i_out, nblocks, 0,
                                                   32, s);
  *order = i_out;
  return e;
}

hipError_t launch_fano_order(const FanoArgs& a, void* scratch, size_t bytes, const uint32_t** order,
                             hipStream_t s) {
  return noise_order(a.in, a.n, a.T, a.nblocks, scratch, bytes, order, s, a.iq != 0);
}

}  // namespace ccv
