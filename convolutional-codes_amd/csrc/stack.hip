// stack.hip -- launches of the sequential decoders: the wave-per-block stack decoder (stack_dev.hpp)
// and the lane-per-block Fano decoder (fano_dev.hpp). Built with -ffp-contract=off: the branch
// metrics' float product and double sum must not fuse.
#include <cstdlib>

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

hipError_t launch_stack(const StackArgs& a, bool hard, hipStream_t s) {
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

template <bool HARD, int NP, bool W32, bool RXL>
static hipError_t launch_fano_v(const FanoArgs& a, int grid, size_t lds, hipStream_t s) {
  const void* fn = reinterpret_cast<const void*>(&fano_decode<HARD, NP, W32, RXL>);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((fano_decode<HARD, NP, W32, RXL>), dim3(grid), dim3(kFanoThreads), lds, s, a);
  return hipGetLastError();
}

template <bool HARD, bool RXL>
static hipError_t launch_fano_h(const FanoArgs& a, int grid, size_t lds, hipStream_t s) {
  if (a.K <= 32) {
    if (a.n == 2) return launch_fano_v<HARD, 2, true, RXL>(a, grid, lds, s);
    if (a.n == 3) return launch_fano_v<HARD, 3, true, RXL>(a, grid, lds, s);
  }
  return launch_fano_v<HARD, 0, false, RXL>(a, grid, lds, s);
}

// Persistent lanes: as many waves as the LDS footprint lets the chip hold (256 CUs x 160 KiB), each
// lane pulls blocks from the queue. The received symbols move into LDS only while the chip still
// holds four waves per CU (one per SIMD): staging soft K=15 input (864 B per lane) would halve the
// resident lanes and measured slower (round-1 note in DESIGN.md); hard-decision input always fits.
hipError_t launch_fano(const FanoArgs& a, bool hard, hipStream_t s) {
  const size_t node_bytes = (size_t)a.T * kFanoThreads * ((hard ? sizeof(int32_t) : sizeof(float)) + 1);
  const size_t rx_bytes = (size_t)a.T * kFanoThreads * (hard ? 1 : (sizeof(float) << a.n));
  bool rxl = node_bytes + rx_bytes <= 40 * 1024;
  if (const char* env = std::getenv("CCV_FANO_RXL")) rxl = env[0] == '1' && node_bytes + rx_bytes <= 80 * 1024;
  const size_t lds = node_bytes + (rxl ? rx_bytes : 0);
  const int per_cu = (int)((160 * 1024) / lds) < 32 ? (int)((160 * 1024) / lds) : 32;
  const int resident = 256 * (per_cu > 0 ? per_cu : 1);
  const int waves_needed = (a.nblocks + kFanoThreads - 1) / kFanoThreads;
  const int grid = waves_needed < resident ? waves_needed : resident;
  if (hard) return rxl ? launch_fano_h<true, true>(a, grid, lds, s) : launch_fano_h<true, false>(a, grid, lds, s);
  return rxl ? launch_fano_h<false, true>(a, grid, lds, s) : launch_fano_h<false, false>(a, grid, lds, s);
}

}  // namespace ccv
