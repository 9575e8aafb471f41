// reg_channel.hpp -- launch templates of the channel-fused decode kernels (channel_dev.hpp), shared
// by reg_channel.hip (BSC, and AWGN with the double-precision Box-Muller) and reg_channel_f32.hip
// (AWGN with the opt-in fp32 Box-Muller): two translation units so they compile in parallel.
#pragma once
#include <array>
#include <mutex>
#include <utility>
#include <vector>

#include "channel_dev.hpp"
#include "reg_codes.hpp"

namespace ccv {
namespace chan_impl {

// LDS budget of the decision column array per wave (opt-in kernel): 20 KiB = 8 waves per CU
constexpr size_t kChanLdsBudget = 20 * 1024;

// Waves per CU of a one-wave-workgroup kernel with `lds` bytes of dynamic LDS, cached per (kernel,
// LDS bytes, device): the auto choice below is fixed per instantiation, block length and device, and a
// sweep launches per chunk (the occupancy queries were paid on every K <= 7 channel launch).
inline int waves_per_cu(const void* fn, size_t lds) {
  struct Entry { const void* fn; size_t lds; int dev; int waves; };
  static std::mutex mu;
  static std::vector<Entry> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lock(mu);
  for (const Entry& e : cache)
    if (e.fn == fn && e.lds == lds && e.dev == dev) return e.waves;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kRegThreads, lds) != hipSuccess) return 0;
  cache.push_back({fn, lds, dev, n});
  return n;
}

// Decisions in LDS only where that costs no occupancy: LDS when its kernel holds at least as many
// waves per CU as the HBM-scratch one. Measured (profiles/r05_chan/chan_bench_lds_ab.jsonl, both
// forced and auto): K = 7 BSC idiom HBM 147 vs LDS 127 Gbit/s, BSC true parity (8 vs 8 waves) LDS
// 107 vs 99, code 3 BSC HBM 194 vs 188, code 0 AWGN fp32 HBM 366 vs 326; every AWGN kernel HBM.
template <size_t I, bool HARD, bool F32>
hipError_t launch_reg(const ChanArgs& a, int grid, hipStream_t stream) {
  constexpr CodeSpec C = kRegCodes[I];
  constexpr size_t word = (1u << (C.K - 1)) > 32 ? 8 : 4;
  const size_t lds = (size_t)(a.r.T - (C.K - 1)) * word * kRegThreads;
  bool use_lds = a.global_decisions != 1 && lds <= kChanLdsBudget;
  if (use_lds && a.global_decisions < 0) {
    const int w_lds = waves_per_cu(reinterpret_cast<const void*>(&viterbi_channel_lds<C, HARD, F32>), lds);
    const int w_reg = waves_per_cu(reinterpret_cast<const void*>(&viterbi_channel_reg<C, HARD, F32>), 0);
    use_lds = w_lds >= w_reg;
  }
  if (use_lds)
    hipLaunchKernelGGL((viterbi_channel_lds<C, HARD, F32>), dim3(grid), dim3(kRegThreads), lds, stream, a);
  else
    hipLaunchKernelGGL((viterbi_channel_reg<C, HARD, F32>), dim3(grid), dim3(kRegThreads), 0, stream, a);
  return hipGetLastError();
}

template <size_t I, bool HARD, bool F32>
hipError_t launch_multi(const ChanArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL((viterbi_channel_multi<kMultiCodes[I], HARD, F32>), dim3(grid), dim3(kRegThreads), 0,
                     stream, a);
  return hipGetLastError();
}

template <size_t I, bool F32>
hipError_t launch_frames(const ChanArgs& a, int grid, hipStream_t stream) {
  if constexpr (kMultiCodes[I].n == 2) {
    hipLaunchKernelGGL((channel_frames<kMultiCodes[I], false, F32>), dim3(grid), dim3(kRegThreads), 0, stream, a);
    return hipGetLastError();
  } else {
    return hipErrorInvalidValue;
  }
}

template <bool HARD, bool F32>
hipError_t launch_frames_rt(const ChanArgs& a, int n, const CodeRT& code, hipStream_t stream) {
  const dim3 grid((unsigned)((a.r.nblocks + kRegThreads - 1) / kRegThreads)), block(kRegThreads);
  if constexpr (!HARD) {
    if (a.iq_out) {   // the received points instead of the distances (CCV_CHANNEL_IQ)
      switch (n) {
        case 1: hipLaunchKernelGGL((channel_frames_rt<1, false, F32, true>), grid, block, 0, stream, a, code); break;
        case 2: hipLaunchKernelGGL((channel_frames_rt<2, false, F32, true>), grid, block, 0, stream, a, code); break;
        case 3: hipLaunchKernelGGL((channel_frames_rt<3, false, F32, true>), grid, block, 0, stream, a, code); break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
  }
  switch (n) {
    case 1: hipLaunchKernelGGL((channel_frames_rt<1, HARD, F32>), grid, block, 0, stream, a, code); break;
    case 2: hipLaunchKernelGGL((channel_frames_rt<2, HARD, F32>), grid, block, 0, stream, a, code); break;
    case 3: hipLaunchKernelGGL((channel_frames_rt<3, HARD, F32>), grid, block, 0, stream, a, code); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <bool HARD, bool F32, size_t... I>
constexpr std::array<ChanLaunchFn, sizeof...(I)> make_reg(std::index_sequence<I...>) {
  return {&launch_reg<I, HARD, F32>...};
}
template <bool HARD, bool F32, size_t... I>
constexpr std::array<ChanLaunchFn, sizeof...(I)> make_multi(std::index_sequence<I...>) {
  return {&launch_multi<I, HARD, F32>...};
}
template <bool F32, size_t... I>
constexpr std::array<ChanLaunchFn, sizeof...(I)> make_frames(std::index_sequence<I...>) {
  return {&launch_frames<I, F32>...};
}

}  // namespace chan_impl

// reg_channel_f32.hip: the fp32-noise AWGN launchers ([kNumRegCodes] / [kNumMultiCodes])
const ChanLaunchFn* channel_launchers_f32(bool multi);
const ChanLaunchFn* channel_frames_launchers_f32();
hipError_t launch_channel_frames_rt_f32(const ChanArgs& a, int n, const CodeRT& code, hipStream_t stream);

}  // namespace ccv
