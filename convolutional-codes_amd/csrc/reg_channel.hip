// reg_channel.hip -- ahead-of-time instantiation of the channel-fused decode kernels
// (channel_dev.hpp): AWGN soft and BSC hard for every register-trellis and multilane code.
// Built with -ffp-contract=off (Makefile) so the channel's float/double arithmetic is not fused.
#include <array>
#include <utility>

#include "channel_dev.hpp"
#include "reg_codes.hpp"

namespace ccv {
namespace {

// LDS budget of the decision column array per wave (opt-in kernel): 20 KiB = 8 waves per CU
constexpr size_t kChanLdsBudget = 20 * 1024;

template <size_t I, bool HARD>
hipError_t launch_reg(const ChanArgs& a, int grid, hipStream_t stream) {
  constexpr CodeSpec C = kRegCodes[I];
  constexpr size_t word = (1u << (C.K - 1)) > 32 ? 8 : 4;
  const size_t lds = (size_t)(a.r.T - (C.K - 1)) * word * kRegThreads;
  if (!a.global_decisions && lds <= kChanLdsBudget)
    hipLaunchKernelGGL((viterbi_channel_lds<C, HARD>), dim3(grid), dim3(kRegThreads), lds, stream, a);
  else
    hipLaunchKernelGGL((viterbi_channel_reg<C, HARD>), dim3(grid), dim3(kRegThreads), 0, stream, a);
  return hipGetLastError();
}

template <size_t I, bool HARD>
hipError_t launch_multi(const ChanArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL((viterbi_channel_multi<kMultiCodes[I], HARD>), dim3(grid), dim3(kRegThreads), 0,
                     stream, a);
  return hipGetLastError();
}

template <bool HARD, size_t... I>
constexpr std::array<ChanLaunchFn, sizeof...(I)> make_reg(std::index_sequence<I...>) {
  return {&launch_reg<I, HARD>...};
}
template <bool HARD, size_t... I>
constexpr std::array<ChanLaunchFn, sizeof...(I)> make_multi(std::index_sequence<I...>) {
  return {&launch_multi<I, HARD>...};
}

template <size_t I>
hipError_t launch_frames(const ChanArgs& a, int grid, hipStream_t stream) {
  if constexpr (kMultiCodes[I].n == 2) {
    hipLaunchKernelGGL((channel_frames<kMultiCodes[I], false>), dim3(grid), dim3(kRegThreads), 0, stream, a);
    return hipGetLastError();
  } else {
    return hipErrorInvalidValue;
  }
}
template <size_t... I>
constexpr std::array<ChanLaunchFn, sizeof...(I)> make_frames(std::index_sequence<I...>) {
  return {&launch_frames<I>...};
}

constexpr auto kRegSoft = make_reg<false>(std::make_index_sequence<kNumRegCodes>{});
constexpr auto kRegHard = make_reg<true>(std::make_index_sequence<kNumRegCodes>{});
constexpr auto kMultiSoft = make_multi<false>(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kMultiHard = make_multi<true>(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kFrames = make_frames(std::make_index_sequence<kNumMultiCodes>{});

}  // namespace

const ChanLaunchFn* channel_frames_launchers() { return kFrames.data(); }

hipError_t launch_channel_frames_any(const ChanArgs& a, int n, int K, const uint64_t* polys, int gen,
                                     bool hard, hipStream_t stream) {
  CodeRT code{K, gen, {polys[0], n > 1 ? polys[1] : 0, n > 2 ? polys[2] : 0}};
  const dim3 grid((unsigned)((a.r.nblocks + kRegThreads - 1) / kRegThreads)), block(kRegThreads);
  switch ((hard ? 4 : 0) + n) {
    case 1: hipLaunchKernelGGL((channel_frames_rt<1, false>), grid, block, 0, stream, a, code); break;
    case 2: hipLaunchKernelGGL((channel_frames_rt<2, false>), grid, block, 0, stream, a, code); break;
    case 3: hipLaunchKernelGGL((channel_frames_rt<3, false>), grid, block, 0, stream, a, code); break;
    case 5: hipLaunchKernelGGL((channel_frames_rt<1, true>), grid, block, 0, stream, a, code); break;
    case 6: hipLaunchKernelGGL((channel_frames_rt<2, true>), grid, block, 0, stream, a, code); break;
    case 7: hipLaunchKernelGGL((channel_frames_rt<3, true>), grid, block, 0, stream, a, code); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

const ChanLaunchFn* channel_launchers(bool multi, bool hard) {
  if (multi) return hard ? kMultiHard.data() : kMultiSoft.data();
  return hard ? kRegHard.data() : kRegSoft.data();
}

}  // namespace ccv
