// reg_channel.hip -- ahead-of-time instantiation of the channel-fused decode kernels
// (channel_dev.hpp): BSC hard and AWGN soft (double-precision Box-Muller) for every register-trellis
// and multilane code; an AWGN launch with CCV_CHANNEL_NOISE_F32 goes to reg_channel_f32.hip.
// Built with -ffp-contract=off (Makefile) so the channel's float/double arithmetic is not fused.
#include "reg_channel.hpp"

namespace ccv {
namespace {

using namespace chan_impl;

constexpr auto kRegSoft = make_reg<false, false>(std::make_index_sequence<kNumRegCodes>{});
constexpr auto kRegHard = make_reg<true, false>(std::make_index_sequence<kNumRegCodes>{});
constexpr auto kMultiSoft = make_multi<false, false>(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kMultiHard = make_multi<true, false>(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kFrames = make_frames<false>(std::make_index_sequence<kNumMultiCodes>{});

// soft launches: the noise mode picks the instantiation
template <size_t I, bool MULTI>
hipError_t launch_soft(const ChanArgs& a, int grid, hipStream_t stream) {
  if (a.noise_f32) return channel_launchers_f32(MULTI)[I](a, grid, stream);
  return MULTI ? kMultiSoft[I](a, grid, stream) : kRegSoft[I](a, grid, stream);
}
template <size_t I>
hipError_t launch_frames_any_noise(const ChanArgs& a, int grid, hipStream_t stream) {
  if (a.noise_f32) return channel_frames_launchers_f32()[I](a, grid, stream);
  return kFrames[I](a, grid, stream);
}
template <bool MULTI, size_t... I>
constexpr std::array<ChanLaunchFn, sizeof...(I)> make_soft(std::index_sequence<I...>) {
  return {&launch_soft<I, MULTI>...};
}
template <size_t... I>
constexpr std::array<ChanLaunchFn, sizeof...(I)> make_frames_any(std::index_sequence<I...>) {
  return {&launch_frames_any_noise<I>...};
}
constexpr auto kRegSoftAny = make_soft<false>(std::make_index_sequence<kNumRegCodes>{});
constexpr auto kMultiSoftAny = make_soft<true>(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kFramesAny = make_frames_any(std::make_index_sequence<kNumMultiCodes>{});

}  // namespace

const ChanLaunchFn* channel_frames_launchers() { return kFramesAny.data(); }

hipError_t launch_channel_frames_any(const ChanArgs& a, int n, int K, const uint64_t* polys, int gen,
                                     bool hard, hipStream_t stream) {
  CodeRT code{K, gen, {polys[0], n > 1 ? polys[1] : 0, n > 2 ? polys[2] : 0}};
  if (hard) return launch_frames_rt<true, false>(a, n, code, stream);
  if (a.noise_f32) return launch_channel_frames_rt_f32(a, n, code, stream);
  return launch_frames_rt<false, false>(a, n, code, stream);
}

const ChanLaunchFn* channel_launchers(bool multi, bool hard) {
  if (multi) return hard ? kMultiHard.data() : kMultiSoftAny.data();
  return hard ? kRegHard.data() : kRegSoftAny.data();
}

}  // namespace ccv
