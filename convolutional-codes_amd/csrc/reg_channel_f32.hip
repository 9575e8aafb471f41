// reg_channel_f32.hip -- the AWGN channel-fused kernels with the opt-in fp32 Box-Muller
// (CCV_CHANNEL_NOISE_F32; channel_dev.hpp ChannelSource<..., F32 = true>), instantiated apart from
// reg_channel.hip so the two compile in parallel. -ffp-contract=off as reg_channel.hip.
#include "reg_channel.hpp"

namespace ccv {
namespace {

using namespace chan_impl;

constexpr auto kRegSoftF32 = make_reg<false, true>(std::make_index_sequence<kNumRegCodes>{});
constexpr auto kMultiSoftF32 = make_multi<false, true>(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kFramesF32 = make_frames<true>(std::make_index_sequence<kNumMultiCodes>{});

}  // namespace

const ChanLaunchFn* channel_launchers_f32(bool multi) { return multi ? kMultiSoftF32.data() : kRegSoftF32.data(); }
const ChanLaunchFn* channel_frames_launchers_f32() { return kFramesF32.data(); }
hipError_t launch_channel_frames_rt_f32(const ChanArgs& a, int n, const CodeRT& code, hipStream_t stream) {
  return launch_frames_rt<false, true>(a, n, code, stream);
}

}  // namespace ccv
