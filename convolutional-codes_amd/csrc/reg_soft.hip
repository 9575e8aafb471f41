// reg_soft.hip -- ahead-of-time instantiation of the soft-decision register-trellis kernel for
// every code in reg_codes.hpp (one translation unit per channel so they compile in parallel).
#include <array>
#include <utility>

#include "reg_codes.hpp"

namespace ccv {
namespace {

template <size_t I, int MODE, int PF>
hipError_t launch(const RegArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL((viterbi_soft_reg<kRegCodes[I], MODE, PF>), dim3(grid), dim3(kRegThreads), 0,
                     stream, a);
  return hipGetLastError();
}

template <size_t... I>
constexpr std::array<RegLaunchFn, sizeof...(I)> make_block_major(std::index_sequence<I...>) {
  return {&launch<I, kSoftMode<(1 << kRegCodes[I].n)>, kSoftPF<(1 << kRegCodes[I].n)>>...};
}

template <size_t... I>
constexpr std::array<RegLaunchFn, sizeof...(I)> make_step_major(std::index_sequence<I...>) {
  return {&launch<I, kLoadStepMajor, kSoftStepMajorPF>...};
}

constexpr auto kBlockMajor = make_block_major(std::make_index_sequence<kNumRegCodes>{});
constexpr auto kStepMajor = make_step_major(std::make_index_sequence<kNumRegCodes>{});

}  // namespace

const RegLaunchFn* soft_reg_launchers(bool step_major) {
  return step_major ? kStepMajor.data() : kBlockMajor.data();
}

}  // namespace ccv
