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

// register-resident decisions: r = 1/2 codes whose input-1 branch out of state 0 has a non-zero
// expected symbol (the neutral padding step of viterbi_soft_regdec needs it)
template <size_t I>
constexpr bool kRegDecOk = kRegCodes[I].n == 2 && expected_symbol(kRegCodes[I], 0, 1) != 0;

template <size_t I>
hipError_t launch_regdec(const RegArgs& a, int grid, hipStream_t stream) {
  if constexpr (kRegDecOk<I>) {
    hipLaunchKernelGGL((viterbi_soft_regdec<kRegCodes[I]>), dim3(grid), dim3(kRegThreads), 0, stream, a);
    return hipGetLastError();
  } else {
    return hipErrorInvalidValue;
  }
}

template <size_t... I>
constexpr std::array<RegLaunchFn, sizeof...(I)> make_regdec(std::index_sequence<I...>) {
  return {(kRegDecOk<I> ? &launch_regdec<I> : nullptr)...};
}

constexpr auto kBlockMajor = make_block_major(std::make_index_sequence<kNumRegCodes>{});
constexpr auto kRegDec = make_regdec(std::make_index_sequence<kNumRegCodes>{});
constexpr auto kStepMajor = make_step_major(std::make_index_sequence<kNumRegCodes>{});

}  // namespace

const RegLaunchFn* soft_regdec_launchers() { return kRegDec.data(); }

const RegLaunchFn* soft_reg_launchers(bool step_major) {
  return step_major ? kStepMajor.data() : kBlockMajor.data();
}

}  // namespace ccv
