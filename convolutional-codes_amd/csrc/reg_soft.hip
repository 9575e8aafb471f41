// reg_soft.hip -- ahead-of-time instantiation of the soft-decision register-trellis kernel for
// every code in reg_codes.hpp (one translation unit per channel so they compile in parallel).
#include <array>
#include <utility>

#include "reg_codes.hpp"

namespace ccv {
namespace {

template <size_t I>
hipError_t launch(const RegArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(viterbi_soft_reg<kRegCodes[I]>, dim3(grid), dim3(kRegThreads), 0, stream, a);
  return hipGetLastError();
}

template <size_t... I>
constexpr std::array<RegLaunchFn, sizeof...(I)> make_table(std::index_sequence<I...>) {
  return {&launch<I>...};
}

constexpr auto kTable = make_table(std::make_index_sequence<kNumRegCodes>{});

}  // namespace

const RegLaunchFn* soft_reg_launchers() { return kTable.data(); }

}  // namespace ccv
