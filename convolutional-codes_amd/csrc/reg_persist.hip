// reg_persist.hip -- ahead-of-time instantiation of the persistent K <= 7 register-trellis kernels
// (acs_persist.hpp) for the codes in reg_codes.hpp: soft for r = 1/2 codes, hard for every code; both
// on the group queue (RegArgs::queue, the plan's) at K = 7, the static walk for smaller codes (persist_*_opt).
#include <array>
#include <utility>

#include "acs_persist.hpp"
#include "reg_codes.hpp"

namespace ccv {
namespace {

template <size_t I>
constexpr bool kSoftOk = kRegCodes[I].n == 2;

template <size_t I>
hipError_t launch_soft(const RegArgs& a, int ngroups, hipStream_t stream) {
  if constexpr (kSoftOk<I>) {
    return launch_persistent(viterbi_soft_persist<kRegCodes[I], kPersistBlen, persist_soft_opt<kRegCodes[I]>()>, a, ngroups, stream);
  } else {
    return hipErrorInvalidValue;
  }
}

template <size_t I>
hipError_t launch_hard(const RegArgs& a, int ngroups, hipStream_t stream) {
  return launch_persistent(viterbi_hard_persist<kRegCodes[I], kPersistBlen, 3, persist_hard_opt<kRegCodes[I]>()>, a, ngroups,
                           stream);
}

template <size_t... I>
constexpr std::array<RegLaunchFn, sizeof...(I)> make_soft(std::index_sequence<I...>) {
  return {(kSoftOk<I> ? &launch_soft<I> : nullptr)...};
}
template <size_t... I>
constexpr std::array<RegLaunchFn, sizeof...(I)> make_hard(std::index_sequence<I...>) {
  return {&launch_hard<I>...};
}

constexpr auto kSoft = make_soft(std::make_index_sequence<kNumRegCodes>{});
constexpr auto kHard = make_hard(std::make_index_sequence<kNumRegCodes>{});

}  // namespace

const RegLaunchFn* persist_launchers(bool hard) { return hard ? kHard.data() : kSoft.data(); }

}  // namespace ccv
