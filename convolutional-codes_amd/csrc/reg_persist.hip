// reg_persist.hip -- ahead-of-time instantiation of the persistent K <= 7 register-trellis kernels
// (acs_persist.hpp) for the codes in reg_codes.hpp: soft for r = 1/2 codes, hard for every code.
#include <array>
#include <cstdlib>
#include <utility>

#include "acs_persist.hpp"
#include "reg_codes.hpp"

namespace ccv {
namespace {

// Resident waves of a one-wave-per-workgroup kernel on the current device (occupancy x CUs), cached
// per kernel and device.
template <class Kern>
int resident_groups(Kern kernel) {
  static int cached[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cached[dev] > 0) return cached[dev];
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kRegThreads, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  // CCV_PERSIST_WAVES_PER_CU caps the resident waves per CU (occupancy studies)
  if (const char* env = std::getenv("CCV_PERSIST_WAVES_PER_CU")) {
    const int cap = std::atoi(env);
    if (cap > 0 && cap < per_cu) per_cu = cap;
  }
  // every wave walks the same number of groups: the same number of waves on each of a CU's four
  // SIMDs, or the SIMDs holding one more wave finish a third later (10 per CU: 0.50 vs 0.39 ms)
  if (per_cu >= 4) per_cu -= per_cu % 4;
  cached[dev] = per_cu * cus;
  return cached[dev];
}

template <class Kern>
hipError_t launch_persistent(Kern kernel, const RegArgs& a, int ngroups, hipStream_t stream) {
  if (ngroups <= 0) return hipSuccess;
  int resident = resident_groups(kernel);
  if (resident <= 0) return hipErrorInvalidDeviceFunction;
  const int grid = ngroups < resident ? ngroups : resident;
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(kRegThreads), 0, stream, a, ngroups);
  return hipGetLastError();
}

template <size_t I>
constexpr bool kSoftOk = kRegCodes[I].n == 2;

template <size_t I>
hipError_t launch_soft(const RegArgs& a, int ngroups, hipStream_t stream) {
  if constexpr (kSoftOk<I>) return launch_persistent(viterbi_soft_persist<kRegCodes[I], kPersistBlen>, a, ngroups, stream);
  else return hipErrorInvalidValue;
}

template <size_t I>
hipError_t launch_hard(const RegArgs& a, int ngroups, hipStream_t stream) {
  return launch_persistent(viterbi_hard_persist<kRegCodes[I], kPersistBlen>, a, ngroups, stream);
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
