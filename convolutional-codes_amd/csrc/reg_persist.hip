// reg_persist.hip -- ahead-of-time instantiation of the persistent K <= 7 register-trellis kernels
// (acs_persist.hpp) for the codes in reg_codes.hpp: soft for r = 1/2 codes, hard for every code.
#include <array>
#include <cstdlib>
#include <utility>

#include "acs_persist.hpp"
#include "reg_codes.hpp"

namespace ccv {
namespace {

template <size_t I>
constexpr bool kSoftOk = kRegCodes[I].n == 2;

// CCV_PERSIST_STAGE=1: the input chunks by coalesced buffer loads + ds_write instead of LDS-DMA (A/B)
inline bool persist_direct() {
  static const bool v = [] {
    const char* env = std::getenv("CCV_PERSIST_STAGE");
    return env != nullptr && env[0] == '1';
  }();
  return v;
}

// The staged kernel addresses its input through a buffer resource with 31-bit offsets: batches
// past 2^31 bytes of input run as several launches of whole groups (the error counter accumulates).
template <size_t I>
hipError_t launch_soft_direct(const RegArgs& a, int ngroups, hipStream_t stream) {
  constexpr auto kern = viterbi_soft_persist<kRegCodes[I], kPersistBlen, kPersistStage>;
  if (g_persist_query.active) return launch_persistent(kern, a, ngroups, stream);
  const size_t block_bytes = (size_t)a.T * 16;
  const int per = (int)(((size_t)0x7FFFFFFF / block_bytes) / kRegThreads);   // groups per launch
  for (int g0 = 0; g0 < ngroups; g0 += per) {
    const int ng = ngroups - g0 < per ? ngroups - g0 : per;
    RegArgs r = a;
    const size_t first = (size_t)g0 * kRegThreads;
    r.in = static_cast<const unsigned char*>(a.in) + first * block_bytes;
    r.out = a.out + first * (size_t)((a.T + 7) >> 3);
    r.info = a.info ? a.info + first * (size_t)((a.blen + 7) >> 3) : nullptr;
    r.nblocks = a.nblocks - (int)first < ng * kRegThreads ? a.nblocks - (int)first : ng * kRegThreads;
    const hipError_t e = launch_persistent(kern, r, ng, stream);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <size_t I>
hipError_t launch_soft(const RegArgs& a, int ngroups, hipStream_t stream) {
  if constexpr (kSoftOk<I>) {
    if (persist_direct()) return launch_soft_direct<I>(a, ngroups, stream);
    return launch_persistent(viterbi_soft_persist<kRegCodes[I], kPersistBlen>, a, ngroups, stream);
  } else {
    return hipErrorInvalidValue;
  }
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
