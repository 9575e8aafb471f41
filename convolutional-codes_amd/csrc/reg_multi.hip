// reg_multi.hip -- ahead-of-time instantiation of the multi-lane register-trellis kernel
// (acs_multi.hpp) for the K = 8 and K = 9 codes, soft and hard decision.
#include <array>
#include <cstdlib>
#include <utility>

#include "acs_multi.hpp"
#include "acs_multi2.hpp"
#include "acs_wide.hpp"
#include "reg_codes.hpp"

namespace ccv {
namespace {

template <size_t I, bool HARD>
hipError_t launch(const RegArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL((viterbi_multi<kMultiCodes[I], HARD>), dim3(grid), dim3(kRegThreads), 0, stream, a);
  return hipGetLastError();
}

template <bool HARD, size_t... I>
constexpr std::array<RegLaunchFn, sizeof...(I)> make(std::index_sequence<I...>) {
  return {&launch<I, HARD>...};
}

// two waves per SIMD (a few scratch spills) measured 24.4 Gbit/s at K=9 against 18.4 for the
// one-wave build that spills to AGPRs only (profiles/r01_k9_regdec.txt)
template <size_t I, bool HARD>
hipError_t launch_regdec(const RegArgs& a, int grid, hipStream_t stream) {
  hipLaunchKernelGGL((viterbi_multi_regdec<kMultiCodes[I], HARD, 2>), dim3(grid), dim3(kRegThreads), 0,
                     stream, a);
  return hipGetLastError();
}

template <bool HARD, size_t... I>
constexpr std::array<RegLaunchFn, sizeof...(I)> make_regdec(std::index_sequence<I...>) {
  return {&launch_regdec<I, HARD>...};
}

template <size_t I>
hipError_t launch_persist(const RegArgs& a, int ngroups, hipStream_t stream) {
  if constexpr (kMultiCodes[I].K == 9 && kMultiCodes[I].n == 2)
    // lane bits at physical state bits {0, 3}, two periods of decisions in LDS (3 waves per SIMD):
    // 0.952x the time of the {6, 7} all-VGPR layout (tools/k9_bench.hip, profiles/r03_k9_layouts.txt)
    return launch_persistent(viterbi_multi_persist<kMultiCodes[I], kPersistBlen, 0, 2, 0, 3>, a, ngroups, stream);
  else
    return hipErrorInvalidValue;
}

template <size_t... I>
constexpr std::array<RegLaunchFn, sizeof...(I)> make_persist(std::index_sequence<I...>) {
  return {((kMultiCodes[I].K == 9 && kMultiCodes[I].n == 2) ? &launch_persist<I> : nullptr)...};
}

// The true-parity K = 9 slot kernel: two lanes per block (default) or four (CCV_K9_TRUE_LANES=4, A/B)
inline bool k9_true_four_lanes() {
  static const bool four = [] {
    const char* env = std::getenv("CCV_K9_TRUE_LANES");
    return env != nullptr && env[0] == '4';
  }();
  return four;
}

// The four-lane slot kernel's waves per SIMD: 3 (134 VGPRs) or 4 (CCV_K9_SLOT_WAVES=4: 128 VGPRs, a
// few spills outside the main loop)
inline int k9_slot_waves() {
  static const int w = [] {
    const char* env = std::getenv("CCV_K9_SLOT_WAVES");
    return env != nullptr && env[0] == '4' ? 4 : 3;
  }();
  return w;
}

// the slot kernels' cross-lane phases through ds_swizzle (default) or DPP (CCV_K9_SLOT_XSWZ=0)
inline bool k9_slot_xswz() {
  static const bool v = [] {
    const char* env = std::getenv("CCV_K9_SLOT_XSWZ");
    return env == nullptr || env[0] != '0';
  }();
  return v;
}

// Codes with a slot kernel (decisions through a per-wave scratch slot): K = 9 r = 1/2
template <size_t I>
constexpr bool has_slot_kernel() {
  return kMultiCodes[I].K == 9 && kMultiCodes[I].n == 2;
}

template <size_t I>
hipError_t launch_wide(const RegArgs& a, int ngroups, hipStream_t stream) {
  if constexpr (has_slot_kernel<I>() && kMultiCodes[I].gen == GEN_REF_X86)
    // one lane per block, one decision per value-numbering class (156 of 256 states, twins.hpp)
    // through a per-wave scratch slot: ~0.57x the time of the four-lane kernel at 32 frames,
    // bit-identical (tools/k9_bench.hip, profiles/r03_k9_wide*.txt)
    return launch_persistent(viterbi_wide_persist<kMultiCodes[I], kPersistBlen, 0, 2>, a, ngroups, stream);
  else if constexpr (has_slot_kernel<I>())
    // true parity (256 distinct metrics), the main periods as a loop with the decisions through a
    // per-wave slot. Production: two lanes per block (acs_multi2.hpp, 128 metrics per lane), every
    // cross-lane move through ds_swizzle: 37.4-37.8 Gbit/s at 32 frames (profiles/r04t/) against
    // 33.3-33.6 for four lanes with ds_swizzle (acs_multi.hpp viterbi_multi_slot, CCV_K9_TRUE_LANES=4,
    // profiles/r04r/). A/B forms: CCV_K9_SLOT_XSWZ=0 the DPP cross phases (two lanes 27.5, four
    // 27.9), CCV_K9_SLOT_WAVES=4 the 4-waves-per-SIMD four-lane build (27.7).
    if (!k9_true_four_lanes())
      return k9_slot_xswz()
                 ? launch_persistent(viterbi_multi2_slot<kMultiCodes[I], kPersistBlen, true>, a, ngroups, stream)
                 : launch_persistent(viterbi_multi2_slot<kMultiCodes[I], kPersistBlen, false>, a, ngroups, stream);
    else if (k9_slot_xswz())
      return launch_persistent(viterbi_multi_slot<kMultiCodes[I], kPersistBlen, 3, true>, a, ngroups, stream);
    else if (k9_slot_waves() == 4)
      return launch_persistent(viterbi_multi_slot<kMultiCodes[I], kPersistBlen, 4>, a, ngroups, stream);
    else
      return launch_persistent(viterbi_multi_slot<kMultiCodes[I], kPersistBlen, 3>, a, ngroups, stream);
  else
    return hipErrorInvalidValue;
}

template <size_t... I>
constexpr std::array<RegLaunchFn, sizeof...(I)> make_wide(std::index_sequence<I...>) {
  return {(has_slot_kernel<I>() ? &launch_wide<I> : nullptr)...};
}

template <size_t I>
size_t slot_bytes() {
  if constexpr (!has_slot_kernel<I>()) return 0;
  else if constexpr (kMultiCodes[I].gen == GEN_REF_X86) return wide_slot_bytes<kMultiCodes[I], 2>(kPersistBlen);
  else
    return k9_true_four_lanes() ? multi_slot_bytes<kMultiCodes[I], kPersistBlen>()
                                : multi2_slot_bytes<kMultiCodes[I], kPersistBlen>();
}

template <size_t I>
int group_blocks() {
  if constexpr (!has_slot_kernel<I>()) return 0;
  else if constexpr (kMultiCodes[I].gen == GEN_REF_X86) return kRegThreads;   // one lane per block
  else return k9_true_four_lanes() ? kRegThreads / 4 : kRegThreads / 2;
}

template <size_t... I>
constexpr std::array<size_t (*)(), sizeof...(I)> make_slot_bytes(std::index_sequence<I...>) {
  return {&slot_bytes<I>...};
}

template <size_t... I>
constexpr std::array<int (*)(), sizeof...(I)> make_group_blocks(std::index_sequence<I...>) {
  return {&group_blocks<I>...};
}

constexpr auto kSoft = make<false>(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kSoftPersist = make_persist(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kSoftWide = make_wide(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kSlotBytes = make_slot_bytes(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kSlotGroupBlocks = make_group_blocks(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kHard = make<true>(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kSoftRegDec = make_regdec<false>(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kHardRegDec = make_regdec<true>(std::make_index_sequence<kNumMultiCodes>{});

}  // namespace

const RegLaunchFn* multi_launchers(bool hard) { return hard ? kHard.data() : kSoft.data(); }

const RegLaunchFn* multi_persist_launchers() { return kSoftPersist.data(); }

const RegLaunchFn* multi_wide_launchers() { return kSoftWide.data(); }

size_t multi_wide_slot_bytes(int index) { return kSlotBytes[(size_t)index](); }

int multi_wide_group_blocks(int index) { return kSlotGroupBlocks[(size_t)index](); }

const RegLaunchFn* multi_regdec_launchers(bool hard) {
  return hard ? kHardRegDec.data() : kSoftRegDec.data();
}

int multi_regdec_max_steps(int K) {
  const int n = K - 1;
  return (kMultiRegDecSteps + n - 1) / n * n;
}

}  // namespace ccv
