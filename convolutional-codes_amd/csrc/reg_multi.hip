// reg_multi.hip -- ahead-of-time instantiation of the multi-lane register-trellis kernel
// (acs_multi.hpp) for the K = 8 and K = 9 codes, soft and hard decision.
#include <array>
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
    // true parity (256 distinct metrics): two lanes per block (acs_multi2.hpp, 128 metrics per lane),
    // the main periods as a loop, the decisions through a per-wave slot, every cross-lane move through
    // ds_swizzle: 37.4-37.8 Gbit/s at 32 frames (profiles/r04t/). Measured and removed in round 5:
    // four lanes per block with ds_swizzle 33.3-33.6 (profiles/r04r/), the DPP cross phases 27.5 (two
    // lanes) / 27.9 (four), four lanes at 4 waves per SIMD 27.7.
    return launch_persistent(viterbi_multi2_slot<kMultiCodes[I], kPersistBlen>, a, ngroups, stream);
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
    return multi2_slot_bytes<kMultiCodes[I], kPersistBlen>();
}

template <size_t I>
int group_blocks() {
  if constexpr (!has_slot_kernel<I>()) return 0;
  else if constexpr (kMultiCodes[I].gen == GEN_REF_X86) return kRegThreads;   // one lane per block
  else return kRegThreads / 2;   // two lanes per block
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
constexpr auto kSoftWide = make_wide(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kSlotBytes = make_slot_bytes(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kSlotGroupBlocks = make_group_blocks(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kHard = make<true>(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kSoftRegDec = make_regdec<false>(std::make_index_sequence<kNumMultiCodes>{});
constexpr auto kHardRegDec = make_regdec<true>(std::make_index_sequence<kNumMultiCodes>{});

}  // namespace

const RegLaunchFn* multi_launchers(bool hard) { return hard ? kHard.data() : kSoft.data(); }

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
