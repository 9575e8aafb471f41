// reg_codes.hpp -- codes that get an ahead-of-time register-trellis kernel (acs_reg.hpp).
//
// The plan matches a code by its expected-symbol TABLE, not by its polynomials, so two descriptions
// with the same trellis (e.g. codebook code 0 in either generator mode) share one kernel. Codes
// not listed here run on the table-driven kernel (acs_generic.hpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#include "acs_reg.hpp"
#include "trellis.hpp"

namespace ccv {

#define CCV_CODE2(K, P0, P1, GEN) \
  CodeSpec { 2, K, {P0##ull, P1##ull, 0, 0, 0, 0, 0, 0}, GEN }
#define CCV_CODE3(K, P0, P1, P2, GEN) \
  CodeSpec { 3, K, {P0##ull, P1##ull, P2##ull, 0, 0, 0, 0, 0}, GEN }

inline constexpr CodeSpec kRegCodes[] = {
    // common/codebook.c:14-54, codes 0-3 and 5 (code 4 is the K=32 WSPR code: no Viterbi)
    CCV_CODE2(3, 0xA000000000000000, 0x6000000000000000, GEN_REF_X86),
    CCV_CODE2(4, 0xB000000000000000, 0xE000000000000000, GEN_REF_X86),
    CCV_CODE2(4, 0xB000000000000000, 0xE000000000000000, GEN_TRUE_PARITY),
    CCV_CODE2(5, 0xA800000000000000, 0xF000000000000000, GEN_REF_X86),
    CCV_CODE2(5, 0xA800000000000000, 0xF000000000000000, GEN_TRUE_PARITY),
    CCV_CODE2(6, 0xB400000000000000, 0xE800000000000000, GEN_REF_X86),
    CCV_CODE2(6, 0xB400000000000000, 0xE800000000000000, GEN_TRUE_PARITY),
    CCV_CODE3(3, 0xA000000000000000, 0xC000000000000000, 0x2000000000000000, GEN_REF_X86),
    // K=7 (171,133)_8, the benchmark code (BASELINE.json configs 2 and 4)
    CCV_CODE2(7, 0xF200000000000000, 0xB600000000000000, GEN_REF_X86),
    CCV_CODE2(7, 0xF200000000000000, 0xB600000000000000, GEN_TRUE_PARITY),
};
inline constexpr size_t kNumRegCodes = sizeof(kRegCodes) / sizeof(kRegCodes[0]);

// Codes with 128 / 256 states: multi-lane register kernel (acs_multi.hpp), 2 / 4 lanes per block.
inline constexpr CodeSpec kMultiCodes[] = {
    // K=8 (371,247)_8 and K=9 (561,753)_8 (BASELINE.json config 3)
    CCV_CODE2(8, 0xF900000000000000, 0xA700000000000000, GEN_REF_X86),
    CCV_CODE2(8, 0xF900000000000000, 0xA700000000000000, GEN_TRUE_PARITY),
    CCV_CODE2(9, 0xB880000000000000, 0xF580000000000000, GEN_REF_X86),
    CCV_CODE2(9, 0xB880000000000000, 0xF580000000000000, GEN_TRUE_PARITY),
};
inline constexpr size_t kNumMultiCodes = sizeof(kMultiCodes) / sizeof(kMultiCodes[0]);

using RegLaunchFn = hipError_t (*)(const RegArgs&, int grid, hipStream_t stream);
const RegLaunchFn* soft_reg_launchers(bool step_major);   // [kNumRegCodes], reg_soft.hip
// [kNumRegCodes], nullptr where the code has no register-resident-decision kernel; valid for
// block-major input with T <= 8 * kRegDecMaxChunks and no decision export (reg_soft.hip)
const RegLaunchFn* soft_regdec_launchers();
const RegLaunchFn* hard_reg_launchers();   // [kNumRegCodes], reg_hard.hip
// [kNumRegCodes] persistent kernels (acs_persist.hpp; the int argument is the number of 64-block
// groups, the launcher sizes the grid to the resident waves), nullptr where a code has none; valid
// for blen == kPersistBlen, no decision export; soft: block-major r = 1/2 input, hard: whole groups
// only (reg_persist.hip)
constexpr int kPersistBlen = 40;   // common/codebook.c:66-68: every Viterbi code of the codebook
const RegLaunchFn* persist_launchers(bool hard);
const RegLaunchFn* multi_launchers(bool hard);   // [kNumMultiCodes], reg_multi.hip
// [kNumMultiCodes], register-resident decisions (acs_multi.hpp viterbi_multi_regdec); valid for
// T <= multi_regdec_max_steps(K) and no decision export (reg_multi.hip)
const RegLaunchFn* multi_regdec_launchers(bool hard);
int multi_regdec_max_steps(int K);
// [kNumMultiCodes] persistent soft kernels whose decisions go through a per-wave scratch slot,
// nullptr where a code has none: the K = 9 x86-idiom code runs one lane per block (acs_wide.hpp
// viterbi_wide_persist: 156 distinct metrics fit one lane's VGPRs), the true-parity K = 9 code two
// lanes per block with its main periods as a loop (acs_multi2.hpp viterbi_multi2_slot). int argument =
// groups of multi_wide_group_blocks(index) blocks; RegArgs::dec = one scratch slot of
// multi_wide_slot_bytes(index) per resident wave of the grid. Valid for blen == kPersistBlen,
// block-major input, no decision export (reg_multi.hip)
const RegLaunchFn* multi_wide_launchers();
size_t multi_wide_slot_bytes(int index);
int multi_wide_group_blocks(int index);

struct ChanArgs;
using ChanLaunchFn = hipError_t (*)(const ChanArgs&, int grid, hipStream_t stream);
// channel-fused decode kernels: [kNumRegCodes] or [kNumMultiCodes], reg_channel.hip
const ChanLaunchFn* channel_launchers(bool multi, bool hard);
// [kNumMultiCodes] frames-only soft channel (channel_dev.hpp channel_frames): info bytes and the
// decoder input [nb][T][4] written to ChanArgs::info_out / ch_out, grid = one lane per block
const ChanLaunchFn* channel_frames_launchers();
// frames only for any code with n <= 3 and K <= 64 (channel_dev.hpp channel_frames_rt; one lane per
// block, ChanArgs::info_out and ch_out required), reg_channel.hip
hipError_t launch_channel_frames_any(const ChanArgs& a, int n, int K, const uint64_t* polys, int gen,
                                     bool hard, hipStream_t stream);

}  // namespace ccv
