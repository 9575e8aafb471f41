// core.hip -- libccv_core.so: plans, kernel selection, launches and the ccv_* C ABI (include/ccv.h).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "acs_generic.hpp"
#include "acs_latency.hpp"
#include "acs_persist.hpp"
#include "channel_dev.hpp"
#include "fano_dev.hpp"
#include "stack_dev.hpp"
#include "ccv.h"
#include "reg_codes.hpp"
#include "trellis.hpp"

namespace ccv {
constexpr size_t kHostLatencyMaxBlocks = 64;   // ccv_decode_host batches decoded by the generic kernel
constexpr size_t kServiceMaxBlocks = 4;        // ... and by the resident streaming service
hipError_t launch_stack(const StackArgs& a, bool hard, hipStream_t s);   // stack.hip
bool stack_rows_eligible(int n, int K, int T);                           // stack.hip
bool stack_symtab_eligible(int n, int K, int T);                         // stack.hip
hipError_t launch_stack_symtab(uint16_t* tab, const StackArgs& a, hipStream_t s);   // stack.hip
hipError_t launch_fano(const FanoArgs& a, bool hard, hipStream_t s);     // stack.hip
size_t fano_order_bytes(int nblocks);                                    // stack.hip
hipError_t launch_fano_order(const FanoArgs& a, void* scratch, size_t bytes, const uint32_t** order,
                             hipStream_t s);                             // stack.hip
}

namespace {

thread_local std::string g_last_error;

int fail(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return -1;
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return fail("%s: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                      __FILE__, __LINE__);                             \
  } while (0)

struct DeviceBuffer {
  void* ptr = nullptr;
  size_t bytes = 0;
  int grow(size_t need, hipStream_t sync_stream) {
    if (need <= bytes) return 0;
    if (ptr) {
      HIP_TRY(hipStreamSynchronize(sync_stream));
      HIP_TRY(hipFree(ptr));
      ptr = nullptr;
      bytes = 0;
    }
    HIP_TRY(hipMalloc(&ptr, need));
    bytes = need;
    return 0;
  }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
  }
};

// Page-locked host memory the device reads and writes directly (zero-copy): the streaming decode
// path's per-plan staging, so a single block costs one kernel launch and one synchronise.
struct PinnedBuffer {
  void* host = nullptr;
  void* dev = nullptr;
  size_t bytes = 0;
  int grow(size_t need, hipStream_t sync_stream, unsigned flags = hipHostMallocDefault) {
    if (need <= bytes) return 0;
    if (host) {
      HIP_TRY(hipStreamSynchronize(sync_stream));
      HIP_TRY(hipHostFree(host));
      host = dev = nullptr;
      bytes = 0;
    }
    HIP_TRY(hipHostMalloc(&host, need, flags));
    memset(host, 0, need);
    HIP_TRY(hipHostGetDevicePointer(&dev, host, 0));
    bytes = need;
    return 0;
  }
  void release() {
    if (host) (void)hipHostFree(host);
    host = dev = nullptr;
    bytes = 0;
  }
};

}  // namespace

struct ccv_plan {
  ccv_plan_desc d{};
  uint64_t polys[ccv::kMaxN] = {};
  std::vector<uint8_t> exp;          // [S][2]
  int reg_index = -1;                // kRegCodes index, or -1
  int multi_index = -1;              // kMultiCodes index (K = 8, 9), or -1
  bool stack = false;                // stack (sequential) decoder plan
  bool fano = false;                 // Fano decoder plan
  DeviceBuffer counter;              // Fano, stack rows: block work counter
  DeviceBuffer symtab;               // stack rows: expected-symbol table (built on first use)
  DeviceBuffer order;                // Fano, soft: noisiest-first queue order scratch
  DeviceBuffer park;                 // Fano: parked searches of the two-pass schedule
  bool symtab_ready = false;
  float metric_weight = 0.0f;        // stack, soft: code_param.metric_weight
  int32_t bit_metrics[2] = {0, 0};   // stack, hard: code_param.bit_metrics
  bool step_major = false;           // soft input layout [T][nblocks][2^n] (CCV_FLAG_STEP_MAJOR)
  bool global_decisions = false;     // CCV_FLAG_GLOBAL_DECISIONS
  bool no_persistent = false;        // CCV_FLAG_NO_PERSISTENT
  int generic_spt = 1, generic_threads = 64, generic_chunk = 1;
  size_t generic_lds = 0;
  uint8_t* d_exp = nullptr;          // device copy of exp (generic kernel)
  DeviceBuffer dec;                  // register-kernel decision scratch
  DeviceBuffer host_in, host_out, host_pm;   // staging for ccv_decode_host
  PinnedBuffer lat_in, lat_out, lat_pm;        // zero-copy staging of small ccv_decode_host calls
  PinnedBuffer svc_mb, svc_in, svc_out, svc_pm; // streaming service: fine-grained mailbox and staging
  hipStream_t svc_stream = nullptr;            // the service kernel's own stream
  bool svc_running = false;
  uint32_t svc_seq = 0;
  bool generic_ok = false;                     // the generic kernel can run this code (d_exp built)
  DeviceBuffer sim_info, sim_out;             // ccv_simulate_device scratch (caller passed none)
  DeviceBuffer sim_frames;                    // ccv_simulate_device: K = 9 frames ahead of the wide decode
  DeviceBuffer hard_rows;                     // K = 9 BSC: the symbols as Hamming-distance rows (hard_rows)
  DeviceBuffer queue;                         // persistent kernels' group queue (acs_persist.hpp GroupQueue)
  hipStream_t stream = nullptr;      // plan-owned stream for ccv_decode_host
  // ccv_plan_set_option (include/ccv.h): kernel A/B switches per plan; defaults = production paths
  struct Options {
    int stack_kernel = 0;            // 0 persistent rows, 1 one search per wave
    int stack_row_lanes = 0;         // 0 auto, 8, 16
    int stack_keys = 1;              // hard rows: packed metric / index keys where they fit
    int stack_symtab = 1;            // rows: expected-symbol table
    int fano_rows = -1;              // -1 auto, else ccv::kRows*
    int fano_symtab = -1;            // -1 auto (hard input), 0 / 1
    int fano_order = 1;              // soft: noisiest first
    long long fano_cap = -1;         // -1 default 4000 x T, 0 one pass
    int fano_count_moves = 0;        // diagnostics: iterations = moves
    int channel_fused = 0;           // K = 8 / 9 device channel: fused multilane kernel
    int channel_lds_decisions = -1;  // device channel K <= 7: -1 auto (BSC LDS, AWGN HBM), 0, 1
    int fano_input = 0;              // soft Fano: 0 the demapper's distances, 1 received points (I/Q)
  } opt;
};

namespace {

// Decision columns: one per wave lane (nblocks * lanes), rounded up to whole waves.
size_t padded_columns(const ccv_plan& p, size_t nblocks) {
  const size_t cols = nblocks * (size_t)p.d.lanes;
  return (cols + ccv::kRegThreads - 1) / ccv::kRegThreads * ccv::kRegThreads;
}

size_t decision_bytes(const ccv_plan& p, size_t nblocks) {
  return padded_columns(p, nblocks) * (size_t)p.d.steps * (size_t)p.d.decision_word_bytes;
}

bool register_path(const ccv_plan& p) { return p.reg_index >= 0 || p.multi_index >= 0; }

// The register-resident-decision kernel (acs_reg.hpp viterbi_soft_regdec, acs_multi.hpp
// viterbi_multi_regdec), or nullptr.
ccv::RegLaunchFn regdec_kernel(const ccv_plan& p, bool export_decisions) {
  if (p.global_decisions || export_decisions) return nullptr;
  if (p.multi_index >= 0)
    return p.d.steps <= ccv::multi_regdec_max_steps(p.d.K)
               ? ccv::multi_regdec_launchers(p.d.channel == CCV_HARD)[p.multi_index]
               : nullptr;
  if (p.reg_index < 0 || p.d.channel != CCV_SOFT || p.step_major ||
      p.d.steps > 8 * ccv::kRegDecMaxChunks)
    return nullptr;
  return ccv::soft_regdec_launchers()[p.reg_index];
}

// The persistent K = 9 soft kernel with a per-wave decision slot (acs_wide.hpp one lane per block for
// the x86-idiom code, acs_multi2.hpp viterbi_multi2_slot two lanes per block for true parity), or
// nullptr: codebook block length, block-major input, decisions not exported.
// (BSC plans too: ccv_decode_device first turns their symbols into Hamming-distance rows, hard_rows)
ccv::RegLaunchFn wide_kernel(const ccv_plan& p, bool export_decisions) {
  if (p.no_persistent || p.global_decisions || export_decisions || p.step_major ||
      p.d.blen != ccv::kPersistBlen || p.multi_index < 0 || p.d.n != 2)
    return nullptr;
  return ccv::multi_wide_launchers()[p.multi_index];
}

// BSC symbols -> the soft K = 9 persistent kernels' input rows: entry k = popcount(k ^ (sym & 3)),
// the Hamming branch metric of expected symbol k (binary-symmetric-channel/viterbi-decoder.c:69-72,
// the symbol masked as at :237). Their fp32 metrics are exact on these small integers, and the
// reference's 0xFF00 saturation only binds at the growth steps' unreachable states, where it and the
// soft kernels' +inf give the same decisions.
__global__ __launch_bounds__(256) void hard_rows(const uint8_t* __restrict__ in, float4* __restrict__ out, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const uint32_t s = in[i] & 3u;
    out[i] = make_float4((float)__builtin_popcount(s), (float)__builtin_popcount(s ^ 1u),
                         (float)__builtin_popcount(s ^ 2u), (float)__builtin_popcount(s ^ 3u));
  }
}

// The persistent kernel (acs_persist.hpp K <= 7, acs_wide.hpp / acs_multi2.hpp K = 9), or nullptr:
// codebook block length, block-major input, decisions not exported.
ccv::RegLaunchFn persist_kernel(const ccv_plan& p, bool export_decisions) {
  if (p.no_persistent || p.global_decisions || export_decisions || p.step_major ||
      p.d.blen != ccv::kPersistBlen)
    return nullptr;
  if (const ccv::RegLaunchFn wide = wide_kernel(p, export_decisions)) return wide;
  if (p.multi_index >= 0) return nullptr;   // K = 8 and other K = 9 codes: the multilane kernels
  if (p.reg_index < 0) return nullptr;
  return ccv::persist_launchers(p.d.channel == CCV_HARD)[p.reg_index];
}

int find_reg_kernel(const ccv_plan& p) {
  using namespace ccv;
  const int S = 1 << (p.d.K - 1);
  std::vector<uint8_t> tab(2 * (size_t)S);
  for (size_t i = 0; i < kNumRegCodes; ++i) {
    const CodeSpec& c = kRegCodes[i];
    if (c.n != p.d.n || c.K != p.d.K) continue;
    build_trellis(c.n, c.K, c.poly, c.gen, tab.data());
    if (tab == p.exp) return (int)i;
  }
  return -1;
}

int find_multi_kernel(const ccv_plan& p) {
  using namespace ccv;
  const int S = 1 << (p.d.K - 1);
  std::vector<uint8_t> tab(2 * (size_t)S);
  for (size_t i = 0; i < kNumMultiCodes; ++i) {
    const CodeSpec& c = kMultiCodes[i];
    if (c.n != p.d.n || c.K != p.d.K) continue;
    build_trellis(c.n, c.K, c.poly, c.gen, tab.data());
    if (tab == p.exp) return (int)i;
  }
  return -1;
}

template <int SPT, bool HARD>
hipError_t launch_generic_t(const ccv::GenericArgs& a, const ccv_plan& p, size_t nblocks,
                            hipStream_t s) {
  const void* fn = reinterpret_cast<const void*>(&ccv::viterbi_generic<SPT, HARD>);
  if (p.generic_lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)p.generic_lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((ccv::viterbi_generic<SPT, HARD>), dim3((unsigned)nblocks),
                     dim3(p.generic_threads), p.generic_lds, s, a);
  return hipGetLastError();
}

template <bool HARD>
hipError_t launch_generic(const ccv::GenericArgs& a, const ccv_plan& p, size_t nblocks,
                          hipStream_t s) {
  switch (p.generic_spt) {
    case 1: return launch_generic_t<1, HARD>(a, p, nblocks, s);
    case 2: return launch_generic_t<2, HARD>(a, p, nblocks, s);
    case 4: return launch_generic_t<4, HARD>(a, p, nblocks, s);
    default: return launch_generic_t<8, HARD>(a, p, nblocks, s);
  }
}

bool latency_kernel_ok(const ccv_plan& p) { return p.d.K >= 2 && p.d.K <= ccv::kLatencyMaxK; }

template <bool HARD>
void launch_latency(const ccv::GenericArgs& a, const ccv_plan& p, int nblocks, size_t lds) {
  const dim3 g((unsigned)nblocks), b(64);
  switch (p.d.K - 1) {
    case 1: hipLaunchKernelGGL((ccv::viterbi_latency<HARD, 1>), g, b, lds, p.stream, a); break;
    case 2: hipLaunchKernelGGL((ccv::viterbi_latency<HARD, 2>), g, b, lds, p.stream, a); break;
    case 3: hipLaunchKernelGGL((ccv::viterbi_latency<HARD, 3>), g, b, lds, p.stream, a); break;
    case 4: hipLaunchKernelGGL((ccv::viterbi_latency<HARD, 4>), g, b, lds, p.stream, a); break;
    case 5: hipLaunchKernelGGL((ccv::viterbi_latency<HARD, 5>), g, b, lds, p.stream, a); break;
    default: hipLaunchKernelGGL((ccv::viterbi_latency<HARD, 6>), g, b, lds, p.stream, a); break;
  }
}

size_t latency_lds(const ccv_plan& p) {
  return ccv::latency_lds_bytes(p.d.n, p.d.steps, p.d.channel == CCV_HARD);
}

template <int SPT, bool HARD, int LATN>
hipError_t launch_service_t(const ccv::GenericArgs& a, const ccv_plan& p, ccv::ServiceMailbox* mb,
                            uint32_t served, hipStream_t s) {
  const void* fn = reinterpret_cast<const void*>(&ccv::viterbi_service<SPT, HARD, LATN>);
  const size_t lds = LATN ? latency_lds(p) : p.generic_lds;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  // idle CCV_SERVICE_IDLE_MS (default 20 ms) of the 100 MHz real-time counter, at most 2,000,000 polls
  // (~2-4 s): while it idles the kernel keeps one workgroup resident and a device-wide synchronise
  // in the process waits for it (include/ccv.h)
  uint64_t idle_ticks = 2000000;
  if (const char* env = std::getenv("CCV_SERVICE_IDLE_MS")) {
    const long ms = std::atol(env);
    idle_ticks = ms <= 0 ? 1 : (uint64_t)(ms > 2000 ? 2000 : ms) * 100000u;
  }
  hipLaunchKernelGGL((ccv::viterbi_service<SPT, HARD, LATN>), dim3(1), dim3(LATN ? 64 : p.generic_threads), lds, s,
                     a, mb, served, idle_ticks, (uint32_t)2000000);
  return hipGetLastError();
}

template <bool HARD>
hipError_t launch_service(const ccv::GenericArgs& a, const ccv_plan& p, ccv::ServiceMailbox* mb,
                          uint32_t served, hipStream_t s) {
  if (latency_kernel_ok(p)) {
    switch (p.d.K - 1) {
      case 1: return launch_service_t<1, HARD, 1>(a, p, mb, served, s);
      case 2: return launch_service_t<1, HARD, 2>(a, p, mb, served, s);
      case 3: return launch_service_t<1, HARD, 3>(a, p, mb, served, s);
      case 4: return launch_service_t<1, HARD, 4>(a, p, mb, served, s);
      case 5: return launch_service_t<1, HARD, 5>(a, p, mb, served, s);
      default: return launch_service_t<1, HARD, 6>(a, p, mb, served, s);
    }
  }
  switch (p.generic_spt) {
    case 1: return launch_service_t<1, HARD, 0>(a, p, mb, served, s);
    case 2: return launch_service_t<2, HARD, 0>(a, p, mb, served, s);
    case 4: return launch_service_t<4, HARD, 0>(a, p, mb, served, s);
    default: return launch_service_t<8, HARD, 0>(a, p, mb, served, s);
  }
}

// The achievable-HBM ceiling of the roofline ("a measured copy-kernel ceiling"): a
// streaming pass over a buffer in 16-byte lanes, U non-temporal global_load_dwordx4 in flight per
// lane, each wave-instruction 1 KiB of consecutive bytes. COPY stores every vector (non-temporal
// global_store_dwordx4); otherwise the loads are folded into one XOR per lane and nothing is stored
// but a never-taken sink write (the read-only stream the decode kernels make of their input). The
// variants measured on the 1.9 GB headline batch (tools/hbm_probe.hip, profiles/r05b/hbm_probe.txt):
// read, non-temporal, U = 8: 7.05-7.11 TB/s (plain loads 6.16-6.45); copy, non-temporal, U = 4:
// 5.66-5.75 TB/s (plain 5.03-5.39) -- both above the guide's 6.29 TB/s float4 copy figure.
typedef uint32_t probe_u32x4 __attribute__((ext_vector_type(4)));
template <bool COPY, int U>
__global__ __launch_bounds__(256) void hbm_stream(const probe_u32x4* __restrict__ src, probe_u32x4* __restrict__ dst,
                                                  size_t n16, uint32_t* sink) {
  const size_t stride = (size_t)gridDim.x * 256 * U;
  uint32_t acc = 0;
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  for (; i + (U - 1) * 256 < n16; i += stride) {
    probe_u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(src + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (COPY) __builtin_nontemporal_store(v[u], dst + i + u * 256);
      else acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
  }
  for (; i < n16; i += 256) {   // the ragged end of the buffer
    const probe_u32x4 v = src[i];
    if constexpr (COPY) dst[i] = v;
    else acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (!COPY && acc == 0x9E3779B9u && sink) sink[0] = acc;   // keeps the loads live
}

}  // namespace

extern "C" {

int ccv_hbm_probe(int mode, void* dst, const void* src, size_t bytes, uint32_t* sink, void* stream) {
  if (mode != 0 && mode != 1) return fail("ccv_hbm_probe: mode must be 0 (copy) or 1 (read)");
  if (!src || (mode == 0 && !dst)) return fail("ccv_hbm_probe: null buffer");
  if (((uintptr_t)src | (uintptr_t)dst | bytes) & 15) return fail("ccv_hbm_probe: 16-byte alignment");
  const size_t n16 = bytes / 16;
  if (n16 == 0) return 0;
  int dev = 0, cus = 0;
  HIP_TRY(hipGetDevice(&dev));
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  // 8 workgroups of 4 waves per CU (4 to 16 measure the same)
  const size_t want = (n16 + 1023) / 1024;
  const unsigned grid = (unsigned)(want < (size_t)cus * 8 ? want : (size_t)cus * 8);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (mode == 0)
    hipLaunchKernelGGL((hbm_stream<true, 4>), dim3(grid), dim3(256), 0, s, static_cast<const probe_u32x4*>(src),
                       static_cast<probe_u32x4*>(dst), n16, sink);
  else
    hipLaunchKernelGGL((hbm_stream<false, 8>), dim3(grid), dim3(256), 0, s, static_cast<const probe_u32x4*>(src),
                       nullptr, n16, sink);
  HIP_TRY(hipGetLastError());
  return 0;
}

const char* ccv_last_error(void) { return g_last_error.c_str(); }

int ccv_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

int ccv_plan_create(ccv_plan** out, int channel, int n, int K, int blen, const uint64_t* polys,
                    int gen_mode, unsigned flags) {
  if (!out) return fail("ccv_plan_create: null output pointer");
  *out = nullptr;
  if (channel != CCV_SOFT && channel != CCV_HARD) return fail("bad channel %d", channel);
  if (n < 1 || n > ccv::kMaxN) return fail("n=%d unsupported (1..%d)", n, ccv::kMaxN);
  if (K < 2 || K > ccv::kMaxK) return fail("K=%d unsupported (2..%d)", K, ccv::kMaxK);
  if (blen < 1 || blen > 255) return fail("blen=%d unsupported (1..255)", blen);
  if (!polys) return fail("null polynomials");
  if (gen_mode != CCV_GEN_REF_X86 && gen_mode != CCV_GEN_TRUE_PARITY)
    return fail("bad generator mode %d", gen_mode);

  ccv_plan* p = new ccv_plan();
  p->d.channel = channel;
  p->d.n = n;
  p->d.K = K;
  p->d.blen = blen;
  p->d.gen_mode = gen_mode;
  p->d.steps = blen + K - 1;
  p->d.states = 1 << (K - 1);
  p->d.info_bytes = (blen + 7) / 8;
  p->d.out_bytes = (p->d.steps + 7) / 8;
  p->d.in_step_bytes = channel == CCV_SOFT ? (int)sizeof(float) << n : 1;
  memcpy(p->polys, polys, sizeof(uint64_t) * (size_t)n);
  p->exp.resize(2 * (size_t)p->d.states);
  ccv::build_trellis(n, K, p->polys, gen_mode, p->exp.data());

  hipError_t e = hipGetDevice(&p->d.device);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    delete p;
    return fail("no HIP device: %s", hipGetErrorString(e));
  }
  p->step_major = (flags & CCV_FLAG_STEP_MAJOR) != 0;
  p->global_decisions = (flags & CCV_FLAG_GLOBAL_DECISIONS) != 0;
  p->no_persistent = (flags & CCV_FLAG_NO_PERSISTENT) != 0;
  if (p->step_major && channel != CCV_SOFT) {
    delete p;
    return fail("step-major input is a soft-decision layout");
  }
  p->reg_index = (flags & CCV_FLAG_GENERIC) ? -1 : find_reg_kernel(*p);
  p->multi_index = (flags & CCV_FLAG_GENERIC) || p->reg_index >= 0 ? -1 : find_multi_kernel(*p);
  if (p->step_major && p->reg_index < 0) {
    delete p;
    return fail("step-major input needs a register-trellis code with K <= 7");
  }
  p->d.lanes = 1;
  if (p->reg_index >= 0) {
    p->d.kernel = CCV_KERNEL_REGISTER;
    p->d.decision_word_bytes = p->d.states > 32 ? 8 : 4;
  } else if (p->multi_index >= 0) {
    p->d.kernel = CCV_KERNEL_MULTILANE;
    p->d.decision_word_bytes = 8;
    p->d.lanes = 1 << (K - 7);
  } else {
    p->d.kernel = CCV_KERNEL_GENERIC;
  }
  // The generic kernel (one workgroup per block) also serves small host batches of the register
  // codes: it decodes a block in a few microseconds, where one register-trellis lane takes ~17 us.
  {
    const int S = p->d.states;
    p->generic_spt = S <= ccv::kGenericMaxThreads ? 1 : S / ccv::kGenericMaxThreads;
    p->generic_threads = S <= 64 ? 64 : (S <= ccv::kGenericMaxThreads ? S : ccv::kGenericMaxThreads);
    const int NS = 1 << n;
    p->generic_chunk = 4096 / NS < 1 ? 1 : 4096 / NS;
    if (p->generic_chunk > p->d.steps) p->generic_chunk = p->d.steps;
    p->generic_lds = ccv::generic_lds_bytes(n, K, p->d.steps, p->generic_chunk, channel == CCV_HARD);
    p->generic_ok = p->generic_lds <= 160 * 1024 && p->generic_spt <= 8;
    if (p->d.kernel == CCV_KERNEL_GENERIC && !p->generic_ok) {
      delete p;
      return fail("code needs %zu B of LDS per block", p->generic_lds);
    }
    if (p->generic_ok &&
        (hipMalloc(&p->d_exp, p->exp.size()) != hipSuccess ||
         hipMemcpy(p->d_exp, p->exp.data(), p->exp.size(), hipMemcpyHostToDevice) != hipSuccess)) {
      (void)hipGetLastError();
      if (p->d_exp) (void)hipFree(p->d_exp);
      delete p;
      return fail("device table upload failed");
    }
  }
  if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    if (p->d_exp) (void)hipFree(p->d_exp);
    delete p;
    return fail("hipStreamCreate failed");
  }
  // the persistent kernels' group queue: zeroed once here, then reset by each launch's last wave
  if (register_path(*p) &&
      (p->queue.grow(ccv::kQueueWords * sizeof(uint32_t), p->stream) ||
       hipMemset(p->queue.ptr, 0, ccv::kQueueWords * sizeof(uint32_t)) != hipSuccess)) {
    (void)hipGetLastError();
    const std::string why = g_last_error;
    ccv_plan_destroy(p);
    return fail("group queue allocation failed: %s", why.c_str());
  }
  *out = p;
  return 0;
}

int ccv_plan_set_option(ccv_plan* p, const char* name, long long value) {
  if (!p) return fail("null plan");
  if (!name) return fail("null option name");
  const std::string n(name);
  auto in = [&](long long lo, long long hi) { return value >= lo && value <= hi; };
  auto need = [&](bool ok, const char* what) { return ok ? 0 : fail("option %s: %s", name, what); };
  if (n == "stack_kernel" || n == "stack_row_lanes" || n == "stack_keys" || n == "stack_symtab") {
    if (need(p->stack, "a stack-decoder plan option")) return -1;
    if (n == "stack_kernel") { if (need(in(0, 1), "0 rows / 1 one search per wave")) return -1; p->opt.stack_kernel = (int)value; }
    if (n == "stack_row_lanes") { if (need(value == 0 || value == 8 || value == 16, "0 (auto), 8 or 16")) return -1; p->opt.stack_row_lanes = (int)value; }
    if (n == "stack_keys") { if (need(in(0, 1), "0 / 1")) return -1; p->opt.stack_keys = (int)value; }
    if (n == "stack_symtab") { if (need(in(0, 1), "0 / 1")) return -1; p->opt.stack_symtab = (int)value; }
    return 0;
  }
  if (n == "fano_rows" || n == "fano_symtab" || n == "fano_order" || n == "fano_cap" || n == "fano_count_moves") {
    if (need(p->fano, "a Fano-decoder plan option")) return -1;
    if (n == "fano_rows") { if (need(in(-1, 2), "-1 (auto) or 0..2")) return -1; p->opt.fano_rows = (int)value; }
    if (n == "fano_symtab") { if (need(in(-1, 1), "-1 (auto), 0 / 1")) return -1; p->opt.fano_symtab = (int)value; }
    if (n == "fano_order") { if (need(in(0, 1), "0 / 1")) return -1; p->opt.fano_order = (int)value; }
    if (n == "fano_cap") { if (need(in(-1, 0xFFFFFFFFll), "-1 (default) or moves")) return -1; p->opt.fano_cap = value; }
    if (n == "fano_count_moves") { if (need(in(0, 1), "0 / 1")) return -1; p->opt.fano_count_moves = (int)value; }
    return 0;
  }
  if (n == "fano_input") {   // soft Fano: received points (ccv_simulate_device CCV_CHANNEL_IQ frames)
    if (need(p->fano, "a Fano-decoder plan option")) return -1;
    if (need(in(0, 1), "0 distances / 1 received points")) return -1;
    if (value == 1 && need(p->d.channel == CCV_SOFT && p->d.n == 2 && p->d.K <= 32,
                           "received points: soft rate-1/2 codes with K <= 32"))
      return -1;
    p->opt.fano_input = (int)value;
    return 0;
  }
  if (n == "channel_fused" || n == "channel_lds_decisions") {
    if (need(!p->stack && !p->fano, "a Viterbi plan option")) return -1;
    if (n == "channel_fused") { if (need(in(0, 1), "0 / 1")) return -1; p->opt.channel_fused = (int)value; }
    if (n == "channel_lds_decisions") { if (need(in(-1, 1), "-1 (auto), 0 / 1")) return -1; p->opt.channel_lds_decisions = (int)value; }
    return 0;
  }
  return fail("unknown option %s", name);
}

void ccv_plan_destroy(ccv_plan* p) {
  if (!p) return;
  if (p->svc_stream) {   // end the streaming service kernel (it polls `stop`), then wait for it
    if (p->svc_mb.host)
      __atomic_store_n(&static_cast<ccv::ServiceMailbox*>(p->svc_mb.host)->stop, 1u, __ATOMIC_RELEASE);
    (void)hipStreamSynchronize(p->svc_stream);
    (void)hipStreamDestroy(p->svc_stream);
  }
  p->svc_mb.release();
  p->svc_in.release();
  p->svc_out.release();
  p->svc_pm.release();
  if (p->stream) (void)hipStreamSynchronize(p->stream);
  p->dec.release();
  p->host_in.release();
  p->host_out.release();
  p->host_pm.release();
  p->lat_in.release();
  p->lat_out.release();
  p->lat_pm.release();
  p->sim_info.release();
  p->sim_out.release();
  p->sim_frames.release();
  p->hard_rows.release();
  p->queue.release();
  p->counter.release();
  p->symtab.release();
  p->order.release();
  p->park.release();
  if (p->d_exp) (void)hipFree(p->d_exp);
  if (p->stream) (void)hipStreamDestroy(p->stream);
  delete p;
}

int ccv_plan_describe(const ccv_plan* p, ccv_plan_desc* desc) {
  if (!p || !desc) return fail("null argument");
  *desc = p->d;
  return 0;
}

int ccv_plan_trellis(const ccv_plan* p, uint8_t* exp) {
  if (!p || !exp) return fail("null argument");
  memcpy(exp, p->exp.data(), p->exp.size());
  return 0;
}

int ccv_plan_decision_storage(const ccv_plan* p) {
  if (!p) return fail("null plan");
  if (p->stack || p->fano) return CCV_DECISIONS_NONE;
  if (!register_path(*p)) return CCV_DECISIONS_LDS;   // acs_generic.hpp: a block's decisions in LDS
  if (wide_kernel(*p, false)) return CCV_DECISIONS_SLOT;
  return persist_kernel(*p, false) || regdec_kernel(*p, false) ? CCV_DECISIONS_REGISTERS
                                                               : CCV_DECISIONS_HBM;
}

const char* ccv_plan_kernel_variant(const ccv_plan* p) {
  if (!p) return "";
  if (p->stack) return "stack";
  if (p->fano) return "fano";
  if (!register_path(*p)) return "generic";
  if (wide_kernel(*p, false)) {
    if (p->d.gen_mode == CCV_GEN_REF_X86) return "persistent-wide";
    return "persistent-slot2";   // two lanes per block (acs_multi2.hpp)
  }
  if (persist_kernel(*p, false)) return "persistent";
  if (p->multi_index >= 0) return regdec_kernel(*p, false) ? "multilane-regdec" : "multilane";
  return regdec_kernel(*p, false) ? "register-regdec" : "register";
}

namespace {
// Grid of a persistent launcher (resident waves): the launcher runs in query mode and launches
// nothing. -1 on error.
int persistent_grid(ccv::RegLaunchFn persist, bool fresh) {
  ccv::g_persist_query = ccv::PersistQuery{true, fresh, 0};
  ccv::RegArgs a{};
  const hipError_t e = persist(a, 1, nullptr);
  const int waves = ccv::g_persist_query.waves;
  ccv::g_persist_query = ccv::PersistQuery{};
  if (e != hipSuccess) return fail("persistent kernel query: %s", hipGetErrorString(e));
  return waves;
}

// The wide kernel's decision scratch: one slot per resident wave (acs_wide.hpp).
int grow_wide_scratch(ccv_plan& p, ccv::RegLaunchFn wide, hipStream_t stream) {
  const int waves = persistent_grid(wide, false);
  if (waves <= 0) return waves < 0 ? -1 : fail("no resident waves for the K = 9 kernel");
  return p.dec.grow((size_t)waves * ccv::multi_wide_slot_bytes(p.multi_index), stream);
}
}  // namespace

int ccv_plan_persistent_waves(const ccv_plan* p, int fresh) {
  if (!p) return fail("null plan");
  const ccv::RegLaunchFn persist = persist_kernel(*p, false);
  if (!persist) return 0;
  return persistent_grid(persist, fresh != 0);
}

int ccv_plan_reserve(ccv_plan* p, size_t max_blocks) {
  if (!p) return fail("null plan");
  if (const ccv::RegLaunchFn wide = wide_kernel(*p, false)) {
    if (grow_wide_scratch(*p, wide, p->stream)) return -1;
    // BSC: the Hamming-distance rows ccv_decode_device builds ahead of the soft kernel (16 B per step)
    if (p->d.channel == CCV_HARD)
      return p->hard_rows.grow(max_blocks * (size_t)p->d.steps * sizeof(float4), p->stream);
    return 0;
  }
  if (persist_kernel(*p, false)) {
    // hard: a partial last group of < 64 blocks runs on viterbi_hard_reg with HBM decisions
    if (p->d.channel != CCV_HARD) return 0;
    return p->dec.grow(decision_bytes(*p, max_blocks < 64 ? max_blocks : 64), p->stream);
  }
  if (!register_path(*p) || regdec_kernel(*p, false)) return 0;   // no decision scratch needed
  return p->dec.grow(decision_bytes(*p, max_blocks), p->stream);
}

int ccv_decode_device(ccv_plan* p, const void* d_in, size_t nblocks, uint8_t* d_out,
                      int32_t* d_path_metric, const uint8_t* d_info, unsigned long long* d_errors,
                      void* d_decisions, void* stream_v) {
  if (!p) return fail("null plan");
  if (nblocks == 0) return 0;
  if (!d_in || !d_out) return fail("null device buffer");
  if (nblocks > 0x7fffffffULL) return fail("too many blocks in one call");
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_v);
  const bool hard = p->d.channel == CCV_HARD;
  if (p->fano) {
    if (d_decisions) return fail("a Fano decoder has no survivor decisions");
    return ccv_fano_decode_device(p, d_in, nblocks, d_out, d_path_metric, d_info, d_errors, nullptr,
                                  stream_v);
  }
  if (p->stack) {
    if (d_decisions) return fail("a stack decoder has no survivor decisions");
    return ccv_stack_decode_device(p, d_in, nblocks, nullptr, d_out, d_path_metric, d_info, d_errors,
                                   nullptr, stream_v);
  }
  if (register_path(*p)) {
    if (d_decisions && p->reg_index < 0)
      return fail("decision export needs the single-lane register kernel (K <= 7)");
    ccv::RegArgs a{};
    a.in = d_in;
    a.T = p->d.steps;
    a.nblocks = (int)nblocks;
    a.blen = p->d.blen;
    a.dec_stride = (int)padded_columns(*p, nblocks);
    a.out = d_out;
    a.path_metric = hard ? d_path_metric : nullptr;
    a.info = d_info;
    a.err = d_info ? d_errors : nullptr;
    a.queue = static_cast<uint32_t*>(p->queue.ptr);
    if (const ccv::RegLaunchFn wide = wide_kernel(*p, d_decisions != nullptr)) {
      // decisions in a per-wave scratch slot, groups of 64 (one lane per block, acs_wide.hpp) or 16
      // (four lanes per block, acs_multi.hpp viterbi_multi_slot) blocks
      if (grow_wide_scratch(*p, wide, stream)) return -1;
      a.dec = p->dec.ptr;
      if (hard) {
        const size_t n = nblocks * (size_t)p->d.steps;
        if (p->hard_rows.grow(n * sizeof(float4), stream)) return -1;
        const size_t grid = std::min<size_t>((n + 255) / 256, 8192);
        hipLaunchKernelGGL(hard_rows, dim3((unsigned)grid), dim3(256), 0, stream,
                           static_cast<const uint8_t*>(d_in), static_cast<float4*>(p->hard_rows.ptr), n);
        HIP_TRY(hipGetLastError());
        a.in = p->hard_rows.ptr;
      }
      const size_t gb = (size_t)ccv::multi_wide_group_blocks(p->multi_index);
      HIP_TRY(wide(a, (int)((nblocks + gb - 1) / gb), stream));
      return 0;
    }
    if (const ccv::RegLaunchFn persist = persist_kernel(*p, d_decisions != nullptr)) {
      // decisions in VGPRs, grid = resident waves walking groups of 64 / lanes blocks
      // (acs_persist.hpp, acs_multi.hpp)
      const size_t per_group = ccv::kRegThreads / (size_t)p->d.lanes;
      const size_t full = nblocks / per_group, rem = nblocks % per_group;
      if (!hard) {
        HIP_TRY(persist(a, (int)(full + (rem ? 1 : 0)), stream));
        return 0;
      }
      if (full) HIP_TRY(persist(a, (int)full, stream));
      if (rem) {   // the hard kernel stages whole groups: the partial last one goes to viterbi_hard_reg
        const size_t done = full * ccv::kRegThreads;
        ccv::RegArgs r = a;
        r.in = static_cast<const uint8_t*>(d_in) + done * (size_t)p->d.steps;
        r.nblocks = (int)rem;
        r.dec_stride = (int)padded_columns(*p, rem);
        r.out = d_out + done * (size_t)p->d.out_bytes;
        r.path_metric = a.path_metric ? a.path_metric + done : nullptr;
        r.info = d_info ? d_info + done * (size_t)p->d.info_bytes : nullptr;
        if (p->dec.grow(decision_bytes(*p, rem), stream)) return -1;
        r.dec = p->dec.ptr;
        HIP_TRY(ccv::hard_reg_launchers()[p->reg_index](r, 1, stream));
      }
      return 0;
    }
    const ccv::RegLaunchFn regdec = regdec_kernel(*p, d_decisions != nullptr);
    if (d_decisions) {
      a.dec = d_decisions;
    } else if (!regdec) {
      if (p->dec.grow(decision_bytes(*p, nblocks), stream)) return -1;
      a.dec = p->dec.ptr;
    }
    const int grid = (int)(padded_columns(*p, nblocks) / ccv::kRegThreads);
    if (regdec) {
      // decisions stay in VGPRs: no scratch traffic, traceback from registers
      HIP_TRY(regdec(a, grid, stream));
    } else if (p->reg_index >= 0) {
      const ccv::RegLaunchFn* fns =
          hard ? ccv::hard_reg_launchers() : ccv::soft_reg_launchers(p->step_major);
      HIP_TRY(fns[p->reg_index](a, grid, stream));
    } else {
      HIP_TRY(ccv::multi_launchers(hard)[p->multi_index](a, grid, stream));
    }
  } else {
    if (d_decisions) return fail("decision export needs the register kernel");
    ccv::GenericArgs a{};
    a.in = d_in;
    a.exp = p->d_exp;
    a.n = p->d.n;
    a.K = p->d.K;
    a.T = p->d.steps;
    a.blen = p->d.blen;
    a.nblocks = (int)nblocks;
    a.chunk = p->generic_chunk;
    a.out = d_out;
    a.path_metric = hard ? d_path_metric : nullptr;
    a.info = d_info;
    a.err = d_info ? d_errors : nullptr;
    HIP_TRY(hard ? launch_generic<true>(a, *p, nblocks, stream)
                 : launch_generic<false>(a, *p, nblocks, stream));
  }
  return 0;
}

static int sequential_plan_create(ccv_plan** out, bool fano, int channel, int n, int K, int blen,
                                  const uint64_t* polys, int gen_mode, float metric_weight,
                                  const int32_t* bit_metrics);

int ccv_stack_plan_create(ccv_plan** out, int channel, int n, int K, int blen, const uint64_t* polys,
                          int gen_mode, float metric_weight, const int32_t* bit_metrics) {
  return sequential_plan_create(out, false, channel, n, K, blen, polys, gen_mode, metric_weight,
                                bit_metrics);
}

int ccv_fano_plan_create(ccv_plan** out, int channel, int n, int K, int blen, const uint64_t* polys,
                         int gen_mode, float fano_metric_weight, const int32_t* fano_bit_metrics) {
  return sequential_plan_create(out, true, channel, n, K, blen, polys, gen_mode, fano_metric_weight,
                                fano_bit_metrics);
}

static int sequential_plan_create(ccv_plan** out, bool fano, int channel, int n, int K, int blen,
                                  const uint64_t* polys, int gen_mode, float metric_weight,
                                  const int32_t* bit_metrics) {
  if (!out) return fail("plan create: null output pointer");
  *out = nullptr;
  if (channel != CCV_SOFT && channel != CCV_HARD) return fail("bad channel %d", channel);
  if (n < 1 || n > ccv::kMaxN) return fail("n=%d unsupported (1..%d)", n, ccv::kMaxN);
  if (K < 2 || K > 64) return fail("K=%d unsupported (2..64, stack-decoder.c keeps a uint64_t state)", K);
  if (blen < 1 || blen > 255) return fail("blen=%d unsupported (1..255)", blen);
  if (!polys) return fail("null polynomials");
  if (gen_mode != CCV_GEN_REF_X86 && gen_mode != CCV_GEN_TRUE_PARITY)
    return fail("bad generator mode %d", gen_mode);
  const int T = blen + K - 1;
  if (T > 255)   // uint8_t blocklen_w_tail / input indices (stack-decoder.c:15, fano-decoder.c:36)
    return fail("T=%d > 255: the reference decoder's uint8_t step indices wrap", T);
  if (channel == CCV_HARD && !bit_metrics) return fail("null bit metrics");
  if (!fano && channel == CCV_SOFT && ((size_t)T << n) > 65535)
    return fail("T * 2^n = %zu floats: the AWGN stack decoder's uint16_t index wraps", (size_t)T << n);
  if (!fano && channel == CCV_SOFT && 2 * ((size_t)T << n) * sizeof(float) > 64 * 1024)
    return fail("T * 2^n too large for the staged input (64 KiB of LDS)");
  ccv_plan* p = new ccv_plan();
  p->stack = !fano;
  p->fano = fano;
  p->metric_weight = metric_weight;
  if (bit_metrics) {
    p->bit_metrics[0] = bit_metrics[0];
    p->bit_metrics[1] = bit_metrics[1];
  }
  p->d.channel = channel;
  p->d.n = n;
  p->d.K = K;
  p->d.blen = blen;
  p->d.gen_mode = gen_mode;
  p->d.steps = T;
  p->d.states = 0;   // no trellis: the search keeps at most 64 paths
  p->d.info_bytes = (blen + 7) / 8;
  p->d.out_bytes = (T + 7) / 8;
  p->d.in_step_bytes = channel == CCV_SOFT ? (int)sizeof(float) << n : 1;
  p->d.kernel = fano ? CCV_KERNEL_FANO : CCV_KERNEL_STACK;
  p->d.lanes = fano ? 1 : ccv::kStackDepth;
  memcpy(p->polys, polys, sizeof(uint64_t) * (size_t)n);
  hipError_t e = hipGetDevice(&p->d.device);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    delete p;
    return fail("no HIP device: %s", hipGetErrorString(e));
  }
  if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    delete p;
    return fail("hipStreamCreate failed");
  }
  *out = p;
  return 0;
}

// The expected-symbol table of the sequential decoders (stack rows kernel, Fano), built on the
// plan's first decode that uses it, stream-ordered before that and every later decode.
static int ensure_symtab(ccv_plan* p, hipStream_t stream) {
  if (p->symtab_ready) return 0;
  ccv::StackArgs sa{};
  sa.n = p->d.n;
  sa.K = p->d.K;
  sa.gen = p->d.gen_mode;
  memcpy(sa.poly, p->polys, sizeof sa.poly);
  if (p->symtab.grow(sizeof(uint16_t) << (sa.K - 1), stream)) return -1;
  HIP_TRY(ccv::launch_stack_symtab(static_cast<uint16_t*>(p->symtab.ptr), sa, stream));
  p->symtab_ready = true;
  return 0;
}

int ccv_fano_decode_device(ccv_plan* p, const void* d_in, size_t nblocks, uint8_t* d_out,
                           int32_t* d_path_metric, const uint8_t* d_info, unsigned long long* d_errors,
                           uint32_t* d_iterations, void* stream_v) {
  if (!p) return fail("null plan");
  if (!p->fano) return fail("not a Fano-decoder plan (ccv_fano_plan_create)");
  if (nblocks == 0) return 0;
  if (!d_in || !d_out) return fail("null device buffer");
  if (nblocks > 0x7fffffffULL) return fail("too many blocks in one call");
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_v);
  // counters: [0] pass-1 queue, [1] pass-2 queue, [2] parked searches; [4..7] diagnostics
  if (p->counter.grow(64, stream)) return -1;
  HIP_TRY(hipMemsetAsync(p->counter.ptr, 0, 64, stream));
  unsigned int* ctr = static_cast<unsigned int*>(p->counter.ptr);
  ccv::FanoArgs a{};
  a.in = d_in;
  a.n = p->d.n;
  a.K = p->d.K;
  a.T = p->d.steps;
  a.blen = p->d.blen;
  a.gen = p->d.gen_mode;
  memcpy(a.poly, p->polys, sizeof a.poly);
  a.weight = p->metric_weight;
  a.bm0 = p->bit_metrics[0];
  a.bm1 = p->bit_metrics[1];
  a.nblocks = (int)nblocks;
  a.next_block = ctr;
  a.out = d_out;
  a.path_metric = p->d.channel == CCV_HARD ? d_path_metric : nullptr;
  a.info = d_info;
  a.err = d_info ? d_errors : nullptr;
  a.iterations = d_iterations;
  // two-pass schedule (fano_dev.hpp): park searches after 6000 x T moves (soft, 0.6 of the timeout)
  // or 1000 x T (hard), resume them in pass 2; option "fano_cap" overrides, 0 = one pass. Measured
  // caps (K = 15, 104 frames): round 3 (tools/fano_caps.py, profiles/r03_fano_caps.txt) 4 dB 47.3 (one
  // pass) -> 49.4 Mbit/s at 216,000 moves, 41.5 at 20,000-108,000 (half the searches park and the
  // parking costs more than the tail it saves); round 6 on the current kernels (tools/fano_cap_sweep.sh,
  // profiles/r06_fano_cap/; mean of 2-4 round-robin runs): soft 4 dB 51.6 / 67.4 / 68.3 / 68.4 / 66.6
  // / 64.9 at 108,000 / 216,000 / 270,000 / 324,000 / 378,000 / 432,000 (61.1 one pass); BSC 5 %
  // 230.1 / 239.9 / 236.9 at 216,000 / 54,000 / one pass.
  long cap = p->opt.fano_cap >= 0 ? (long)p->opt.fano_cap
                                  : (p->d.channel == CCV_HARD ? 1000L : 6000L) * a.T;
  if (cap > 0 && nblocks > 64) {
    const size_t cap_slots = nblocks / 8 > 65536 ? nblocks / 8 : (nblocks < 65536 ? nblocks : 65536);
    const size_t mt = p->d.channel == CCV_HARD ? sizeof(int32_t) : sizeof(float);
    const size_t hdr = cap_slots * ccv::kFanoParkWords * sizeof(uint32_t);
    const size_t met = (cap_slots * (size_t)(a.T + 1) * mt + 255) & ~(size_t)255;
    const size_t flg = cap_slots * (size_t)(a.T + 1);
    if (p->park.grow(hdr + met + flg, stream)) return -1;
    char* base = static_cast<char*>(p->park.ptr);
    a.cap = (uint32_t)cap;
    a.park_capacity = (unsigned int)cap_slots;
    a.park_count = ctr + 2;
    a.park_hdr = reinterpret_cast<uint32_t*>(base);
    a.park_metric = base + hdr;
    a.park_flags = reinterpret_cast<uint8_t*>(base + hdr + met);
  }
  a.count_moves = p->opt.fano_count_moves;
  a.iq = p->opt.fano_input;   // before the queue order: its score kernel reads the input too
  // the expected-symbol table: hard input only. For soft input the table load sits in each move's
  // dependent chain next to the row load, and the kernel waits on memory (PMC, round 4: wait 0.66 of
  // wave time, valu_frac 0.17): the ~25 VALU of parities are cheaper (4 dB: 49.6 -> 57.7 Mbit/s, with
  // the candidate rows prefetched 55.7 -> 67.2, profiles/r04c/fano_ab.txt). Option "fano_symtab"
  // overrides.
  const bool tab_ok = a.K <= ccv::kSymtabMaxK && (a.n == 2 || a.n == 3);
  const bool tab = tab_ok && (p->opt.fano_symtab < 0 ? p->d.channel == CCV_HARD : p->opt.fano_symtab != 0);
  if (tab) {
    if (ensure_symtab(p, stream)) return -1;
    a.symtab = static_cast<const uint16_t*>(p->symtab.ptr);
  }
  // soft input: hand out the noisiest blocks first (fano_dev.hpp, fano_score); option "fano_order" 0 off
  const bool order = p->opt.fano_order && p->d.channel == CCV_SOFT && (a.n == 2 || a.n == 3) && nblocks > 64;
  if (order) {
    const size_t need = ccv::fano_order_bytes(a.nblocks);
    if (p->order.grow(need, stream)) return -1;
    HIP_TRY(ccv::launch_fano_order(a, p->order.ptr, p->order.bytes, &a.order, stream));
  }
  a.rows_mode = p->opt.fano_rows;
  const bool debug = std::getenv("CCV_DEBUG") != nullptr;
  if (debug)   // diagnostics: synchronous, prints lane utilisation (both passes together)
    a.stats = reinterpret_cast<unsigned long long*>(ctr + 4);
  HIP_TRY(ccv::launch_fano(a, p->d.channel == CCV_HARD, stream));
  if (a.cap) {   // pass 2: the parked searches (the count is read on the device)
    ccv::FanoArgs r = a;
    r.resume = 1;
    r.cap = 0;
    r.next_block = ctr + 1;
    r.order = nullptr;
    HIP_TRY(ccv::launch_fano(r, p->d.channel == CCV_HARD, stream));
  }
  if (debug) {
    unsigned long long st[2] = {0, 0};
    unsigned int parked = 0;
    HIP_TRY(hipMemcpyAsync(st, a.stats, sizeof st, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(&parked, ctr + 2, sizeof parked, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    std::fprintf(stderr, "fano: %zu blocks, %u parked after %u moves, wave passes %llu, busy lane passes %llu, "
                 "lane utilisation %.3f\n", nblocks, parked, a.cap, st[0], st[1],
                 st[0] ? (double)st[1] / (64.0 * (double)st[0]) : 0.0);
  }
  return 0;
}

int ccv_stack_decode_device(ccv_plan* p, const void* d_in, size_t nblocks, const void* d_prev,
                            uint8_t* d_out, int32_t* d_path_metric, const uint8_t* d_info,
                            unsigned long long* d_errors, int32_t* d_status, void* stream_v) {
  if (!p) return fail("null plan");
  if (!p->stack) return fail("not a stack-decoder plan (ccv_stack_plan_create)");
  if (nblocks == 0) return 0;
  if (!d_in || !d_out) return fail("null device buffer");
  if (nblocks > 0x7fffffffULL) return fail("too many blocks in one call");
  ccv::StackArgs a{};
  a.in = d_in;
  a.prev = d_prev;
  a.n = p->d.n;
  a.K = p->d.K;
  a.T = p->d.steps;
  a.blen = p->d.blen;
  a.gen = p->d.gen_mode;
  memcpy(a.poly, p->polys, sizeof a.poly);
  a.weight = p->metric_weight;
  a.bm0 = p->bit_metrics[0];
  a.bm1 = p->bit_metrics[1];
  a.nblocks = (int)nblocks;
  a.out = d_out;
  a.path_metric = p->d.channel == CCV_HARD ? d_path_metric : nullptr;
  a.info = d_info;
  a.err = d_info ? d_errors : nullptr;
  a.status = d_status;
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_v);
  a.opt_row_lanes = p->opt.stack_row_lanes;
  a.opt_keys = p->opt.stack_keys;
  // persistent rows pull blocks from a counter (the noisiest-first order of the Fano decoder was
  // measured 3 % slower here, profiles/r04x/, and removed in round 5)
  if (p->opt.stack_kernel == 0 && ccv::stack_rows_eligible(a.n, a.K, a.T)) {
    if (p->counter.grow(sizeof(unsigned int), stream)) return -1;
    HIP_TRY(hipMemsetAsync(p->counter.ptr, 0, sizeof(unsigned int), stream));
    a.next_block = static_cast<unsigned int*>(p->counter.ptr);
    if (p->opt.stack_symtab && ccv::stack_symtab_eligible(a.n, a.K, a.T)) {
      if (ensure_symtab(p, stream)) return -1;
      a.symtab = static_cast<const uint16_t*>(p->symtab.ptr);
    }
  }
  HIP_TRY(ccv::launch_stack(a, p->d.channel == CCV_HARD, stream));
  return 0;
}

// CCV_CHANNEL_FRAMES_ONLY: the channel's frames (info bytes, decoder input) for any plan's code, no
// decode (channel_dev.hpp channel_frames_rt) -- the producer of the stack / Fano device sweeps.
static int simulate_frames_only(ccv_plan* p, uint64_t seed, uint64_t first_block, size_t nblocks,
                                double channel_param, unsigned channel_flags, uint8_t* d_info,
                                void* d_channel, void* stream_v) {
  const bool hard = p->d.channel == CCV_HARD;
  if (!d_channel) return fail("CCV_CHANNEL_FRAMES_ONLY needs d_channel");
  // the frames are written block-major, which a step-major plan would decode as scrambled input
  if (p->step_major) return fail("CCV_CHANNEL_FRAMES_ONLY writes block-major frames: not for a step-major plan");
  if (p->d.n > 3) return fail("frames-only channel: n = %d (n <= 3)", p->d.n);
  if (hard && !(channel_param >= 0.0 && channel_param <= 1000000.0))
    return fail("BSC p_ppm must be in [0, 1e6]");
  if (!hard && !(channel_param >= 0.0 && channel_param < 268435456.0))
    return fail("AWGN noise scaling must be in [0, 2^28)");
  if (hard && (channel_flags & CCV_CHANNEL_HARD_DEMAP)) return fail("the hard demapper belongs to the AWGN channel");
  if (hard && (channel_flags & CCV_CHANNEL_NOISE_F32)) return fail("the fp32 Box-Muller belongs to the AWGN channel");
  if (nblocks == 0) return 0;
  if (nblocks > 0x7fffffffULL) return fail("too many blocks in one call");
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_v);
  if (!d_info) {
    if (p->sim_info.grow(nblocks * (size_t)p->d.info_bytes, stream)) return -1;
    d_info = static_cast<uint8_t*>(p->sim_info.ptr);
  }
  ccv::ChanArgs a{};
  a.r.T = p->d.steps;
  a.r.nblocks = (int)nblocks;
  a.r.blen = p->d.blen;
  a.seed = seed;
  a.first_block = first_block;
  a.scaling = (float)channel_param;
  a.p_ppm = hard ? (int32_t)channel_param : 0;
  a.hard_demap = (channel_flags & CCV_CHANNEL_HARD_DEMAP) != 0;
  a.noise_f32 = (channel_flags & CCV_CHANNEL_NOISE_F32) != 0;
  a.iq_out = (channel_flags & CCV_CHANNEL_IQ) != 0;
  if (hard && a.iq_out) return fail("CCV_CHANNEL_IQ: received points belong to the AWGN channel");
  a.info_out = d_info;
  a.ch_out = d_channel;
  HIP_TRY(ccv::launch_channel_frames_any(a, p->d.n, p->d.K, p->polys, p->d.gen_mode, hard, stream));
  return 0;
}

int ccv_simulate_device(ccv_plan* p, uint64_t seed, uint64_t first_block, size_t nblocks,
                        double channel_param, unsigned channel_flags, uint8_t* d_info, uint8_t* d_out,
                        int32_t* d_path_metric, unsigned long long* d_errors, void* d_channel,
                        void* stream_v) {
  if (!p) return fail("null plan");
  if (channel_flags & CCV_CHANNEL_FRAMES_ONLY)
    return simulate_frames_only(p, seed, first_block, nblocks, channel_param, channel_flags, d_info,
                                d_channel, stream_v);
  if (channel_flags & CCV_CHANNEL_IQ) return fail("CCV_CHANNEL_IQ is an output of CCV_CHANNEL_FRAMES_ONLY");
  if (p->stack || p->fano)
    return fail("a sequential-decoder plan takes the on-device channel with CCV_CHANNEL_FRAMES_ONLY");
  if (!register_path(*p))
    return fail("the on-device channel needs a register-trellis code (K <= 9 with a specialised kernel)");
  if (p->d.channel == CCV_SOFT && p->d.n > 3)
    return fail("no constellation for n = %d (common/constellations.c has n = 1..3)", p->d.n);
  if (nblocks == 0) return 0;
  if (nblocks > 0x7fffffffULL) return fail("too many blocks in one call");
  const bool hard = p->d.channel == CCV_HARD;
  if (hard && !(channel_param >= 0.0 && channel_param <= 1000000.0))
    return fail("BSC p_ppm must be in [0, 1e6]");
  // the demapper's 3-instruction division is exact for squared distances below 2^64, which holds
  // for noise scalings below 2^28 (channel_dev.hpp div_const; Eb/N0 above -160 dB)
  if (!hard && !(channel_param >= 0.0 && channel_param < 268435456.0))
    return fail("AWGN noise scaling must be in [0, 2^28)");
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_v);
  if (!d_info) {
    if (p->sim_info.grow(nblocks * (size_t)p->d.info_bytes, stream)) return -1;
    d_info = static_cast<uint8_t*>(p->sim_info.ptr);
  }
  if (!d_out) {
    if (p->sim_out.grow(nblocks * (size_t)p->d.out_bytes, stream)) return -1;
    d_out = static_cast<uint8_t*>(p->sim_out.ptr);
  }
  // K = 8, 9: frames to HBM once per block, then the decode with the fused error count (soft at
  // blen 40: the persistent kernels, acs_wide.hpp / acs_multi2.hpp; BSC: the multilane kernel, its
  // input one byte per step) -- the fused multilane channel kernel draws every block's channel once
  // per lane of its group (option channel_fused 1 keeps it)
  const bool frames_path = p->multi_index >= 0 && !p->opt.channel_fused && !p->step_major &&
                           (hard || persist_kernel(*p, false) != nullptr);
  if (!frames_path && p->dec.grow(decision_bytes(*p, nblocks), stream)) return -1;
  ccv::ChanArgs a{};
  a.r.in = nullptr;
  a.r.T = p->d.steps;
  a.r.nblocks = (int)nblocks;
  a.r.blen = p->d.blen;
  a.r.dec_stride = (int)padded_columns(*p, nblocks);
  a.r.out = d_out;
  a.r.path_metric = hard ? d_path_metric : nullptr;
  a.r.dec = p->dec.ptr;
  a.r.info = d_info;
  a.r.err = d_errors;
  a.seed = seed;
  a.first_block = first_block;
  a.scaling = (float)channel_param;
  a.p_ppm = hard ? (int32_t)channel_param : 0;
  a.hard_demap = (channel_flags & CCV_CHANNEL_HARD_DEMAP) != 0;
  a.noise_f32 = (channel_flags & CCV_CHANNEL_NOISE_F32) != 0;
  if (hard && a.hard_demap) return fail("the hard demapper belongs to the AWGN channel");
  if (hard && a.noise_f32) return fail("the fp32 Box-Muller belongs to the AWGN channel");
  a.info_out = d_info;
  a.ch_out = d_channel;
  // K <= 7 decisions in LDS (viterbi_channel_lds) or in HBM scratch (viterbi_channel_reg): the LDS
  // column (20 KiB per wave at K = 7) caps a CU's waves; by default the launch compares the two
  // kernels' occupancy (reg_channel.hpp). Option "channel_lds_decisions" 1 / 0 forces either (A/B).
  a.global_decisions = p->global_decisions ? 1
                       : p->opt.channel_lds_decisions < 0 ? -1
                                                          : (p->opt.channel_lds_decisions != 0 ? 0 : 1);
  if (frames_path) {
    void* frames = d_channel;
    if (!frames) {
      if (p->sim_frames.grow(nblocks * (size_t)p->d.steps * (size_t)p->d.in_step_bytes, stream)) return -1;
      frames = p->sim_frames.ptr;
    }
    a.ch_out = frames;
    if (hard)
      HIP_TRY(ccv::launch_channel_frames_any(a, p->d.n, p->d.K, p->polys, p->d.gen_mode, true, stream));
    else
      HIP_TRY(ccv::channel_frames_launchers()[p->multi_index](
          a, (int)((nblocks + ccv::kRegThreads - 1) / ccv::kRegThreads), stream));
    return ccv_decode_device(p, frames, nblocks, d_out, hard ? d_path_metric : nullptr, d_info, d_errors,
                             nullptr, stream_v);
  }
  const int grid = (int)(padded_columns(*p, nblocks) / ccv::kRegThreads);
  const bool multi = p->reg_index < 0;
  HIP_TRY(ccv::channel_launchers(multi, hard)[multi ? p->multi_index : p->reg_index](a, grid, stream));
  return 0;
}

int ccv_stack_decode_host(ccv_plan* p, const void* in, size_t nblocks, const void* prev, uint8_t* out,
                          int32_t* path_metric, int32_t* status) {
  if (!p) return fail("null plan");
  if (!p->stack) return fail("not a stack-decoder plan (ccv_stack_plan_create)");
  if (nblocks == 0) return 0;
  if (!in || !out) return fail("null host buffer");
  const size_t block_bytes = (size_t)p->d.steps * (size_t)p->d.in_step_bytes;
  const size_t in_bytes = (nblocks + 1) * block_bytes;   // slot 0: the previous block
  const size_t out_bytes = nblocks * (size_t)p->d.out_bytes;
  const size_t aux_bytes = 2 * nblocks * sizeof(int32_t);   // path metrics, status
  if (p->host_in.grow(in_bytes, p->stream) || p->host_out.grow(out_bytes, p->stream) ||
      p->host_pm.grow(aux_bytes, p->stream))
    return -1;
  unsigned char* d_in = static_cast<unsigned char*>(p->host_in.ptr);
  int32_t* d_pm = static_cast<int32_t*>(p->host_pm.ptr);
  if (prev) HIP_TRY(hipMemcpyAsync(d_in, prev, block_bytes, hipMemcpyHostToDevice, p->stream));
  HIP_TRY(hipMemcpyAsync(d_in + block_bytes, in, nblocks * block_bytes, hipMemcpyHostToDevice, p->stream));
  if (ccv_stack_decode_device(p, d_in + block_bytes, nblocks, prev ? d_in : nullptr,
                              static_cast<uint8_t*>(p->host_out.ptr), d_pm, nullptr, nullptr,
                              d_pm + nblocks, p->stream))
    return -1;
  HIP_TRY(hipMemcpyAsync(out, p->host_out.ptr, out_bytes, hipMemcpyDeviceToHost, p->stream));
  if (path_metric && p->d.channel == CCV_HARD)
    HIP_TRY(hipMemcpyAsync(path_metric, d_pm, nblocks * sizeof(int32_t), hipMemcpyDeviceToHost, p->stream));
  if (status)
    HIP_TRY(hipMemcpyAsync(status, d_pm + nblocks, nblocks * sizeof(int32_t), hipMemcpyDeviceToHost,
                           p->stream));
  HIP_TRY(hipStreamSynchronize(p->stream));
  return 0;
}

// The streaming path through the resident service kernel (acs_generic.hpp viterbi_service): post the
// block(s) in the fine-grained mailbox, relaunch the kernel if it has ended (idle timeout), spin on
// `done`. One block costs two PCIe round trips and the decode, no launch.
static int decode_host_service(ccv_plan* p, const void* in, size_t nblocks, uint8_t* out,
                               int32_t* path_metric) {
  const bool hard = p->d.channel == CCV_HARD;
  const size_t in_bytes = nblocks * (size_t)p->d.steps * (size_t)p->d.in_step_bytes;
  const size_t out_bytes = nblocks * (size_t)p->d.out_bytes;
  if (!p->svc_stream) HIP_TRY(hipStreamCreateWithFlags(&p->svc_stream, hipStreamNonBlocking));
  if (p->svc_mb.grow(sizeof(ccv::ServiceMailbox), p->svc_stream, hipHostMallocCoherent)) return -1;
  ccv::ServiceMailbox* mb = static_cast<ccv::ServiceMailbox*>(p->svc_mb.host);
  if (p->svc_in.bytes < in_bytes || p->svc_out.bytes < out_bytes || p->svc_pm.bytes < nblocks * 4) {
    // the resident kernel holds the old buffers: end it before they are replaced
    if (p->svc_running) {
      __atomic_store_n(&mb->stop, 1u, __ATOMIC_RELEASE);
      HIP_TRY(hipStreamSynchronize(p->svc_stream));
      __atomic_store_n(&mb->stop, 0u, __ATOMIC_RELEASE);
      p->svc_running = false;
    }
    const size_t cap_blocks = ccv::kServiceMaxBlocks;
    if (p->svc_in.grow(cap_blocks * (size_t)p->d.steps * (size_t)p->d.in_step_bytes, p->svc_stream,
                       hipHostMallocCoherent) ||
        p->svc_out.grow(cap_blocks * (size_t)p->d.out_bytes, p->svc_stream, hipHostMallocCoherent) ||
        p->svc_pm.grow(cap_blocks * sizeof(int32_t), p->svc_stream, hipHostMallocCoherent))
      return -1;
  }
  memcpy(p->svc_in.host, in, in_bytes);
  ccv::GenericArgs a{};
  a.in = p->svc_in.dev;
  a.exp = p->d_exp;
  a.n = p->d.n;
  a.K = p->d.K;
  a.T = p->d.steps;
  a.blen = p->d.blen;
  a.nblocks = (int)nblocks;
  a.chunk = p->generic_chunk;
  a.out = static_cast<uint8_t*>(p->svc_out.dev);
  a.path_metric = hard ? static_cast<int32_t*>(p->svc_pm.dev) : nullptr;
  auto launch = [&](uint32_t served) -> int {
    __atomic_store_n(&mb->exited, 0u, __ATOMIC_RELEASE);
    HIP_TRY(hard ? launch_service<true>(a, *p, mb, served, p->svc_stream)
                 : launch_service<false>(a, *p, mb, served, p->svc_stream));
    p->svc_running = true;
    return 0;
  };
  const uint32_t seq = ++p->svc_seq;
  if (!p->svc_running || __atomic_load_n(&mb->exited, __ATOMIC_ACQUIRE)) {
    if (p->svc_running) HIP_TRY(hipStreamSynchronize(p->svc_stream));   // the ended kernel is gone
    if (launch(seq - 1)) return -1;
  }
  __atomic_store_n(&mb->req, ((uint64_t)nblocks << 32) | seq, __ATOMIC_RELEASE);
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spins = 0; __atomic_load_n(&mb->done, __ATOMIC_ACQUIRE) != seq; ++spins) {
    if (__atomic_load_n(&mb->exited, __ATOMIC_ACQUIRE) && __atomic_load_n(&mb->done, __ATOMIC_ACQUIRE) != seq) {
      // it reached its idle timeout just before the request arrived: wait for it to end, relaunch
      HIP_TRY(hipStreamSynchronize(p->svc_stream));
      if (__atomic_load_n(&mb->done, __ATOMIC_ACQUIRE) == seq) break;
      if (launch(seq - 1)) return -1;
    }
    if ((spins & 1023u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
      // end the kernel before giving up: a service left polling could answer the NEXT call's request
      // (and a relaunched one decode it again). It exits on `stop` or after its bounded poll count.
      __atomic_store_n(&mb->stop, 1u, __ATOMIC_RELEASE);
      const hipError_t e = hipStreamSynchronize(p->svc_stream);
      __atomic_store_n(&mb->stop, 0u, __ATOMIC_RELEASE);
      p->svc_running = false;
      if (e != hipSuccess) return fail("streaming service: %s", hipGetErrorString(e));
      return fail("streaming service did not answer within 10 s");
    }
    __builtin_ia32_pause();
  }
  memcpy(out, p->svc_out.host, out_bytes);
  if (hard && path_metric) memcpy(path_metric, p->svc_pm.host, nblocks * sizeof(int32_t));
  return 0;
}

// Small host batches (the streaming decoder_input path completes one block per call): the input is
// copied into page-locked memory the kernel reads directly, the generic kernel (one workgroup per
// block, a few microseconds) writes the output and path metrics straight into page-locked memory, and
// one synchronise ends the call -- no device allocation, no DMA copies. CCV_HOST_LATENCY=0 turns it
// off (A/B).
static int decode_host_latency(ccv_plan* p, const void* in, size_t nblocks, uint8_t* out,
                               int32_t* path_metric) {
  const bool hard = p->d.channel == CCV_HARD;
  const size_t in_bytes = nblocks * (size_t)p->d.steps * (size_t)p->d.in_step_bytes;
  const size_t out_bytes = nblocks * (size_t)p->d.out_bytes;
  if (p->lat_in.grow(in_bytes, p->stream) || p->lat_out.grow(out_bytes, p->stream) ||
      p->lat_pm.grow(nblocks * sizeof(int32_t), p->stream))
    return -1;
  memcpy(p->lat_in.host, in, in_bytes);
  ccv::GenericArgs a{};
  a.in = p->lat_in.dev;
  a.exp = p->d_exp;
  a.n = p->d.n;
  a.K = p->d.K;
  a.T = p->d.steps;
  a.blen = p->d.blen;
  a.nblocks = (int)nblocks;
  a.chunk = p->generic_chunk;
  a.out = static_cast<uint8_t*>(p->lat_out.dev);
  a.path_metric = hard ? static_cast<int32_t*>(p->lat_pm.dev) : nullptr;
  if (latency_kernel_ok(*p)) {   // one wave per block (acs_latency.hpp)
    const size_t lds = latency_lds(*p);
    if (hard) launch_latency<true>(a, *p, (int)nblocks, lds);
    else launch_latency<false>(a, *p, (int)nblocks, lds);
    HIP_TRY(hipGetLastError());
  } else {
    HIP_TRY(hard ? launch_generic<true>(a, *p, nblocks, p->stream)
                 : launch_generic<false>(a, *p, nblocks, p->stream));
  }
  HIP_TRY(hipStreamSynchronize(p->stream));
  memcpy(out, p->lat_out.host, out_bytes);
  if (hard && path_metric) memcpy(path_metric, p->lat_pm.host, nblocks * sizeof(int32_t));
  return 0;
}

int ccv_decode_host(ccv_plan* p, const void* in, size_t nblocks, uint8_t* out, int32_t* path_metric) {
  if (!p) return fail("null plan");
  if (p->step_major) return fail("ccv_decode_host takes block-major input");
  if (nblocks == 0) return 0;
  if (!in || !out) return fail("null host buffer");
  if (nblocks <= ccv::kHostLatencyMaxBlocks && p->generic_ok && !p->stack && !p->fano) {
    // CCV_HOST_LATENCY: 2 (default) the resident service kernel for up to kServiceMaxBlocks blocks,
    // 1 a launch per call on zero-copy staging, 0 the device-staged batch path (A/B)
    const char* env = std::getenv("CCV_HOST_LATENCY");
    const int mode = env && env[0] ? env[0] - '0' : 2;
    if (mode >= 2 && nblocks <= ccv::kServiceMaxBlocks) return decode_host_service(p, in, nblocks, out, path_metric);
    if (mode >= 1) return decode_host_latency(p, in, nblocks, out, path_metric);
  }
  const size_t in_bytes = nblocks * (size_t)p->d.steps * (size_t)p->d.in_step_bytes;
  const size_t out_bytes = nblocks * (size_t)p->d.out_bytes;
  const bool want_pm = p->d.channel == CCV_HARD && path_metric;
  if (p->host_in.grow(in_bytes, p->stream) || p->host_out.grow(out_bytes, p->stream)) return -1;
  if (want_pm && p->host_pm.grow(nblocks * sizeof(int32_t), p->stream)) return -1;
  HIP_TRY(hipMemcpyAsync(p->host_in.ptr, in, in_bytes, hipMemcpyHostToDevice, p->stream));
  if (ccv_decode_device(p, p->host_in.ptr, nblocks, static_cast<uint8_t*>(p->host_out.ptr),
                        want_pm ? static_cast<int32_t*>(p->host_pm.ptr) : nullptr, nullptr, nullptr,
                        nullptr, p->stream))
    return -1;
  HIP_TRY(hipMemcpyAsync(out, p->host_out.ptr, out_bytes, hipMemcpyDeviceToHost, p->stream));
  if (want_pm)
    HIP_TRY(hipMemcpyAsync(path_metric, p->host_pm.ptr, nblocks * sizeof(int32_t),
                           hipMemcpyDeviceToHost, p->stream));
  HIP_TRY(hipStreamSynchronize(p->stream));
  return 0;
}

}  // extern "C"
