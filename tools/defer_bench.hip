// defer_bench.hip -- paired ABBA of the persistent kernels with and without kPersistDeferOut (a
// group's output stores issued behind the next group's first DMA instead of right before the next
// vmcnt wait), on the bench batches: K = 7 soft (headline) and BSC (config 4), 104 frames; code 0 BSC
// (config 1 at GPU scale), 104 frames. Outputs and path metrics are compared first. "production" =
// the production schedule without the flag (rounds 2-6 until it was adopted).
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -fno-slp-vectorize -I../include
//   -I../convolutional-codes_amd/csrc defer_bench.hip -o defer_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "acs_persist.hpp"
#include "reg_codes.hpp"

using namespace ccv;
constexpr CodeSpec kK7 = kRegCodes[8];
constexpr CodeSpec kC0 = kRegCodes[0];
static_assert(kK7.K == 7 && kC0.K == 3, "codes");

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void fill_soft(float* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint32_t x = (uint32_t)i * 0x9E3779B9u ^ (uint32_t)(i >> 32);
    x ^= x >> 15; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
    p[i] = (float)(x >> 8) * (1.0f / 16777216.0f) * 3.0f;
  }
}
__global__ void fill_hard(uint8_t* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint32_t x = (uint32_t)i * 0x9E3779B9u;
    x ^= x >> 15; x *= 0x85EBCA6Bu; x ^= x >> 13;
    p[i] = (uint8_t)(x >> 29);
  }
}

using Kern = void (*)(RegArgs, int);

int grid_of(Kern k, int ngroups) {
  int per_cu = 0, cus = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 64, 0));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  if (per_cu >= 4) per_cu -= per_cu % 4;
  return std::min(per_cu * cus, ngroups);
}

float sustained(Kern k, const RegArgs& a, int ng, int n) {
  const int grid = grid_of(k, ng);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, 0));
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, a, ng);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ms / n;
}

int main() {
  const int nb = 2600000, ng = nb / 64;
  float* d_soft;
  uint8_t *d_hard, *d_info, *d_out_a, *d_out_b;
  int32_t *d_pm_a, *d_pm_b;
  uint32_t* d_queue;
  unsigned long long* d_err;
  CHECK(hipMalloc(&d_soft, (size_t)nb * 46 * 16));
  CHECK(hipMalloc(&d_hard, (size_t)nb * 46));
  CHECK(hipMalloc(&d_info, (size_t)nb * 5));
  CHECK(hipMalloc(&d_out_a, (size_t)nb * 8));
  CHECK(hipMalloc(&d_out_b, (size_t)nb * 8));
  CHECK(hipMalloc(&d_pm_a, (size_t)nb * 4));
  CHECK(hipMalloc(&d_pm_b, (size_t)nb * 4));
  CHECK(hipMalloc(&d_queue, kQueueWords * 4));
  CHECK(hipMalloc(&d_err, 16));
  CHECK(hipMemset(d_queue, 0, kQueueWords * 4));
  CHECK(hipMemset(d_err, 0, 16));
  hipLaunchKernelGGL(fill_soft, dim3(8192), dim3(256), 0, 0, d_soft, (size_t)nb * 46 * 4);
  hipLaunchKernelGGL(fill_hard, dim3(8192), dim3(256), 0, 0, d_hard, (size_t)nb * 46);
  hipLaunchKernelGGL(fill_hard, dim3(8192), dim3(256), 0, 0, d_info, (size_t)nb * 5);
  CHECK(hipDeviceSynchronize());

  struct Case {
    const char* name;
    Kern prod, defer;
    bool hard;
    int T;
  };
  constexpr int DF = kPersistDeferOut;
  const Case cases[] = {
      {"soft K=7 (headline)", viterbi_soft_persist<kK7, 40, (persist_soft_opt<kK7>() & ~DF)>,
       viterbi_soft_persist<kK7, 40, persist_soft_opt<kK7>() | DF>, false, 46},
      {"BSC K=7 (config 4)", viterbi_hard_persist<kK7, 40, 3, (persist_hard_opt<kK7>() & ~DF)>,
       viterbi_hard_persist<kK7, 40, 3, persist_hard_opt<kK7>() | DF>, true, 46},
      {"BSC code 0 (config 1 at scale)", viterbi_hard_persist<kC0, 40, 3, (persist_hard_opt<kC0>() & ~DF)>,
       viterbi_hard_persist<kC0, 40, 3, persist_hard_opt<kC0>() | DF>, true, 42},
      {"soft code 0", viterbi_soft_persist<kC0, 40, (persist_soft_opt<kC0>() & ~DF)>,
       viterbi_soft_persist<kC0, 40, persist_soft_opt<kC0>() | DF>, false, 42},
  };
  int bad = 0;
  for (const Case& c : cases) {
    RegArgs a{};
    a.in = c.hard ? (const void*)d_hard : (const void*)d_soft;
    a.T = c.T;
    a.nblocks = nb;
    a.blen = 40;
    a.queue = d_queue;
    a.info = d_info;
    a.err = d_err;
    const int OB = (c.T + 7) / 8;
    // exactness (three launches of the variant: the queue resets itself), then ragged sizes
    for (int n : {nb, 64 * 7, 64 * 3001}) {
      const int g = n / 64;
      for (uint8_t* o : {d_out_a, d_out_b}) CHECK(hipMemset(o, 0xA5, (size_t)nb * 8));
      for (int32_t* p : {d_pm_a, d_pm_b}) CHECK(hipMemset(p, 0x5A, (size_t)nb * 4));
      RegArgs x = a;
      x.nblocks = n;
      x.out = d_out_a;
      x.path_metric = c.hard ? d_pm_a : nullptr;
      hipLaunchKernelGGL(c.prod, dim3(grid_of(c.prod, g)), dim3(64), 0, 0, x, g);
      x.out = d_out_b;
      x.path_metric = c.hard ? d_pm_b : nullptr;
      for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(c.defer, dim3(grid_of(c.defer, g)), dim3(64), 0, 0, x, g);
      CHECK(hipDeviceSynchronize());
      std::vector<uint8_t> p((size_t)n * OB), q((size_t)n * OB);
      CHECK(hipMemcpy(p.data(), d_out_a, p.size(), hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(q.data(), d_out_b, q.size(), hipMemcpyDeviceToHost));
      std::vector<int32_t> pa(n), pb(n);
      CHECK(hipMemcpy(pa.data(), d_pm_a, (size_t)n * 4, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(pb.data(), d_pm_b, (size_t)n * 4, hipMemcpyDeviceToHost));
      const bool same = p == q && (!c.hard || pa == pb);
      printf("%s, %d blocks: variant outputs%s %s\n", c.name, n, c.hard ? " and path metrics" : "",
             same ? "identical" : "DIFFER");
      bad += !same;
    }
    a.out = d_out_a;
    a.path_metric = c.hard ? d_pm_a : nullptr;
    sustained(c.prod, a, ng, 200);
    double r = 0, at = 0, bt = 0;
    for (int qd = 0; qd < 4; ++qd) {
      const float a0 = sustained(c.prod, a, ng, 40), b0 = sustained(c.defer, a, ng, 40),
                  b1 = sustained(c.defer, a, ng, 40), a1 = sustained(c.prod, a, ng, 40);
      r += (b0 + b1) / (a0 + a1);
      at += a0 + a1;
      bt += b0 + b1;
    }
    const double bits = (double)nb * 40;
    printf("%-32s A %.4f ms (%.1f Gbit/s)  B (variant) %.4f ms (%.1f Gbit/s)  time ratio %.3f\n",
           c.name, at / 8, bits / (at / 8 * 1e-3) / 1e9, bt / 8, bits / (bt / 8 * 1e-3) / 1e9, r / 4);
    fflush(stdout);
  }
  return bad ? 2 : 0;
}
