// k9_bench.hip -- timing ablations of the persistent K=9 soft kernel (acs_multi.hpp
// viterbi_multi_persist): production, the round-2 ds_bpermute traceback, no traceback, no input
// traffic (synthetic rows), neither. Outputs of the production and round-2 variants are compared
// byte for byte. Build: make -C tools k9_bench (or the hipcc line below).
//   hipcc -O3 -std=c++20 --offload-arch=gfx950 -fno-slp-vectorize -I../include
//         -I../convolutional-codes_amd/csrc k9_bench.hip -o k9_bench
// usage: k9_bench [frames=16]; build with -DCCV_VMIN_BUILTIN for the compiler's v_min (A/B of the
// inline-asm one). Also times the K=7 headline persistent kernel at 104 frames.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <vector>

#include "acs_multi.hpp"
#include "reg_codes.hpp"

using namespace ccv;
constexpr CodeSpec kK9 = kMultiCodes[2];   // K=9 (561,753) x86 idiom
constexpr CodeSpec kK7 = kRegCodes[8];     // K=7 (171,133) x86 idiom (the headline kernel)

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

template <int AB, int LDSP = 0, int LB0 = 6, int LB1 = 7>
double run(const char* name, RegArgs a, int ngroups, int cus) {
  auto kern = viterbi_multi_persist<kK9, 40, AB, LDSP, LB0, LB1>;
  int per_cu = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, 0));
  if (per_cu >= 4) per_cu -= per_cu % 4;
  const int grid = per_cu * cus < ngroups ? per_cu * cus : ngroups;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int rep = 0; rep < 100; ++rep) hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, a, ngroups);
  CHECK(hipEventRecord(e0, 0));
  for (int rep = 0; rep < 40; ++rep) hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, a, ngroups);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 40;
  const double bits = (double)a.nblocks * 40;
  printf("%-34s waves/CU %2d  %.4f ms  %6.2f Gbit/s\n", name, per_cu, ms, bits / (ms * 1e-3) / 1e9);
  fflush(stdout);
  return ms;
}

// the headline K=7 persistent kernel at 104 frames (bench.py's workload), same timing loop
double run_k7(int frames, int cus) {
  const int nb = frames * 25000, T = 46, ngroups = (nb + 63) / 64;
  std::vector<float> h_in((size_t)nb * T * 4);
  uint32_t x = 777;
  for (auto& v : h_in) {
    x = x * 1664525u + 1013904223u;
    v = (float)(x >> 8) * (4.0f / 16777216.0f);
  }
  float* d_in;
  uint8_t* d_out;
  CHECK(hipMalloc(&d_in, h_in.size() * 4));
  CHECK(hipMemcpy(d_in, h_in.data(), h_in.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMalloc(&d_out, (size_t)nb * 6));
  RegArgs a{};
  a.in = d_in;
  a.T = T;
  a.nblocks = nb;
  a.blen = 40;
  a.out = d_out;
  auto kern = viterbi_soft_persist<kK7, 40, 0>;
  int per_cu = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, 0));
  if (per_cu >= 4) per_cu -= per_cu % 4;
  const int grid = per_cu * cus < ngroups ? per_cu * cus : ngroups;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int rep = 0; rep < 200; ++rep) hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, a, ngroups);
  CHECK(hipEventRecord(e0, 0));
  for (int rep = 0; rep < 40; ++rep) hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, a, ngroups);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 40;
  printf("%-34s waves/CU %2d  %.4f ms  %6.2f Gbit/s\n", "K=7 headline persistent", per_cu, ms,
         (double)nb * 40 / (ms * 1e-3) / 1e9);
  fflush(stdout);
  CHECK(hipFree(d_in));
  CHECK(hipFree(d_out));
  return ms;
}

int main(int argc, char** argv) {
  const int frames = argc > 1 ? atoi(argv[1]) : 16;
  const int nb = frames * 25000, T = 48, ngroups = (nb + 15) / 16;
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  std::vector<float> h_in((size_t)nb * T * 4);
  uint32_t x = 12345;
  for (auto& v : h_in) {   // demapper-like distances in [0, 4)
    x = x * 1664525u + 1013904223u;
    v = (float)(x >> 8) * (4.0f / 16777216.0f);
  }
  float* d_in;
  uint8_t *d_out, *d_out2;
  CHECK(hipMalloc(&d_in, h_in.size() * 4));
  CHECK(hipMemcpy(d_in, h_in.data(), h_in.size() * 4, hipMemcpyHostToDevice));
  const size_t out_bytes = (size_t)nb * 4 * 8;   // no-traceback variants write 8 B per lane
  CHECK(hipMalloc(&d_out, out_bytes));
  CHECK(hipMalloc(&d_out2, out_bytes));
  RegArgs a{};
  a.in = d_in;
  a.T = T;
  a.nblocks = nb;
  a.blen = 40;
  a.out = d_out;
  run<0>("production (DPP traceback)", a, ngroups, cus);
  RegArgs b = a;
  b.out = d_out2;
  run<kMultiBpermuteTraceback>("round-2 ds_bpermute traceback", b, ngroups, cus);
  std::vector<uint8_t> o1((size_t)nb * 6), o2((size_t)nb * 6);
  CHECK(hipMemcpy(o1.data(), d_out, o1.size(), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(o2.data(), d_out2, o2.size(), hipMemcpyDeviceToHost));
  printf("outputs identical: %s\n", memcmp(o1.data(), o2.data(), o1.size()) == 0 ? "yes" : "NO");
  RegArgs c = a;
  c.out = d_out2;
  auto check = [&]() {
    CHECK(hipMemcpy(o2.data(), d_out2, o2.size(), hipMemcpyDeviceToHost));
    if (memcmp(o1.data(), o2.data(), o1.size()) != 0) printf("   OUTPUTS DIFFER\n");
  };
  // round-robin repeats: the clock drifts over a run, so candidates are interleaved and the median
  // of each one's repeats is compared
  std::vector<std::vector<double>> t(7);
  const char* names[7] = {"production {6,7}", "{0,3} LDS x2", "{0,5} LDS x2", "{2,5}", "{2,5} LDS x3",
                          "{4,7} LDS x2", "{0,3}"};
  for (int round = 0; round < 5; ++round) {
    t[0].push_back(run<0>(names[0], a, ngroups, cus));
    t[1].push_back(run<0, 2, 0, 3>(names[1], c, ngroups, cus)); check();
    t[2].push_back(run<0, 2, 0, 5>(names[2], c, ngroups, cus)); check();
    t[3].push_back(run<0, 0, 2, 5>(names[3], c, ngroups, cus)); check();
    t[4].push_back(run<0, 3, 2, 5>(names[4], c, ngroups, cus)); check();
    t[5].push_back(run<0, 2, 4, 7>(names[5], c, ngroups, cus)); check();
    t[6].push_back(run<0, 0, 0, 3>(names[6], c, ngroups, cus)); check();
  }
  printf("medians (relative to production):\n");
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  for (int k = 0; k < 7; ++k)
    printf("  %-20s %.4f ms  %.3f\n", names[k], med(t[k]), med(t[k]) / med(t[0]));
  run<kMultiNoTraceback>("no traceback", a, ngroups, cus);
  run<kMultiNoMem>("no input traffic", a, ngroups, cus);
  run<kMultiNoMem | kMultiNoTraceback>("no input, no traceback", a, ngroups, cus);
  run<0>("production (again)", a, ngroups, cus);
  CHECK(hipFree(d_in));
  run_k7(104, cus);
  return 0;
}
