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
#include "acs_wide.hpp"
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

// the one-lane-per-block kernel (acs_wide.hpp), decisions in a per-wave global scratch slot
template <int AB = 0, int PACK = 0>
double run_wide(const char* name, RegArgs a, int ngroups, int cus) {
  auto kern = viterbi_wide_persist<kK9, 40, AB, PACK>;
  ngroups = (a.nblocks + 63) / 64;   // 64-block groups (one lane per block)
  int per_cu = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, 0));
  if (per_cu >= 4) per_cu -= per_cu % 4;
  const int grid = per_cu * cus < ngroups ? per_cu * cus : ngroups;
  static void* scratch = nullptr;
  if (!scratch) CHECK(hipMalloc(&scratch, (size_t)grid * wide_slot_bytes<kK9>(40)));
  a.dec = scratch;
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
  printf("%-34s waves/CU %2d  %.4f ms  %6.2f Gbit/s\n", name, per_cu, ms, (double)a.nblocks * 40 / (ms * 1e-3) / 1e9);
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
  const bool wide_only = argc > 2 && strcmp(argv[2], "wide") == 0;
  {
    std::vector<std::vector<double>> t(2);
    const char* names[2] = {"production {0,3} LDS x2", "one lane per block (wide)"};
    for (int round = 0; round < (wide_only ? 1 : 5); ++round) {
      t[0].push_back(run<0, 2, 0, 3>(names[0], a, ngroups, cus));
      CHECK(hipMemcpy(o1.data(), d_out, o1.size(), hipMemcpyDeviceToHost));
      t[1].push_back(run_wide(names[1], c, ngroups, cus)); check();
    }
    printf("medians (relative to production):\n");
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    for (int k = 0; k < 2; ++k) printf("  %-26s %.4f ms  %.3f\n", names[k], med(t[k]), med(t[k]) / med(t[0]));
    {
      std::vector<std::vector<double>> tw(4);
      const char* wn[4] = {"wide (8 words per step)", "packed 6 words (collapsed butterflies)", "5 words, one per twin class", "5 words, no table (wrong output)"};
      for (int round = 0; round < 5; ++round) {
        tw[0].push_back(run_wide<0>(wn[0], c, ngroups, cus)); check();
        tw[1].push_back(run_wide<0, 1>(wn[1], c, ngroups, cus)); check();
        tw[2].push_back(run_wide<0, 2>(wn[2], c, ngroups, cus)); check();
        tw[3].push_back(run_wide<32, 2>(wn[3], c, ngroups, cus));
      }
      for (int k = 0; k < 4; ++k) printf("  %-26s %.4f ms  %.3f\n", wn[k], med(tw[k]), med(tw[k]) / med(tw[0]));
    }
    run_wide<1>("wide, no decision stores", c, ngroups, cus);
    if (wide_only) return 0;
  }
  run<kMultiNoTraceback>("no traceback", a, ngroups, cus);
  run<kMultiNoMem>("no input traffic", a, ngroups, cus);
  run<kMultiNoMem | kMultiNoTraceback>("no input, no traceback", a, ngroups, cus);
  run<0>("production (again)", a, ngroups, cus);
  CHECK(hipFree(d_in));
  run_k7(104, cus);
  return 0;
}
