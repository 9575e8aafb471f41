// persist_bench.hip -- timing ablations of the persistent K=7 soft kernel (acs_persist.hpp):
// full kernel, no input traffic (VALU + traceback only), no traceback, neither; at 2 and 3 waves/SIMD.
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -fno-slp-vectorize -I../include
//        -I../convolutional-codes_amd/csrc persist_bench.hip -o persist_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "acs_persist.hpp"

using namespace ccv;
constexpr CodeSpec kK7Ref{2, 7, {0xF200000000000000ull, 0xB600000000000000ull, 0, 0, 0, 0, 0, 0}, GEN_REF_X86};
constexpr CodeSpec kK7True{2, 7, {0xF200000000000000ull, 0xB600000000000000ull, 0, 0, 0, 0, 0, 0},
                           GEN_TRUE_PARITY};

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
      return 1;                                                               \
    }                                                                         \
  } while (0)

template <CodeSpec C, int AB, int BLEN = 40>
int run(const char* name, RegArgs a, int ngroups, int waves_per_cu, int cus) {
  auto kern = viterbi_soft_persist<C, BLEN, AB>;
  int per_cu = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, 0));
  const int w = waves_per_cu < per_cu ? waves_per_cu : per_cu;
  const int grid = w * cus < ngroups ? w * cus : ngroups;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 12; ++rep) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, a, ngroups);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (rep >= 2 && ms < best) best = ms;
  }
  // sustained: 40 back-to-back launches (as bench.py's timed steps), mean per launch
  CHECK(hipEventRecord(e0, 0));
  for (int rep = 0; rep < 40; ++rep) hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, a, ngroups);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float sus = 0;
  CHECK(hipEventElapsedTime(&sus, e0, e1));
  sus /= 40;
  const double bits = (double)ngroups * 64 * BLEN;
  printf("%-28s waves/CU %2d (max %2d)  isolated %.4f ms %6.1f Gbit/s  sustained %.4f ms %6.1f Gbit/s\n",
         name, w, per_cu, best, bits / (best * 1e-3) / 1e9, sus, bits / (sus * 1e-3) / 1e9);
  return 0;
}

// Per-launch times over a long back-to-back run: clock ramp-up vs power throttling.
template <CodeSpec C>
int trace(RegArgs a, int ngroups, int waves_per_cu, int cus, int n) {
  auto kern = viterbi_soft_persist<C, 40, 0>;
  const int grid = waves_per_cu * cus < ngroups ? waves_per_cu * cus : ngroups;
  std::vector<hipEvent_t> ev(n + 1);
  for (auto& evt : ev) CHECK(hipEventCreate(&evt));
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(ev[0], 0));
  for (int i = 0; i < n; ++i) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, a, ngroups);
    CHECK(hipEventRecord(ev[i + 1], 0));
  }
  CHECK(hipEventSynchronize(ev[n]));
  printf("trace (ms per launch, mean of 10):");
  for (int i = 0; i < n; i += 10) {
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, ev[i], ev[i + 10 < n ? i + 10 : n]));
    printf(" %.3f", ms / 10);
  }
  printf("\n");
  return 0;
}

// Interleaved A/B after a clock warm-up: each variant's sustained time in rounds A B C .. A B C ..,
// so clock ramp and box-to-box power differences do not bias one variant.
template <CodeSpec C, int AB, int BLEN = 40>
float sustained(RegArgs a, int ngroups, int waves_per_cu, int cus, int n) {
  auto kern = viterbi_soft_persist<C, BLEN, AB>;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, 0) != hipSuccess) return -1;
  const int w = waves_per_cu < per_cu ? waves_per_cu : per_cu;
  const int grid = w * cus < ngroups ? w * cus : ngroups;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  for (int rep = 0; rep < n; ++rep) hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, a, ngroups);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms / n;
}

// Paired A/B: production (A) against each variant (B) in ABBA blocks of 40 launches, so a linear
// clock/thermal drift cancels; the ratio B/A per block quadruple, mean and spread over 4 quadruples.
int ab(RegArgs a, int ng, int cus, bool only_first = false) {
  sustained<kK7Ref, 0>(a, ng, 8, cus, 300);   // clock warm-up
  RegArgs a42 = a;
  a42.T = 48;
  a42.blen = 42;
  const int ng42 = (int)((size_t)a.nblocks * 46 / 48) / 64;
  a42.nblocks = ng42 * 64;
  const float scale42 = (float)((double)ng * 40 / ((double)ng42 * 42));   // per blen-40 bit
  auto A = [&]() { return sustained<kK7Ref, 0>(a, ng, 8, cus, 40); };
  struct V { const char* name; float (*f)(RegArgs, int, int, int, int); bool b42; };
  const V vs_all[] = {
    {"input nt (aux 2)", sustained<kK7Ref, kPersistInputNt>, false},
    {"2-deep DMA", sustained<kK7Ref, kPersistDepth2>, false},
    {"no DMA (stale LDS rows)", sustained<kK7Ref, kPersistNoDma>, false},
    {"DMA, no LDS reads (synth)", sustained<kK7Ref, kPersistNoLdsRead>, false},
    {"no memory, synth rows", sustained<kK7Ref, kPersistNoMem | kPersistNoMemRandom>, false},
    {"blen42 aligned (per bit)", sustained<kK7Ref, 0, 42>, true},
    {"L2-resident input", sustained<kK7Ref, kPersistCachedInput>, false},
    {"no traceback", sustained<kK7Ref, kPersistNoTraceback>, false},
    {"no memory, int rows", sustained<kK7Ref, kPersistNoMem>, false},
  };
  double asum = 0;
  int an = 0;
  const int nv = only_first ? 1 : (int)(sizeof(vs_all) / sizeof(vs_all[0]));
  for (int vi = 0; vi < nv; ++vi) {
    const V& v = vs_all[vi];
    double r[4], rs = 0, lo = 1e9, hi = 0;
    for (int q = 0; q < 4; ++q) {
      auto B = [&]() { return v.b42 ? v.f(a42, ng42, 8, cus, 40) * scale42 : v.f(a, ng, 8, cus, 40); };
      const float a0 = A(), b0 = B(), b1 = B(), a1 = A();
      asum += a0 + a1;
      an += 2;
      r[q] = (b0 + b1) / (a0 + a1);
      rs += r[q];
      lo = r[q] < lo ? r[q] : lo;
      hi = r[q] > hi ? r[q] : hi;
    }
    printf("%-26s time ratio vs production %.3f (%.3f .. %.3f)\n", v.name, rs / 4, lo, hi);
  }
  const double bits = (double)ng * 64 * 40;
  printf("production mean %.4f ms  %.1f Gbit/s\n", asum / an, bits / (asum / an * 1e-3) / 1e9);
  return 0;
}

template <CodeSpec C, int MM>
float sustained_hard(RegArgs a, int ngroups, int waves_per_cu, int cus, int n) {
  auto kern = viterbi_hard_persist<C, 40, MM>;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, 0) != hipSuccess) return -1;
  const int w = waves_per_cu < per_cu ? waves_per_cu : per_cu;
  const int grid = w * cus < ngroups ? w * cus : ngroups;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  for (int rep = 0; rep < n; ++rep) hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, a, ngroups);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms / n;
}

// BSC persistent kernel: 16-bit inline-asm metrics (production) against plain u32 metrics, ABBA.
template <int MODE>
int ab_hard(int cus) {
  const int nb = 1600000, T = 46, ng = nb / 64;
  std::vector<uint8_t> h((size_t)nb * T);
  uint32_t x = 777;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    v = (uint8_t)(x >> 30);
  }
  uint8_t *d_in, *d_out;
  CHECK(hipMalloc(&d_in, h.size()));
  CHECK(hipMalloc(&d_out, (size_t)nb * 8));
  CHECK(hipMemcpy(d_in, h.data(), h.size(), hipMemcpyHostToDevice));
  RegArgs a{};
  a.in = d_in;
  a.T = T;
  a.nblocks = nb;
  a.blen = 40;
  a.out = d_out;
  sustained_hard<kK7Ref, 0>(a, ng, 8, cus, 300);
  double rs = 0, asum = 0;
  for (int q = 0; q < 4; ++q) {
    const float a0 = sustained_hard<kK7Ref, 0>(a, ng, 8, cus, 40), b0 = sustained_hard<kK7Ref, MODE>(a, ng, 8, cus, 40),
                b1 = sustained_hard<kK7Ref, MODE>(a, ng, 8, cus, 40), a1 = sustained_hard<kK7Ref, 0>(a, ng, 8, cus, 40);
    rs += (b0 + b1) / (a0 + a1);
    asum += a0 + a1;
    printf("quad %d: h16 %.4f %.4f  u32 %.4f %.4f\n", q, a0, a1, b0, b1);
  }
  printf("hard mode %d metrics: time ratio vs h16", MODE); printf(" %.3f; h16 %.4f ms %.1f Gbit/s\n", rs / 4, asum / 8,
         (double)ng * 64 * 40 / (asum / 8 * 1e-3) / 1e9);
  return 0;
}

int main(int argc, char** argv) {
  const int nb = 1600000, T = 46;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<float> h((size_t)nb * T * 4);
  uint32_t x = 12345;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    v = (float)(x >> 8) * (1.0f / 16777216.0f) * 3.0f;
  }
  float* d_in;
  uint8_t* d_out;
  CHECK(hipMalloc(&d_in, h.size() * 4));
  CHECK(hipMalloc(&d_out, (size_t)nb * 8));
  CHECK(hipMemcpy(d_in, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  RegArgs a{};
  a.in = d_in;
  a.T = T;
  a.nblocks = nb;
  a.blen = 40;
  a.out = d_out;
  const int ng = nb / 64;
  if (argc > 1 && std::string(argv[1]) == "ab") return ab(a, ng, cus);
  if (argc > 1 && std::string(argv[1]) == "abtw") return ab(a, ng, cus, true);   // twin classes only
  if (argc > 1 && std::string(argv[1]) == "abh") return ab_hard<1>(cus) | ab_hard<2>(cus);
  if (argc > 1) {   // persist_bench trace [launches]
    const int n = argc > 2 ? atoi(argv[2]) : 300;
    trace<kK7Ref>(a, ng, 8, cus, n);
    return 0;
  }
  for (int w : {8}) {
    run<kK7Ref, 0>("ref full", a, ng, w, cus);
    run<kK7Ref, kPersistNoMem>("ref no-mem", a, ng, w, cus);
    run<kK7Ref, kPersistNoTraceback>("ref no-traceback", a, ng, w, cus);
    run<kK7Ref, kPersistNoMem | kPersistNoTraceback>("ref no-mem no-traceback", a, ng, w, cus);
  }
  run<kK7Ref, kPersistDepth2>("ref full, 2-deep double-buffered DMA", a, ng, 8, cus);
  {   // blen 42: T = 48, a block is exactly 6 x 128-byte lines -> no chunk straddles a line
    RegArgs a42 = a;
    a42.T = 48;
    a42.blen = 42;
    const int nb42 = (int)((size_t)nb * 46 / 48) / 64 * 64;   // same input bytes
    a42.nblocks = nb42;
    run<kK7Ref, 0, 42>("ref full blen42 (aligned)", a42, nb42 / 64, 8, cus);
    run<kK7Ref, kPersistCachedInput, 42>("ref blen42 L2-resident", a42, nb42 / 64, 8, cus);
  }
  run<kK7Ref, kPersistCachedInput>("ref full, L2-resident input", a, ng, 8, cus);
  run<kK7Ref, kPersistCachedInput | kPersistNoTraceback>("ref L2 input, no-tb", a, ng, 8, cus);
  run<kK7Ref, kPersistSelectAcs>("ref select-acs full", a, ng, 8, cus);
  run<kK7Ref, kPersistSelectAcs | kPersistNoMem | kPersistNoTraceback>("ref select-acs no-mem no-tb", a, ng, 8, cus);
  run<kK7True, kPersistSelectAcs>("true select-acs full", a, ng, 8, cus);
  run<kK7True, kPersistSelectAcs | kPersistNoMem | kPersistNoTraceback>("true select-acs no-mem no-tb", a, ng, 8, cus);
  run<kK7True, 0>("true full", a, ng, 8, cus);
  run<kK7True, kPersistNoMem | kPersistNoTraceback>("true no-mem no-traceback", a, ng, 8, cus);
  return 0;
}
