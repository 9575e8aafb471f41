// kbench.hip -- microbenchmark of soft register-trellis kernel variants (input paths, chunking) on
// K=7 (171,133), interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -fno-slp-vectorize -I include
//        -I convolutional-codes_amd/csrc tools/kbench.hip -o tools/kbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "acs_reg.hpp"
#include "reg_codes.hpp"

using namespace ccv;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr CodeSpec kK7Ref = kRegCodes[8];
constexpr CodeSpec kK7True = kRegCodes[9];

template <CodeSpec C>
void launch_rd(const RegArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((viterbi_soft_regdec<C>), dim3(grid), dim3(kRegThreads), 0, s, a);
}

struct Variant {
  const char* name;
  void (*launch)(const RegArgs&, int, hipStream_t);
  bool step_major;
};

template <CodeSpec C, int MODE, int PF, int AB = 0, int NT = 0>
void launch_v(const RegArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((viterbi_soft_reg<C, MODE, PF, AB, NT>), dim3(grid), dim3(kRegThreads), 0, s, a);
}

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 400000;
  const int rounds = argc > 2 ? atoi(argv[2]) : 10;
  const char* filter = argc > 3 ? argv[3] : "";
  const int T = 46, NS = 4;
  std::vector<float> h((size_t)nb * T * NS), hs(h.size());
  std::mt19937 rng(1);
  std::exponential_distribution<float> ex(1.0f);
  if (const char* f = getenv("KB_INPUT")) {   // raw float32 [nb][T][4], e.g. the bench's AWGN frames
    FILE* fp = fopen(f, "rb");
    if (!fp || fread(h.data(), 4, h.size(), fp) != h.size()) { fprintf(stderr, "bad KB_INPUT\n"); return 1; }
    fclose(fp);
  } else {
    for (auto& x : h) x = ex(rng);
  }
  for (int b = 0; b < nb; ++b)
    for (int t = 0; t < T; ++t)
      for (int k = 0; k < NS; ++k) hs[((size_t)t * nb + b) * NS + k] = h[((size_t)b * T + t) * NS + k];
  float *d_in, *d_ins;
  uint8_t* d_out;
  void* d_dec;
  unsigned long long* d_err;
  CK(hipMalloc(&d_in, h.size() * 4));
  CK(hipMalloc(&d_ins, h.size() * 4));
  CK(hipMalloc(&d_out, (size_t)nb * 6));
  CK(hipMalloc(&d_dec, (size_t)(nb + 63) / 64 * 64 * T * 8));
  CK(hipMalloc(&d_err, 8));
  uint8_t* d_info = nullptr;
  CK(hipMalloc(&d_info, (size_t)nb * 5));
  CK(hipMemset(d_info, 0x5a, (size_t)nb * 5));
  const bool with_err = getenv("KB_ERR") != nullptr;   // fused error count, as bench.py runs it
  CK(hipMemcpy(d_in, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ins, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
  Variant vs[] = {
      {"ref/per-step4", launch_v<kK7Ref, kLoadPerStep, 4>, false},
      {"ref/per-step8", launch_v<kK7Ref, kLoadPerStep, 8>, false},
      {"ref/lds-dma4", launch_v<kK7Ref, kLoadLdsDma, 4>, false},
      {"ref/lds-dma8", launch_v<kK7Ref, kLoadLdsDma, 8>, false},
      {"ref/step-major4", launch_v<kK7Ref, kLoadStepMajor, 4>, true},
      {"ref/step-major8", launch_v<kK7Ref, kLoadStepMajor, 8>, true},
      {"true/per-step4", launch_v<kK7True, kLoadPerStep, 4>, false},
      {"true/per-step8", launch_v<kK7True, kLoadPerStep, 8>, false},
      {"true/lds-dma4", launch_v<kK7True, kLoadLdsDma, 4>, false},
      {"true/lds-dma8", launch_v<kK7True, kLoadLdsDma, 8>, false},
      {"true/step-major4", launch_v<kK7True, kLoadStepMajor, 4>, true},
      {"true/step-major8", launch_v<kK7True, kLoadStepMajor, 8>, true},
      {"ref/dma4-nt", launch_v<kK7Ref, kLoadLdsDma, 4, 0, 1>, false},
      {"ref/dma8-nt", launch_v<kK7Ref, kLoadLdsDma, 8, 0, 1>, false},
      {"ref/sm4-nt", launch_v<kK7Ref, kLoadStepMajor, 4, 0, 1>, true},
      {"true/dma4-nt", launch_v<kK7True, kLoadLdsDma, 4, 0, 1>, false},
      {"true/dma8-nt", launch_v<kK7True, kLoadLdsDma, 8, 0, 1>, false},
      {"true/sm4-nt", launch_v<kK7True, kLoadStepMajor, 4, 0, 1>, true},
      {"true/sm4-nodecst", launch_v<kK7True, kLoadStepMajor, 4, kAblateDecStore>, true},
      {"true/sm4-notb", launch_v<kK7True, kLoadStepMajor, 4, kAblateTraceback>, true},
      {"true/sm4-neither", launch_v<kK7True, kLoadStepMajor, 4, 3>, true},
      {"true/ps8-neither", launch_v<kK7True, kLoadPerStep, 8, 3>, false},
      {"true/noload-neither", launch_v<kK7True, kLoadStepMajor, 4, 7>, true},
      {"ref/noload-neither", launch_v<kK7Ref, kLoadStepMajor, 4, 7>, true},
      {"true/noload", launch_v<kK7True, kLoadStepMajor, 4, 4>, true},
      {"ref/regdec", launch_rd<kK7Ref>, false},
      {"true/regdec", launch_rd<kK7True>, false},
      {"ref/dma8-nodecst", launch_v<kK7Ref, kLoadLdsDma, 8, kAblateDecStore>, false},
      {"ref/dma8-notb", launch_v<kK7Ref, kLoadLdsDma, 8, kAblateTraceback>, false},
      {"ref/dma8-neither", launch_v<kK7Ref, kLoadLdsDma, 8, 3>, false},
  };
  const int nv = sizeof(vs) / sizeof(vs[0]);
  const char* ring_env = getenv("KB_FRAMES");   // >1: rotate over distinct input copies (> MALL)
  (void)ring_env;
  std::vector<std::vector<float>> ms(nv);
  std::vector<std::vector<uint8_t>> outs(nv, std::vector<uint8_t>((size_t)nb * 6));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = (nb + kRegThreads - 1) / kRegThreads;
  for (int r = 0; r < rounds + 1; ++r) {
    for (int v = 0; v < nv; ++v) {
      if (!strstr(vs[v].name, filter)) continue;
      RegArgs a{};
      a.in = vs[v].step_major ? (const void*)d_ins : (const void*)d_in;
      a.T = T; a.nblocks = nb; a.blen = 40; a.out = d_out; a.dec = d_dec;
      a.dec_stride = (nb + 63) / 64 * 64;
      if (with_err) { a.info = d_info; a.err = d_err; }
      const int burst = getenv("KB_BURST") ? atoi(getenv("KB_BURST")) : 1;   // back-to-back launches
      CK(hipEventRecord(e0, 0));
      for (int q = 0; q < burst; ++q) vs[v].launch(a, grid, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (r > 0) ms[v].push_back(t / burst);
      if (r == 0) CK(hipMemcpy(outs[v].data(), d_out, outs[v].size(), hipMemcpyDeviceToHost));
    }
  }
  for (int v = 0; v < nv; ++v) {
    if (!strstr(vs[v].name, filter)) continue;
    std::sort(ms[v].begin(), ms[v].end());
    int ref = strncmp(vs[v].name, "ref", 3) == 0 ? 0 : 6;
    bool same = outs[v] == outs[ref];
    double gbit = (double)nb * 40 / (ms[v][ms[v].size() / 2] * 1e-3) / 1e9;
    printf("%-18s median %.4f ms  min %.4f ms  %.1f Gbit/s  %s\n", vs[v].name, ms[v][ms[v].size() / 2],
           ms[v][0], gbit, same ? "same-output" : "OUTPUT-DIFFERS");
  }
  return 0;
}
