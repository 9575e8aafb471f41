// lat_probe.hip -- where a lone block's time goes in the streaming latency kernel (acs_latency.hpp).
// Launches viterbi_latency on one block, synchronising after each launch as the launch-per-block
// streaming path does, with the block's input and output in device memory or in page-locked host
// memory (zero-copy, the production streaming layout), and reads the kernel's 100 MHz phase stamps
// (built with -DCCV_LAT_STAMPS): stage (input + expected-symbol table), forward ACS, argmin,
// traceback. Timing only: synthetic input and expected-symbol tables.
// build: hipcc -O3 -std=c++20 --offload-arch=gfx950 -DCCV_LAT_STAMPS -Iconvolutional-codes_amd/csrc
//        -Iinclude tools/lat_probe.hip -o tools/lat_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "acs_latency.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

static void run(const char* name, int K, int n, int blen, bool hard, bool host_mem, int iters) {
  const int T = blen + K - 1, S = 1 << (K - 1), NS = 1 << n, OB = (T + 7) / 8;
  const size_t in_bytes = hard ? (size_t)T : (size_t)T * NS * 4;
  std::vector<uint8_t> exp_h(2 * S);
  for (int k = 0; k < 2 * S; ++k) exp_h[k] = (uint8_t)((k * 7 + 3) % NS);
  std::vector<uint8_t> in_h(in_bytes);
  for (size_t k = 0; k < in_bytes; ++k) in_h[k] = (uint8_t)(hard ? (k * 5) % NS : 0);
  if (!hard)
    for (int k = 0; k < T * NS; ++k) reinterpret_cast<float*>(in_h.data())[k] = (float)((k * 37) % 11) * 0.25f;
  uint8_t *d_exp, *in, *out;
  int32_t* pm;
  CK(hipMalloc(&d_exp, exp_h.size()));
  CK(hipMemcpy(d_exp, exp_h.data(), exp_h.size(), hipMemcpyHostToDevice));
  if (host_mem) {
    CK(hipHostMalloc(&in, in_bytes, hipHostMallocMapped));
    CK(hipHostMalloc(&out, 64, hipHostMallocMapped));
    CK(hipHostMalloc(&pm, 64, hipHostMallocMapped));
    std::copy(in_h.begin(), in_h.end(), in);
  } else {
    CK(hipMalloc(&in, in_bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&pm, 64));
    CK(hipMemcpy(in, in_h.data(), in_bytes, hipMemcpyHostToDevice));
  }
  ccv::GenericArgs a{};
  a.in = in; a.exp = d_exp; a.n = n; a.K = K; a.T = T; a.blen = blen; a.nblocks = 1; a.chunk = T;
  a.out = out; a.path_metric = hard ? pm : nullptr;
  const size_t lds = ccv::latency_lds_bytes(n, T, hard);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<double> wall, kern, ph[4], ghz;
  for (int it = 0; it < iters; ++it) {
    const auto t0 = std::chrono::steady_clock::now();
    CK(hipEventRecord(e0, 0));
    if (K == 7) {
      if (hard) hipLaunchKernelGGL((ccv::viterbi_latency<true, 6>), dim3(1), dim3(64), lds, 0, a);
      else hipLaunchKernelGGL((ccv::viterbi_latency<false, 6>), dim3(1), dim3(64), lds, 0, a);
    } else {
      if (hard) hipLaunchKernelGGL((ccv::viterbi_latency<true, 2>), dim3(1), dim3(64), lds, 0, a);
      else hipLaunchKernelGGL((ccv::viterbi_latency<false, 2>), dim3(1), dim3(64), lds, 0, a);
    }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    const auto t1 = std::chrono::steady_clock::now();
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long st[16];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(ccv::ccv_lat_stamps), sizeof st));
    if (it < 50) continue;   // warm-up
    wall.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    kern.push_back(ms * 1e3);
    for (int k = 0; k < 4; ++k) ph[k].push_back((double)(st[k + 1] - st[k]) * 0.01);   // 100 MHz ticks -> us
    ghz.push_back((double)(st[12] - st[8]) / ((double)(st[4] - st[0]) * 10.0));      // shader clocks per ns
  }
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  std::printf("%-22s %-6s wall %7.2f  event %7.2f  stage %6.2f  forward %6.2f  argmin %6.2f  traceback %6.2f us"
              "  s_memtime/ns %.3f\n", name, host_mem ? "host" : "device", med(wall), med(kern), med(ph[0]), med(ph[1]),
              med(ph[2]), med(ph[3]), med(ghz));
  if (host_mem) { CK(hipHostFree(in)); CK(hipHostFree(out)); CK(hipHostFree(pm)); }
  else { CK(hipFree(in)); CK(hipFree(out)); CK(hipFree(pm)); }
  CK(hipFree(d_exp));
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 1000;
  for (int host = 0; host < 2; ++host) {
    run("soft K=7 n=2 blen=40", 7, 2, 40, false, host, iters);
    run("hard K=7 n=2 blen=40", 7, 2, 40, true, host, iters);
    run("hard K=3 n=2 blen=40", 3, 2, 40, true, host, iters);
    run("soft K=3 n=2 blen=40", 3, 2, 40, false, host, iters);
  }
  return 0;
}
