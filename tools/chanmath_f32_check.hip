// chanmath_f32_check.hip -- error analysis of the opt-in fp32 Box-Muller of the on-device channel
// (channel_dev.hpp box_muller_f32, CCV_CHANNEL_NOISE_F32) against the production double-precision one
// (channel_math.hpp neg2_log / sqrt_nonneg / sincos_2pi, itself within a few ulp of glibc), over EVERY
// uniform the channel can draw: all k1 in [1, 2^31 - 1] for R = sqrt(-2 ln(k1 / M)) and all k2 in
// [0, 2^31 - 1] for (cos, sin)(2 pi k2 / M), M = 2^31 - 1, computed on the device.
// Reports the largest absolute and relative error of R per decade of u1 (the tail u1 -> 2^-31 is where
// the largest noise samples come from) and the largest absolute sin / cos errors, then the bound on a
// noisy coordinate x + scaling * R * cos: |err| <= scaling * (dR + R_max * dTrig) + 2 fp32 roundings.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../convolutional-codes_amd/csrc -I../include
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

#include "channel_dev.hpp"

constexpr int kBins = 11;   // u1 decades: [1e-1, 1], [1e-2, 1e-1], ..., below 1e-10

__device__ __forceinline__ void amax(float* p, float v) {
  atomicMax(reinterpret_cast<unsigned int*>(p), __float_as_uint(v));   // v >= 0
}

__global__ void check_r(float* abs_err, float* rel_err, float* rmax) {
  __shared__ float sa[kBins], sr[kBins], sm;
  if (threadIdx.x < kBins) sa[threadIdx.x] = sr[threadIdx.x] = 0.0f;
  if (threadIdx.x == 0) sm = 0.0f;
  __syncthreads();
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; k < 2147483648ull;
       k += (uint64_t)gridDim.x * blockDim.x) {
    const double u1 = ccv::div_rand_max((uint32_t)k);
    const double r64 = ccv::chanmath::sqrt_nonneg(ccv::chanmath::neg2_log(u1));
    const float r32 = ccv::radius_f32((uint32_t)k);
    const double e = fabs((double)r32 - r64);
    int bin = (int)floor(-log10(u1));
    bin = bin < 0 ? 0 : (bin >= kBins ? kBins - 1 : bin);
    amax(&sa[bin], (float)e);
    if (r64 > 0.0) amax(&sr[bin], (float)(e / r64));
    amax(&sm, (float)r64);
  }
  __syncthreads();
  if (threadIdx.x < kBins) {
    amax(&abs_err[threadIdx.x], sa[threadIdx.x]);
    amax(&rel_err[threadIdx.x], sr[threadIdx.x]);
  }
  if (threadIdx.x == 0) amax(rmax, sm);
}

__global__ void check_trig(float* err) {   // err[0] cos, err[1] sin
  __shared__ float sc, ss;
  if (threadIdx.x == 0) sc = ss = 0.0f;
  __syncthreads();
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < 2147483648ull;
       k += (uint64_t)gridDim.x * blockDim.x) {
    const double u2 = ccv::div_rand_max((uint32_t)k);
    double s64, c64;
    ccv::chanmath::sincos_2pi(u2, &s64, &c64);
    const float u = (float)k * (1.0f / 2147483647.0f);
    const float c32 = __builtin_amdgcn_cosf(u), s32 = __builtin_amdgcn_sinf(u);
    amax(&sc, (float)fabs((double)c32 - c64));
    amax(&ss, (float)fabs((double)s32 - s64));
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    amax(&err[0], sc);
    amax(&err[1], ss);
  }
}

int main() {
  float *d = nullptr, h[2 * kBins + 3] = {};
  if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
  (void)hipMemset(d, 0, sizeof h);
  hipLaunchKernelGGL(check_r, dim3(8192), dim3(256), 0, 0, d, d + kBins, d + 2 * kBins);
  hipLaunchKernelGGL(check_trig, dim3(8192), dim3(256), 0, 0, d + 2 * kBins + 1);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  std::printf("fp32 Box-Muller vs the double-precision channel, every k1 in [1, 2^31 - 1], every k2\n");
  std::printf("u1 decade            max |dR|      max |dR|/R\n");
  float worst_abs = 0.0f;
  for (int b = 0; b < kBins; ++b) {
    std::printf("[1e-%-2d, 1e-%-2d]     %.3e    %.3e\n", b + 1, b, h[b], h[kBins + b]);
    worst_abs = h[b] > worst_abs ? h[b] : worst_abs;
  }
  const float rmax = h[2 * kBins], ec = h[2 * kBins + 1], es = h[2 * kBins + 2];
  std::printf("R_max %.6f; max |d cos| %.3e, max |d sin| %.3e\n", rmax, ec, es);
  const float trig = ec > es ? ec : es;
  std::printf("noisy coordinate: |err| <= scaling * (%.3e + %.6f * %.3e) = scaling * %.3e, plus two fp32 "
              "roundings of the result\n", worst_abs, rmax, trig, worst_abs + rmax * trig);
  return 0;
}
