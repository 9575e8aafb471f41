// divcheck.hip -- exhaustive check, on the device, that division by the channel's two constants can
// use the Markstein correction (q0 = a*r, e = fma(-q0, b, a), q = fma(e, r, q0), r = RN(1/b))
// instead of the IEEE division sequence (v_div_scale / v_div_fmas / v_div_fixup):
//   double: k / 2147483647.0 for every k in [0, 2^31)          (gaussian.c:23-24, u1 / u2)
//   float : x / ndist for every non-negative finite float x, and for 2^-60 <= x < 2^64 (demapper.c:70,
//           ndist of the n = 1, 2, 3 constellations)
// Prints the mismatch count per case (0 = the fast form is bit-identical for the whole domain).
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void check_double(unsigned long long* bad, unsigned long long* first) {
  const double M = 2147483647.0;
  const double r = 1.0 / M;
  const unsigned long long n = 1ull << 31;
  for (unsigned long long k = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; k < n;
       k += (unsigned long long)gridDim.x * blockDim.x) {
    const double a = (double)k;
    const double ref = a / M;
    const double q0 = a * r;
    const double e = __builtin_fma(-q0, M, a);
    const double q = __builtin_fma(e, r, q0);
    if (__double_as_longlong(q) != __double_as_longlong(ref)) {
      atomicAdd(bad, 1ull);
      atomicMin(first, k);
    }
  }
}

// [lo, hi) bit patterns: every non-negative finite float, or the channel's domain [2^-60, 2^64)
__global__ void check_float(float b, unsigned lo, unsigned long long hi, unsigned long long* bad,
                            unsigned long long* first) {
  const float r = 1.0f / b;
  const unsigned long long n = hi;
  for (unsigned long long i = lo + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    const float x = __uint_as_float((unsigned)i);
    const float ref = x / b;
    const float q0 = x * r;
    const float e = __builtin_fmaf(-q0, b, x);
    const float q = __builtin_fmaf(e, r, q0);
    if (__float_as_uint(q) != __float_as_uint(ref)) {
      atomicAdd(bad, 1ull);
      atomicMin(first, i);
    }
  }
}

int main() {
  unsigned long long *d, h[2];
  if (hipMalloc(&d, 16) != hipSuccess) return 1;
  auto run = [&](const char* name, auto launch) {
    h[0] = 0;
    h[1] = ~0ull;
    (void)hipMemcpy(d, h, 16, hipMemcpyHostToDevice);
    launch();
    (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("%-40s mismatches %llu (first at 0x%llx)\n", name, h[0], h[0] ? h[1] : 0ull);
  };
  run("double k / 2147483647.0, k < 2^31", [&] { hipLaunchKernelGGL(check_double, dim3(8192), dim3(256), 0, 0, d, d + 1); });
  // ndist of the reference constellations (common/constellations.c, demapper.c:61-65)
  const float q = 0.707107f;
  const float nd2 = ((q - q) * (q - q)) + ((q - (-q)) * (q - (-q)));   // n = 2: points 0 and 1
  const float nd1 = ((q - (-q)) * (q - (-q))) + ((q - (-q)) * (q - (-q)));
  const float a = 0.408248f, c = 1.224745f;
  const float nd3 = ((a - a) * (a - a)) + ((a - c) * (a - c));
  const float nds[3] = {nd1, nd2, nd3};
  for (float b : nds) {
    char name[64];
    snprintf(name, sizeof name, "float x / %.9g, all x >= 0 finite", b);
    run(name, [&] { hipLaunchKernelGGL(check_float, dim3(8192), dim3(256), 0, 0, b, 0u, 0x7f800000ull, d, d + 1); });
    // 2^-60 = 0x21800000, 2^64 = 0x5f800000: the channel's squared distances (channel_dev.hpp)
    snprintf(name, sizeof name, "float x / %.9g, 2^-60 <= x < 2^64", b);
    run(name, [&] { hipLaunchKernelGGL(check_float, dim3(8192), dim3(256), 0, 0, b, 0x21800000u, 0x5f800000ull, d, d + 1); });
  }
  return 0;
}
