// Host check of csrc/channel_math.hpp (the on-device channel's Box-Muller pieces) against glibc,
// the producer of the host frames (csrc/sim.cpp:150-170) the device channel tests compare with.
// The hardware rcp / rsq approximations are emulated with their low 28 mantissa bits cleared, so
// the Newton / Goldschmidt corrections run as they must on the device.
//
//   g++ -O2 -std=c++20 -o /tmp/chanmath_check tools/chanmath_check.cpp && /tmp/chanmath_check [M draws]
//
// Reports (1) the largest error of each piece in ulp of the long-double value and (2) the fraction
// of fp32 channel samples (point 0.707107 + scaling * R * cos / sin, Eb/N0 0..14 dB) that differ
// from the glibc-based ones.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

static double trunc28(double x) {
  uint64_t b;
  std::memcpy(&b, &x, 8);
  b &= ~((1ull << 28) - 1);
  std::memcpy(&x, &b, 8);
  return x;
}
static double ccv_rcp_approx(double d) { return trunc28(1.0 / d); }
static double ccv_rsq_approx(double x) { return x > 0 ? trunc28(1.0 / std::sqrt(x)) : INFINITY; }
static double ccv_fma_const(double a, double b, double c) { return __builtin_fma(a, b, c); }
#define CCV_HD
#include "../convolutional-codes_amd/csrc/channel_math.hpp"

static uint64_t sm = 0x9E3779B97F4A7C15ull;
static uint64_t splitmix() {
  uint64_t z = (sm += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static double div_rand_max(uint32_t k) { return (double)k / 2147483647.0; }

static double ulp_err(double got, long double exact) {
  if (exact == 0) return got == 0 ? 0 : 1e300;
  const double e = (double)exact;
  const double ulp = std::nextafter(std::fabs(e), INFINITY) - std::fabs(e);
  return (double)std::fabs((long double)got - exact) / ulp;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) * 1000000L : 1L << 26;
  double max_log = 0, max_sqrt = 0, max_sin = 0, max_cos = 0;
  double g_log = 0, g_sin = 0, g_cos = 0;
  long mism[8] = {0}, total = 0;
  const float px = 0.707107f;
  auto check = [&](uint32_t k1, uint32_t k2) {
    const double u1 = div_rand_max(k1), u2 = div_rand_max(k2);
    const long double L = -2.0L * logl((long double)u1);
    const double a = ccv::chanmath::neg2_log(u1), ga = -2.0 * std::log(u1);
    max_log = std::fmax(max_log, ulp_err(a, L));
    g_log = std::fmax(g_log, ulp_err(ga, L));
    const double R = ccv::chanmath::sqrt_nonneg(a);
    max_sqrt = std::fmax(max_sqrt, ulp_err(R, sqrtl((long double)a)));
    double sn, cs;
    ccv::chanmath::sincos_2pi(u2, &sn, &cs);
    const long double T = 2.0L * 3.141592653589793238462643383279502884L * (long double)u2;
    max_sin = std::fmax(max_sin, std::fabs(sn - (double)sinl(T)));
    max_cos = std::fmax(max_cos, std::fabs(cs - (double)cosl(T)));
    const double Tt = 2.0 * M_PI * u2;
    g_sin = std::fmax(g_sin, std::fabs(std::sin(Tt) - (double)sinl(T)));
    g_cos = std::fmax(g_cos, std::fabs(std::cos(Tt) - (double)cosl(T)));
    const double gR = std::sqrt(ga), gs = std::sin(Tt), gc = std::cos(Tt);
    for (int db = 0; db < 8; ++db) {
      const double sc = std::sqrt(0.5) * std::pow(10.0, -2.0 * db / 20.0);
      const float x = (float)((double)px + sc * (R * cs)), y = (float)((double)px + sc * (R * sn));
      const float gx = (float)((double)px + sc * (gR * gc)), gy = (float)((double)px + sc * (gR * gs));
      mism[db] += (x != gx) + (y != gy);
    }
    total += 2;
  };
  // edges: the smallest and largest u1, u2 at 0, 1 and the quadrant boundaries
  const uint32_t M = 2147483647u;
  const uint32_t edges[] = {1u, 2u, 3u, M, M - 1, M / 2, M / 2 + 1, M / 4, M / 4 + 1, (uint32_t)(3.0 * M / 4),
                            0u, M / 8, M / 8 + 1, 1u << 30, (1u << 30) - 1};
  for (uint32_t k1 : edges)
    for (uint32_t k2 : edges)
      if (k1) check(k1, k2);
  for (long i = 0; i < n; ++i) {
    const uint64_t r = splitmix();
    uint32_t k1 = (uint32_t)(r >> 33), k2 = (uint32_t)(r & 0x7FFFFFFFu);
    if (k1 == 0) continue;   // gaussian.c:27 redraws u1 == 0
    check(k1, k2);
  }
  printf("draws %ld (+ %zu edge pairs)\n", n, sizeof(edges) / sizeof(edges[0]) * sizeof(edges) / sizeof(edges[0]));
  printf("max error, ulp of the exact value: -2 ln u  channel_math %.2f  glibc %.2f\n", max_log, g_log);
  printf("max error, ulp: sqrt  channel_math %.2f\n", max_sqrt);
  printf("max abs error sin / cos of 2 pi u: channel_math %.3g / %.3g  glibc(2 pi u rounded) %.3g / %.3g\n",
         max_sin, max_cos, g_sin, g_cos);
  for (int db = 0; db < 8; ++db)
    printf("Eb/N0 %2d dB: fp32 samples differing from glibc's: %ld of %ld (%.3g)\n", 2 * db, mism[db], total,
           (double)mism[db] / total);
  return 0;
}
