// channel_math.hpp -- the double-precision Box-Muller pieces of the on-device AWGN channel
// (channel_dev.hpp ChannelSource), written for the domain the channel draws from instead of calling
// the general ocml log / sqrt / sincos.
//
// The reference draws R = sqrt(-2 ln u1), T = 2 pi u2 with u1, u2 = k / (2^31 - 1) for 31-bit k
// (common/gaussian.c:23-33) and adds scaling * R * {cos, sin} T to an fp32 point in double, rounding
// the sum to fp32 (the product's host producer csrc/sim.cpp:150-170 does the same with glibc). The
// general ocml routines carry what this domain never needs: log's double-double tail (~75 VALU per
// call), sqrt's denormal scaling and second correction (~17), sincos's Payne-Hanek branch (~55 on
// the taken path). Here:
//   * neg2_log(u), u in [2^-31, 1]: u = 2^e m, m in [sqrt(1/2), sqrt(2)), ln m = 2 atanh(s),
//     s = (m - 1) / (m + 1), |s| <= 0.1716, the atanh series to s^21 (truncation < 3e-17 relative);
//   * sqrt_nonneg(x): the hardware reciprocal square root and one Goldschmidt correction pair;
//   * sincos_2pi(u, &s, &c), u in [0, 1]: quadrant q = rint(4u) (exact), t = u - q/4 (exact),
//     r = 2 pi t with a two-part 2 pi, |r| <= pi/4, the Taylor series to r^15 / r^16.
// Each result is within a few ulp of the correctly rounded value; the channel rounds the noisy
// sample to fp32 (2^29 times coarser), so the fp32 frames equal glibc's except where the double
// sum lands within those few ulp of an fp32 rounding boundary (tools/chanmath_check.cpp measures the
// match rate over 2^28 draws on the host with a reduced-precision rcp / rsq, profiles/
// r04_chanmath_check.txt; the device tests hold it to >= 99.9 %, test_device_channel_awgn).
//
// The includer defines CCV_HD (function qualifiers), ccv_rcp_approx / ccv_rsq_approx (device:
// the v_rcp_f64 / v_rsq_f64 hardware approximations; the host checker: emulations with the low 28
// mantissa bits cleared, so the Newton / Goldschmidt steps are exercised as on the device) and
// ccv_fma_const (a * b + c, c a constant: the device forces the three-address FMA).
#pragma once
#include <cstdint>
#include <cstring>

namespace ccv {
namespace chanmath {

CCV_HD inline double bits_to_double(uint64_t b) {
  double d;
  std::memcpy(&d, &b, sizeof d);
  return d;
}
CCV_HD inline uint64_t double_to_bits(double d) {
  uint64_t b;
  std::memcpy(&b, &d, sizeof b);
  return b;
}

// -2 ln(u) for u in [2^-31, 1] (normal doubles; u = 1 gives exactly 0).
CCV_HD inline double neg2_log(double u) {
  const uint64_t b = double_to_bits(u);
  const uint32_t hi = (uint32_t)(b >> 32);
  // mantissa field >= that of sqrt(2) (0x3FF6A09E...) -> m in [sqrt(1/2), 1) with e + 1
  const uint32_t up = (hi & 0x000FFFFFu) >= 0x0006A09Eu ? 1u : 0u;
  const int e = (int)(hi >> 20) - 1023 + (int)up;
  const double m = bits_to_double((b & 0x000FFFFFFFFFFFFFull) | ((uint64_t)(0x3FF - up) << 52));
  const double f = m - 1.0;        // exact (Sterbenz)
  const double d = m + 1.0;
  // s = f / d: approximate reciprocal, two Newton steps, one residual correction
  double r = ccv_rcp_approx(d);
  r = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
  r = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
  double s = f * r;
  s = __builtin_fma(__builtin_fma(-d, s, f), r, s);
  const double z = s * s;
  // 2 atanh(s) = 2s + s z (2/3 + 2/5 z + ... + 2/21 z^9)
  double p = 2.0 / 21.0;
  p = ccv_fma_const(p, z, 2.0 / 19.0);
  p = ccv_fma_const(p, z, 2.0 / 17.0);
  p = ccv_fma_const(p, z, 2.0 / 15.0);
  p = ccv_fma_const(p, z, 2.0 / 13.0);
  p = ccv_fma_const(p, z, 2.0 / 11.0);
  p = ccv_fma_const(p, z, 2.0 / 9.0);
  p = ccv_fma_const(p, z, 2.0 / 7.0);
  p = ccv_fma_const(p, z, 2.0 / 5.0);
  p = ccv_fma_const(p, z, 2.0 / 3.0);
  const double lnm = __builtin_fma(s * z, p, 2.0 * s);
  // ln 2 split so that e * LN2_HI is exact for |e| < 2^11
  constexpr double LN2_HI = 6.93147180369123816490e-01;   // 0x3FE62E42FEE00000
  constexpr double LN2_LO = 1.90821492927058770002e-10;
  const double ed = (double)e;
  return -2.0 * __builtin_fma(ed, LN2_HI, __builtin_fma(ed, LN2_LO, lnm));
}

// sqrt(x) for x >= 0 (x = 0 gives 0).
CCV_HD inline double sqrt_nonneg(double x) {
  const double r = ccv_rsq_approx(x);
  double y = x * r, h = 0.5 * r;
  const double e = __builtin_fma(-y, h, 0.5);
  y = __builtin_fma(y, e, y);
  h = __builtin_fma(h, e, h);
  const double dd = __builtin_fma(-y, y, x);
  y = __builtin_fma(dd, h, y);
  return x > 0.0 ? y : 0.0;
}

// sin and cos of 2 pi u for u in [0, 1].
CCV_HD inline void sincos_2pi(double u, double* sn, double* cs) {
  const double q = __builtin_rint(4.0 * u);        // 0 .. 4, 4u exact
  const double t = __builtin_fma(q, -0.25, u);    // exact: |t| <= 1/8
  constexpr double TWO_PI_HI = 6.28318530717958623200e+00;
  constexpr double TWO_PI_LO = 2.44929359829470635445e-16;
  const double r = __builtin_fma(t, TWO_PI_HI, t * TWO_PI_LO);
  const double z = r * r;
  // sin r = r + r z S(z), S to the r^15 term; cos r = 1 + z C(z), C to the r^16 term
  double ps = -1.0 / 1307674368000.0;
  ps = ccv_fma_const(ps, z, 1.0 / 6227020800.0);
  ps = ccv_fma_const(ps, z, -1.0 / 39916800.0);
  ps = ccv_fma_const(ps, z, 1.0 / 362880.0);
  ps = ccv_fma_const(ps, z, -1.0 / 5040.0);
  ps = ccv_fma_const(ps, z, 1.0 / 120.0);
  ps = ccv_fma_const(ps, z, -1.0 / 6.0);
  const double sr = __builtin_fma(r * z, ps, r);
  double pc = 1.0 / 20922789888000.0;
  pc = ccv_fma_const(pc, z, -1.0 / 87178291200.0);
  pc = ccv_fma_const(pc, z, 1.0 / 479001600.0);
  pc = ccv_fma_const(pc, z, -1.0 / 3628800.0);
  pc = ccv_fma_const(pc, z, 1.0 / 40320.0);
  pc = ccv_fma_const(pc, z, -1.0 / 720.0);
  pc = ccv_fma_const(pc, z, 1.0 / 24.0);
  pc = ccv_fma_const(pc, z, -0.5);
  const double cr = __builtin_fma(z, pc, 1.0);
  // 2 pi u = q pi/2 + r
  const int qi = (int)q & 3;
  const double a = (qi & 1) ? cr : sr;    // |sin|
  const double c = (qi & 1) ? sr : cr;    // |cos|
  *sn = (qi & 2) ? -a : a;
  *cs = ((qi + 1) & 2) ? -c : c;
}

}  // namespace chanmath
}  // namespace ccv
