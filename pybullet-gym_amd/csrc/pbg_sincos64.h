// pbg_sincos64.h -- float64 sin/cos for the physics of the float64 kernels (joint rotations, the base's
// exponential map).  The device library's double sincos carries a Payne-Hanek large-argument path and
// costs ~150 VALU instructions per call (108 of them float64, half-rate); the physics' arguments are
// joint angles and half-angle increments.  Here: Cody-Waite reduction by pi/2 (fdlibm's pio2_1 +
// pio2_1t split, the reduced argument carried as a double-double), then the minimax kernels of FreeBSD
// msun's k_sin.c / k_cos.c on [-pi/4, pi/4] (the published coefficients), ~45 instructions, no branch.  tests/test_sincos64.py checks the host build of this header against long-double
// sinl / cosl: within 0.8 ulp for |x| <= 1e5 (the C library: 0.52) and 1e-15 absolute up to 1e6 (past
// 1e5 a result near a zero of sin loses relative accuracy: the neglected part of pi/2 times n); the
// float64 parity bound is 1e-9.  NaN / inf give NaN.
// Plain C++ (no HIP types), so the host test compiles it with g++.
#pragma once

#ifndef PBG_SC64_FN
#define PBG_SC64_FN inline
#endif

namespace pbg {
// r + y in [-pi/4, pi/4] (y: the reduction's tail, |y| <= ulp(r)): (sin, cos) of r + y
PBG_SC64_FN void sincos_kernel64(double r, double y, double* sp, double* cp) {
  const double z = r * r, w = z * z;
  // k_sin.c: S1..S6 (sin(r + y) = r + v S1 + ... with the tail's first-order terms)
  const double sr = 8.33333333332248946124e-03 + z * (-1.98412698298579493134e-04 + z * 2.75573137070700676789e-06) +
                    z * w * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10);
  const double v = z * r;
  *sp = r - ((z * (0.5 * y - v * sr) - y) - v * -1.66666666666666324348e-01);
  // k_cos.c: C1..C6, 1 - z/2 + z cr - r y with the rounding of 1 - z/2 recovered
  const double cr = z * (4.16666666666666019037e-02 + z * (-1.38888888888741095749e-03 + z * 2.48015872894767294178e-05)) +
                    w * w * (-2.75573143513906633035e-07 + z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11));
  const double hz = 0.5 * z, one_m = 1.0 - hz;
  *cp = one_m + (((1.0 - one_m) - hz) + (z * cr - r * y));
}
// x = n pi/2 + (r + y), r + y a double-double (fdlibm's
// __ieee754_rem_pio2 medium case with FMAs: n pio2_1 is exact, the product n pio2_1t and the
// subtraction are carried exactly by TwoProd / TwoSum), then the quadrant
PBG_SC64_FN void sincos_reduced64(double x, double* sp, double* cp) {
  const double n = __builtin_rint(x * 6.36619772367581382433e-01);  // 2 / pi
  const double r1 = __builtin_fma(-n, 1.57079632673412561417e+00, x);  // pio2_1: pi/2, first 33 bits
  const double p = n * 6.07710050650619224932e-11;                     // pio2_1t = pi/2 - pio2_1
  const double pe = __builtin_fma(n, 6.07710050650619224932e-11, -p);
  const double r = r1 - p, bb = r - r1;
  const double y = ((r1 - (r - bb)) - (p + bb)) - pe;
  double s, c;
  sincos_kernel64(r, y, &s, &c);
  const int q = (int)n & 3;
  const double s0 = (q & 1) ? c : s, c0 = (q & 1) ? s : c;
  *sp = (q & 2) ? -s0 : s0;
  *cp = ((q + 1) & 2) ? -c0 : c0;
}
}  // namespace pbg
