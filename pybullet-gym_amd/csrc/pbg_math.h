// Small fixed-size vector / matrix helpers and Philox4x32-10 for the step kernels.
//
// The physics types are templates over the scalar S: float for the float32 kernels, double for
// the reference-precision path (pybullet's btScalar is double, scene_bases.py:75-76 ->
// stepSimulation).  The float names (f3, m3, s6) are the S = float instances; every helper
// deduces S from its vector / matrix operands, and compile-time model constants enter through
// a non-deduced scalar (nd<S>), so a float kernel's code is what it was before the templates.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#ifdef PBG_DEV_CHECKS
#include <cassert>
#endif

#define PBG_DEV __device__ __forceinline__
#define PBG_SC64_FN __host__ __device__ __forceinline__

#include <type_traits>
#include <utility>

#include "pbg_sincos64.h"

// Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E).  Guarantees a
// constant induction variable where `#pragma unroll` may give up on big bodies.
template <int B, class F, int... I>
PBG_DEV void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, B + I>{}), ...);
}
template <int B, int E, class F>
PBG_DEV void static_for(F&& f) {
  if constexpr (E > B) static_for_impl<B>(f, std::make_integer_sequence<int, E - B>{});
}

// a scalar parameter that takes part in no deduction (converted to S)
template <class S>
struct nd_ {
  using type = S;
};
template <class S>
using nd = typename nd_<S>::type;

template <class S>
struct V3 {
  S x, y, z;
};
using f3 = V3<float>;
// mk3(x, y, z): a float vector; mk3<double>(x, y, z): a double one
template <class S = float>
PBG_DEV V3<S> mk3(nd<S> x, nd<S> y, nd<S> z) { V3<S> r; r.x = x; r.y = y; r.z = z; return r; }
template <class S>
PBG_DEV V3<S> operator+(V3<S> a, V3<S> b) { return mk3<S>(a.x + b.x, a.y + b.y, a.z + b.z); }
template <class S>
PBG_DEV V3<S> operator-(V3<S> a, V3<S> b) { return mk3<S>(a.x - b.x, a.y - b.y, a.z - b.z); }
template <class S>
PBG_DEV V3<S> operator-(V3<S> a) { return mk3<S>(-a.x, -a.y, -a.z); }
template <class S>
PBG_DEV V3<S> operator*(nd<S> s, V3<S> a) { return mk3<S>(s * a.x, s * a.y, s * a.z); }
template <class S>
PBG_DEV V3<S>& operator+=(V3<S>& a, V3<S> b) { a.x += b.x; a.y += b.y; a.z += b.z; return a; }
template <class S>
PBG_DEV S dot3(V3<S> a, V3<S> b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
template <class S>
PBG_DEV V3<S> cross3(V3<S> a, V3<S> b) {
  return mk3<S>(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// Physics-side fast reciprocal / sqrt (v_rcp_f32 / v_sqrt_f32 / v_rsq_f32, ~1 ulp); the
// numpy-exact pack keeps IEEE division and sqrt.  The double overloads: fast_sqrt is the IEEE
// (correctly rounded) sqrt, fast_rsq an IEEE division of it, and fast_rcp is NOT correctly rounded
// -- it is within 1 ulp of the IEEE quotient for finite, non-zero, non-overflowing-reciprocal
// arguments only (x = 0 gives NaN, not inf).  Every call site guards its argument; the checks build
// (-DPBG_DEV_CHECKS) asserts it.
PBG_DEV float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
PBG_DEV float fast_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
PBG_DEV float fast_rsq(float x) { return __builtin_amdgcn_rsqf(x); }
// float64 reciprocal: v_rcp_f64 refined by two Newton steps (within 1 ulp of the IEEE quotient for
// the finite non-zero arguments the physics passes; the IEEE division's scaling and fix-up cost
// twice the instructions)
PBG_DEV double fast_rcp(double x) {
#ifdef PBG_DEV_CHECKS
  assert(x != 0.0 && __builtin_isfinite(x));
#endif
  double r = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-x, r, 1.0);
  return __builtin_fma(r, e, r);
}
PBG_DEV double fast_sqrt(double x) { return __builtin_sqrt(x); }
PBG_DEV double fast_rsq(double x) { return 1.0 / __builtin_sqrt(x); }
template <class S>
PBG_DEV S norm3(V3<S> a) { return fast_sqrt(dot3(a, a)); }
// clamp(x, lo, hi) for lo <= hi in one v_med3_f32 (fminf(fmaxf()) costs two instructions
// plus the IEEE canonicalisations of its operands); same result for non-NaN x
template <class S>
PBG_DEV S clampf(S x, nd<S> lo, nd<S> hi) {
  if constexpr (std::is_same<S, float>::value) return __builtin_amdgcn_fmed3f(x, lo, hi);
  else return __builtin_fmin(__builtin_fmax(x, lo), hi);
}


// sin/cos for the moderate arguments of the physics (joint angles, exp-map half angles):
// 3-part Cody-Waite reduction by pi/2 + minimax polynomials on [-pi/4, pi/4], a few ulp
// for |x| < 1e5.  Branch-free and short: the library sincosf carries a Payne-Hanek
// large-argument path that, executed as selects, costs ~50 instructions per call.
PBG_DEV void sincos_fast(float x, float* sp, float* cp) {
  const float k = __builtin_rintf(x * 0.636619772367581343f);
  float r = __builtin_fmaf(-k, 1.5703125f, x);
  r = __builtin_fmaf(-k, 4.837512969970703125e-4f, r);
  r = __builtin_fmaf(-k, 7.54978995489188216e-8f, r);
  const float r2 = r * r;
  const float sr = __builtin_fmaf(r * r2, __builtin_fmaf(r2, __builtin_fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f), -1.6666654611e-1f), r);
  const float cr = __builtin_fmaf(r2 * r2, __builtin_fmaf(r2, __builtin_fmaf(r2, 2.443315711809948e-5f, -1.388731625493765e-3f), 4.166664568298827e-2f),
                                  __builtin_fmaf(-0.5f, r2, 1.0f));
  const int q = (int)k;
  const float s0 = (q & 1) ? cr : sr, c0 = (q & 1) ? sr : cr;
  *sp = (q & 2) ? -s0 : s0;
  *cp = ((q + 1) & 2) ? -c0 : c0;
}
// float64: Cody-Waite reduction + the msun minimax kernels (pbg_sincos64.h): within 0.8 ulp for
// |x| <= 1e5, 1e-15 absolute to 1e6 (tests/test_sincos64.py), ~45 instructions and no branch, where the
// device library's sincos takes ~150 with its Payne-Hanek path behind a branch (the physics' joint
// angles and half-angle increments never need it; NaN and inf give NaN, as the library does)
PBG_DEV void sincos_fast(double x, double* sp, double* cp) {
#ifdef PBG_SC64_LIB  // diagnostic builds: the device library's sincos
  sincos(x, sp, cp);
#else
  pbg::sincos_reduced64(x, sp, cp);
#endif
}

// row-major 3x3
template <class S>
struct M3 {
  S m[9];
};
using m3 = M3<float>;
template <class S>
PBG_DEV V3<S> mul(const M3<S>& A, V3<S> v) {
  return mk3<S>(A.m[0] * v.x + A.m[1] * v.y + A.m[2] * v.z, A.m[3] * v.x + A.m[4] * v.y + A.m[5] * v.z,
                A.m[6] * v.x + A.m[7] * v.y + A.m[8] * v.z);
}
template <class S>
PBG_DEV M3<S> mul(const M3<S>& A, const M3<S>& B) {
  M3<S> C;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
      C.m[3 * i + j] = A.m[3 * i] * B.m[j] + A.m[3 * i + 1] * B.m[3 + j] + A.m[3 * i + 2] * B.m[6 + j];
  return C;
}
template <class S>
PBG_DEV M3<S> quat_to_m3(S x, S y, S z, S w) {
  M3<S> R;
  R.m[0] = 1 - 2 * (y * y + z * z); R.m[1] = 2 * (x * y - w * z); R.m[2] = 2 * (x * z + w * y);
  R.m[3] = 2 * (x * y + w * z); R.m[4] = 1 - 2 * (x * x + z * z); R.m[5] = 2 * (y * z - w * x);
  R.m[6] = 2 * (x * z - w * y); R.m[7] = 2 * (y * z + w * x); R.m[8] = 1 - 2 * (x * x + y * y);
  return R;
}
// rotation by angle about a unit axis given by compile-time constants
template <class S>
PBG_DEV M3<S> axis_angle_m3(nd<S> ax, nd<S> ay, nd<S> az, S ang) {
  S s, c;
  sincos_fast(ang, &s, &c);
  S t = 1 - c;
  M3<S> R;
  R.m[0] = t * ax * ax + c;      R.m[1] = t * ax * ay - s * az; R.m[2] = t * ax * az + s * ay;
  R.m[3] = t * ax * ay + s * az; R.m[4] = t * ay * ay + c;      R.m[5] = t * ay * az - s * ax;
  R.m[6] = t * ax * az - s * ay; R.m[7] = t * ay * az + s * ax; R.m[8] = t * az * az + c;
  return R;
}

// ---- products with compile-time model constants.  After inlining/unrolling the
// constant c is known, so a 0 / +-1 factor costs nothing: kmul returns -0 for c == 0 and
// x + (-0) == x exactly, so whole terms fold away (no fast-math needed).
// Only a compile-time c is inspected (__builtin_constant_p resolves after inlining); a
// run-time c is a plain product (no selects).
template <class S>
PBG_DEV S kmul(nd<S> c, S x) {
  if (__builtin_constant_p(c)) return c == S(0) ? -S(0) : (c == S(1) ? x : (c == S(-1) ? -x : c * x));
  return c * x;
}
// A * c for a constant vector c
template <class S>
PBG_DEV V3<S> mulc(const M3<S>& A, nd<S> cx, nd<S> cy, nd<S> cz) {
  return mk3<S>(kmul<S>(cx, A.m[0]) + kmul<S>(cy, A.m[1]) + kmul<S>(cz, A.m[2]),
                kmul<S>(cx, A.m[3]) + kmul<S>(cy, A.m[4]) + kmul<S>(cz, A.m[5]),
                kmul<S>(cx, A.m[6]) + kmul<S>(cy, A.m[7]) + kmul<S>(cz, A.m[8]));
}
template <class S>
PBG_DEV V3<S> mulc(const M3<S>& A, V3<S> c) { return mulc<S>(A, c.x, c.y, c.z); }
// A * C for a constant matrix C (row-major)
template <class S>
PBG_DEV M3<S> mulc(const M3<S>& A, const M3<S>& C) {
  M3<S> O;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
      O.m[3 * i + j] = kmul<S>(C.m[j], A.m[3 * i]) + kmul<S>(C.m[3 + j], A.m[3 * i + 1]) + kmul<S>(C.m[6 + j], A.m[3 * i + 2]);
  return O;
}
// constant quaternion (x,y,z,w) -> matrix, folded at compile time
template <class S = float>
PBG_DEV M3<S> quat_to_m3c(double x, double y, double z, double w) {
  M3<S> R;
  R.m[0] = (S)(1 - 2 * (y * y + z * z)); R.m[1] = (S)(2 * (x * y - w * z)); R.m[2] = (S)(2 * (x * z + w * y));
  R.m[3] = (S)(2 * (x * y + w * z)); R.m[4] = (S)(1 - 2 * (x * x + z * z)); R.m[5] = (S)(2 * (y * z - w * x));
  R.m[6] = (S)(2 * (x * z - w * y)); R.m[7] = (S)(2 * (y * z + w * x)); R.m[8] = (S)(1 - 2 * (x * x + y * y));
  return R;
}
// sin / cos of the physics: the kernels' own (sincos_fast), or the device library's when LIB (the
// float64 lane kernel, pbg_types.h F64L)
template <bool LIB = false, class S>
PBG_DEV void sincos_phys(S x, S* sp, S* cp) {
  if constexpr (LIB && sizeof(S) == 8) sincos(x, sp, cp);
  else sincos_fast(x, sp, cp);
}
// rotation about a constant unit axis
template <class S, bool LIB = false>
PBG_DEV M3<S> axis_angle_m3c(nd<S> ax, nd<S> ay, nd<S> az, S ang) {
  S s, c;
  sincos_phys<LIB>(ang, &s, &c);
  const S t = 1 - c;
  M3<S> R;
  R.m[0] = kmul<S>(ax * ax, t) + c;       R.m[1] = kmul<S>(ax * ay, t) - kmul<S>(az, s); R.m[2] = kmul<S>(ax * az, t) + kmul<S>(ay, s);
  R.m[3] = kmul<S>(ax * ay, t) + kmul<S>(az, s); R.m[4] = kmul<S>(ay * ay, t) + c;       R.m[5] = kmul<S>(ay * az, t) - kmul<S>(ax, s);
  R.m[6] = kmul<S>(ax * az, t) - kmul<S>(ay, s); R.m[7] = kmul<S>(ay * az, t) + kmul<S>(ax, s); R.m[8] = kmul<S>(az * az, t) + c;
  return R;
}

// symmetric 3x3 stored (xx, yy, zz, xy, xz, yz)
template <class S>
struct S6 {
  S a[6];
};
using s6 = S6<float>;
template <class S>
PBG_DEV V3<S> mul(const S6<S>& W, V3<S> v) {
  return mk3<S>(W.a[0] * v.x + W.a[3] * v.y + W.a[4] * v.z, W.a[3] * v.x + W.a[1] * v.y + W.a[5] * v.z,
                W.a[4] * v.x + W.a[5] * v.y + W.a[2] * v.z);
}
// R I R^T for body-frame inertia I6 = (xx, yy, zz, xy, xz, yz) (model constants: converted to S
// first)
template <class S, class IT>
PBG_DEV S6<S> rotate_inertia(const M3<S>& R, const IT* I6) {
  const S I[9] = {(S)I6[0], (S)I6[3], (S)I6[4], (S)I6[3], (S)I6[1], (S)I6[5], (S)I6[4], (S)I6[5], (S)I6[2]};
  S RI[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
      RI[3 * i + j] = kmul<S>(I[j], R.m[3 * i]) + kmul<S>(I[3 + j], R.m[3 * i + 1]) + kmul<S>(I[6 + j], R.m[3 * i + 2]);
  S6<S> W;
  W.a[0] = RI[0] * R.m[0] + RI[1] * R.m[1] + RI[2] * R.m[2];
  W.a[1] = RI[3] * R.m[3] + RI[4] * R.m[4] + RI[5] * R.m[5];
  W.a[2] = RI[6] * R.m[6] + RI[7] * R.m[7] + RI[8] * R.m[8];
  W.a[3] = RI[0] * R.m[3] + RI[1] * R.m[4] + RI[2] * R.m[5];
  W.a[4] = RI[0] * R.m[6] + RI[1] * R.m[7] + RI[2] * R.m[8];
  W.a[5] = RI[3] * R.m[6] + RI[4] * R.m[7] + RI[5] * R.m[8];
  return W;
}

// ---------------------------------------------------------------- Philox4x32-10
struct u4 {
  uint32_t x, y, z, w;
};
PBG_DEV u4 philox4x32_10(u4 ctr, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    uint32_t hi0 = __umulhi(0xD2511F53u, ctr.x), lo0 = 0xD2511F53u * ctr.x;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, ctr.z), lo1 = 0xCD9E8D57u * ctr.z;
    u4 n;
    n.x = hi1 ^ ctr.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ ctr.w ^ k1;
    n.w = lo0;
    ctr = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return ctr;
}
// uniform in [0, 1) with 24 random bits
PBG_DEV float u01(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }
