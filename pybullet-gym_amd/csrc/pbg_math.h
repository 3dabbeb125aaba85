// Small fixed-size vector / matrix helpers and Philox4x32-10 for the step kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PBG_DEV __device__ __forceinline__

#include <type_traits>
#include <utility>

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

struct f3 {
  float x, y, z;
};
PBG_DEV f3 mk3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
PBG_DEV f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
PBG_DEV f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
PBG_DEV f3 operator-(f3 a) { return mk3(-a.x, -a.y, -a.z); }
PBG_DEV f3 operator*(float s, f3 a) { return mk3(s * a.x, s * a.y, s * a.z); }
PBG_DEV f3& operator+=(f3& a, f3 b) { a.x += b.x; a.y += b.y; a.z += b.z; return a; }
PBG_DEV float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PBG_DEV f3 cross3(f3 a, f3 b) { return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
// Physics-side fast reciprocal / sqrt (v_rcp_f32 / v_sqrt_f32 / v_rsq_f32, ~1 ulp); the
// numpy-exact pack keeps IEEE division and sqrt.
PBG_DEV float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
PBG_DEV float fast_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
PBG_DEV float fast_rsq(float x) { return __builtin_amdgcn_rsqf(x); }
PBG_DEV float norm3(f3 a) { return fast_sqrt(dot3(a, a)); }
// clamp(x, lo, hi) for lo <= hi in one v_med3_f32 (fminf(fmaxf()) costs two instructions
// plus the IEEE canonicalisations of its operands); same result for non-NaN x
PBG_DEV float clampf(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }


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

// row-major 3x3
struct m3 {
  float m[9];
};
PBG_DEV f3 mul(const m3& A, f3 v) {
  return mk3(A.m[0] * v.x + A.m[1] * v.y + A.m[2] * v.z, A.m[3] * v.x + A.m[4] * v.y + A.m[5] * v.z,
             A.m[6] * v.x + A.m[7] * v.y + A.m[8] * v.z);
}
PBG_DEV m3 mul(const m3& A, const m3& B) {
  m3 C;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
      C.m[3 * i + j] = A.m[3 * i] * B.m[j] + A.m[3 * i + 1] * B.m[3 + j] + A.m[3 * i + 2] * B.m[6 + j];
  return C;
}
PBG_DEV m3 quat_to_m3(float x, float y, float z, float w) {
  m3 R;
  R.m[0] = 1 - 2 * (y * y + z * z); R.m[1] = 2 * (x * y - w * z); R.m[2] = 2 * (x * z + w * y);
  R.m[3] = 2 * (x * y + w * z); R.m[4] = 1 - 2 * (x * x + z * z); R.m[5] = 2 * (y * z - w * x);
  R.m[6] = 2 * (x * z - w * y); R.m[7] = 2 * (y * z + w * x); R.m[8] = 1 - 2 * (x * x + y * y);
  return R;
}
// rotation by angle about a unit axis given by compile-time constants
PBG_DEV m3 axis_angle_m3(float ax, float ay, float az, float ang) {
  float s, c;
  sincos_fast(ang, &s, &c);
  float t = 1 - c;
  m3 R;
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
PBG_DEV float kmul(float c, float x) {
  if (__builtin_constant_p(c)) return c == 0.f ? -0.f : (c == 1.f ? x : (c == -1.f ? -x : c * x));
  return c * x;
}
// A * c for a constant vector c
PBG_DEV f3 mulc(const m3& A, float cx, float cy, float cz) {
  return mk3(kmul(cx, A.m[0]) + kmul(cy, A.m[1]) + kmul(cz, A.m[2]), kmul(cx, A.m[3]) + kmul(cy, A.m[4]) + kmul(cz, A.m[5]),
             kmul(cx, A.m[6]) + kmul(cy, A.m[7]) + kmul(cz, A.m[8]));
}
PBG_DEV f3 mulc(const m3& A, f3 c) { return mulc(A, c.x, c.y, c.z); }
// A * C for a constant matrix C (row-major)
PBG_DEV m3 mulc(const m3& A, const m3& C) {
  m3 O;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
      O.m[3 * i + j] = kmul(C.m[j], A.m[3 * i]) + kmul(C.m[3 + j], A.m[3 * i + 1]) + kmul(C.m[6 + j], A.m[3 * i + 2]);
  return O;
}
// constant quaternion (x,y,z,w) -> matrix, folded at compile time
PBG_DEV m3 quat_to_m3c(double x, double y, double z, double w) {
  m3 R;
  R.m[0] = (float)(1 - 2 * (y * y + z * z)); R.m[1] = (float)(2 * (x * y - w * z)); R.m[2] = (float)(2 * (x * z + w * y));
  R.m[3] = (float)(2 * (x * y + w * z)); R.m[4] = (float)(1 - 2 * (x * x + z * z)); R.m[5] = (float)(2 * (y * z - w * x));
  R.m[6] = (float)(2 * (x * z - w * y)); R.m[7] = (float)(2 * (y * z + w * x)); R.m[8] = (float)(1 - 2 * (x * x + y * y));
  return R;
}
// rotation about a constant unit axis
PBG_DEV m3 axis_angle_m3c(float ax, float ay, float az, float ang) {
  float s, c;
  sincos_fast(ang, &s, &c);
  const float t = 1 - c;
  m3 R;
  R.m[0] = kmul(ax * ax, t) + c;       R.m[1] = kmul(ax * ay, t) - kmul(az, s); R.m[2] = kmul(ax * az, t) + kmul(ay, s);
  R.m[3] = kmul(ax * ay, t) + kmul(az, s); R.m[4] = kmul(ay * ay, t) + c;       R.m[5] = kmul(ay * az, t) - kmul(ax, s);
  R.m[6] = kmul(ax * az, t) - kmul(ay, s); R.m[7] = kmul(ay * az, t) + kmul(ax, s); R.m[8] = kmul(az * az, t) + c;
  return R;
}

// symmetric 3x3 stored (xx, yy, zz, xy, xz, yz)
struct s6 {
  float a[6];
};
PBG_DEV f3 mul(const s6& S, f3 v) {
  return mk3(S.a[0] * v.x + S.a[3] * v.y + S.a[4] * v.z, S.a[3] * v.x + S.a[1] * v.y + S.a[5] * v.z,
             S.a[4] * v.x + S.a[5] * v.y + S.a[2] * v.z);
}
// R I R^T for body-frame inertia I6 = (xx, yy, zz, xy, xz, yz)
PBG_DEV s6 rotate_inertia(const m3& R, const float* I6) {
  const float I[9] = {I6[0], I6[3], I6[4], I6[3], I6[1], I6[5], I6[4], I6[5], I6[2]};
  float RI[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
      RI[3 * i + j] = kmul(I[j], R.m[3 * i]) + kmul(I[3 + j], R.m[3 * i + 1]) + kmul(I[6 + j], R.m[3 * i + 2]);
  s6 W;
  W.a[0] = RI[0] * R.m[0] + RI[1] * R.m[1] + RI[2] * R.m[2];
  W.a[1] = RI[3] * R.m[3] + RI[4] * R.m[4] + RI[5] * R.m[5];
  W.a[2] = RI[6] * R.m[6] + RI[7] * R.m[7] + RI[8] * R.m[8];
  W.a[3] = RI[0] * R.m[3] + RI[1] * R.m[4] + RI[2] * R.m[5];
  W.a[4] = RI[0] * R.m[6] + RI[1] * R.m[7] + RI[2] * R.m[8];
  W.a[5] = RI[3] * R.m[6] + RI[4] * R.m[7] + RI[5] * R.m[8];
  return W;
}

PBG_DEV s6 rotate_inertia(const m3& R, const double* I6) {
  const float I[6] = {(float)I6[0], (float)I6[1], (float)I6[2], (float)I6[3], (float)I6[4], (float)I6[5]};
  return rotate_inertia(R, I);
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
