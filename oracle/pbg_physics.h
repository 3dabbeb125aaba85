// pbg_physics.h -- the oracle's restatement of Bullet's btMultiBody step (stepSimulation
// sub-step), templated on the scalar type T.  TEST INFRASTRUCTURE ONLY (included by
// pbg_oracle.cpp inside its anonymous namespace).
//
//   T = double         the oracle proper (the parity reference of every physics test)
//   T = float          the same algorithm in IEEE float32: how far an honest float32
//                      implementation lands from the float64 one on a given state (the
//                      conditioning probe of the GPU parity tests, tests/test_gpu.py)
//   T = Counted<float> counts every arithmetic operation: algorithmic FP32 flops per
//                      env-step (tools/count_flops.py)
//
// Every constant enters the arithmetic as T(...) so that no operation silently widens to
// double (Counted<float> has no mixed-type operators: a missed cast does not compile).
// [EXT] = Bullet semantics restated from its published algorithm.
#pragma once
#include <type_traits>

using std::cos;
using std::fabs;
using std::sin;
using std::sqrt;

template <class T> inline T tmin(T a, T b) { return b < a ? b : a; }
template <class T> inline T tmax(T a, T b) { return a < b ? b : a; }

// ------------------------------------------------------------------ small linear algebra
template <class T> struct V3T { T x, y, z; };
template <class T> inline V3T<T> v3(T x, T y, T z) { V3T<T> r = {x, y, z}; return r; }
template <class T> inline V3T<T> v3c(const double* p) { return v3(T(p[0]), T(p[1]), T(p[2])); }
template <class T> inline V3T<T> v3p(const T* p) { return v3(p[0], p[1], p[2]); }
template <class T> inline V3T<T> vzero() { return v3(T(0), T(0), T(0)); }
template <class T> inline V3T<T> operator+(V3T<T> a, V3T<T> b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
template <class T> inline V3T<T> operator-(V3T<T> a, V3T<T> b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
template <class T> inline V3T<T> operator*(T s, V3T<T> a) { return v3(s * a.x, s * a.y, s * a.z); }
template <class T> inline T dot(V3T<T> a, V3T<T> b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
template <class T> inline V3T<T> cross(V3T<T> a, V3T<T> b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
template <class T> inline T norm(V3T<T> a) { return sqrt(dot(a, a)); }

template <class T> struct M3T { T m[3][3]; };
template <class T> inline V3T<T> mul(const M3T<T>& A, V3T<T> v) {
  return v3(A.m[0][0] * v.x + A.m[0][1] * v.y + A.m[0][2] * v.z, A.m[1][0] * v.x + A.m[1][1] * v.y + A.m[1][2] * v.z,
            A.m[2][0] * v.x + A.m[2][1] * v.y + A.m[2][2] * v.z);
}
template <class T> inline M3T<T> mul(const M3T<T>& A, const M3T<T>& B) {
  M3T<T> C;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) C.m[i][j] = A.m[i][0] * B.m[0][j] + A.m[i][1] * B.m[1][j] + A.m[i][2] * B.m[2][j];
  return C;
}
template <class T> inline M3T<T> quat_to_m3(T x, T y, T z, T w) {  // q = (x, y, z, w)
  const T one(1), two(2);
  M3T<T> R;
  R.m[0][0] = one - two * (y * y + z * z); R.m[0][1] = two * (x * y - w * z); R.m[0][2] = two * (x * z + w * y);
  R.m[1][0] = two * (x * y + w * z); R.m[1][1] = one - two * (x * x + z * z); R.m[1][2] = two * (y * z - w * x);
  R.m[2][0] = two * (x * z - w * y); R.m[2][1] = two * (y * z + w * x); R.m[2][2] = one - two * (x * x + y * y);
  return R;
}
template <class T> inline M3T<T> quat_to_m3c(const double* q) { return quat_to_m3(T(q[0]), T(q[1]), T(q[2]), T(q[3])); }
template <class T> inline M3T<T> axis_angle_m3(V3T<T> a, T ang) {  // unit axis
  const T c = cos(ang), s = sin(ang), t = T(1) - c;
  M3T<T> R;
  R.m[0][0] = t * a.x * a.x + c;       R.m[0][1] = t * a.x * a.y - s * a.z; R.m[0][2] = t * a.x * a.z + s * a.y;
  R.m[1][0] = t * a.x * a.y + s * a.z; R.m[1][1] = t * a.y * a.y + c;       R.m[1][2] = t * a.y * a.z - s * a.x;
  R.m[2][0] = t * a.x * a.z - s * a.y; R.m[2][1] = t * a.y * a.z + s * a.x; R.m[2][2] = t * a.z * a.z + c;
  return R;
}
// world inertia R I R^T from the 6-vector (xx,yy,zz,xy,xz,yz)
template <class T> inline M3T<T> world_inertia(const M3T<T>& R, const double* I6) {
  M3T<T> I = {{{T(I6[0]), T(I6[3]), T(I6[4])}, {T(I6[3]), T(I6[1]), T(I6[5])}, {T(I6[4]), T(I6[5]), T(I6[2])}}};
  M3T<T> RI = mul(R, I), W;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) W.m[i][j] = RI.m[i][0] * R.m[j][0] + RI.m[i][1] * R.m[j][1] + RI.m[i][2] * R.m[j][2];
  return W;
}

// ------------------------------------------------------------------ kinematics
template <class T> struct KinT {
  M3T<T> R[MAXL + 1];             // index 0 = base, l+1 = link l
  V3T<T> x[MAXL + 1];             // frame origin (base: COM)
  V3T<T> c[MAXL + 1];             // COM world
  V3T<T> w[MAXL + 1], v[MAXL + 1];    // angular velocity, COM linear velocity
  V3T<T> al[MAXL + 1], ac[MAXL + 1];  // bias angular / COM linear acceleration
  V3T<T> ja[MAXD], jo[MAXD];          // per joint dof: world axis, world anchor
  M3T<T> Rc;                          // HumanoidFlagrunHarder's cube: orientation, COM
  V3T<T> xc;
};

// HumanoidFlagrunHarder: the attacking cube is a second free body (its state words follow the
// robot's, sim_params.h PBG_STATE_WORDS; its 6 velocity coordinates [v, w] follow the robot's
// in the generalized velocity).  Contact bodies: b >= 0 robot body, -1 floor, -2 cube.
inline int cube_word(const MV& m) { return PBG_BASE_WORDS + 2 * m.NJ; }
inline int n_total(const MV& m) { return m.NDOF + (m.harder ? 6 : 0); }
#define CUBE_BODY (-2)

// s: the env's state record in T (layout of sim_params.h)
template <class T> void forward_kinematics(const MV& m, const T* s, KinT<T>& k) {
  const T* q = s + PBG_BASE_WORDS;
  const T* qd = q + m.NJ;
  k.R[0] = quat_to_m3(s[3], s[4], s[5], s[6]);
  k.x[0] = v3p(s);
  k.c[0] = k.x[0];
  k.w[0] = m.floating ? v3p(s + 10) : vzero<T>();
  k.v[0] = m.floating ? v3p(s + 7) : vzero<T>();
  k.al[0] = vzero<T>();
  k.ac[0] = vzero<T>();
  if (m.harder) {
    const T* cs = s + cube_word(m);
    k.Rc = quat_to_m3(cs[3], cs[4], cs[5], cs[6]);
    k.xc = v3p(cs);
  }
  for (int l = 0; l < m.NL; l++) {
    int p = m.link_parent[l] + 1;
    M3T<T> Ro = quat_to_m3c<T>(m.off_quat[l]);
    M3T<T> R0 = mul(k.R[p], Ro);
    V3T<T> x0 = k.x[p] + mul(k.R[p], v3c<T>(m.off_pos[l]));
    V3T<T> axl = v3c<T>(m.axis[l]), anl = v3c<T>(m.anchor[l]);
    int jt = m.link_jtype[l], d = m.link_dof[l];
    M3T<T> R = R0;
    V3T<T> x = x0;
    if (jt == 0) {
      M3T<T> Rj = axis_angle_m3(axl, q[d]);
      R = mul(R0, Rj);
      x = x0 + mul(R0, anl - mul(Rj, anl));
    } else if (jt == 1) {
      x = x0 + mul(R0, q[d] * axl);
    }
    k.R[l + 1] = R;
    k.x[l + 1] = x;
    k.c[l + 1] = x + mul(R, v3c<T>(m.com[l]));
    V3T<T> cp = k.c[p], wp = k.w[p], vp = k.v[p], alp = k.al[p], acp = k.ac[p];
    V3T<T> c = k.c[l + 1];
    if (jt == 0) {
      V3T<T> a = mul(R0, axl), o = x0 + mul(R0, anl);
      k.ja[d] = a; k.jo[d] = o;
      V3T<T> ro = o - cp;
      V3T<T> vo = vp + cross(wp, ro);
      V3T<T> ao = acp + cross(alp, ro) + cross(wp, cross(wp, ro));
      V3T<T> w = wp + qd[d] * a;
      V3T<T> al = alp + qd[d] * cross(wp, a);
      V3T<T> rc = c - o;
      k.w[l + 1] = w; k.al[l + 1] = al;
      k.v[l + 1] = vo + cross(w, rc);
      k.ac[l + 1] = ao + cross(al, rc) + cross(w, cross(w, rc));
    } else if (jt == 1) {
      V3T<T> a = mul(R0, axl);
      k.ja[d] = a; k.jo[d] = x0;
      V3T<T> r = c - cp;
      k.w[l + 1] = wp; k.al[l + 1] = alp;
      k.v[l + 1] = vp + cross(wp, r) + qd[d] * a;
      k.ac[l + 1] = acp + cross(alp, r) + cross(wp, cross(wp, r)) + (T(2) * qd[d]) * cross(wp, a);
    } else {
      V3T<T> r = c - cp;
      k.w[l + 1] = wp; k.al[l + 1] = alp;
      k.v[l + 1] = vp + cross(wp, r);
      k.ac[l + 1] = acp + cross(alp, r) + cross(wp, cross(wp, r));
    }
  }
}

// generalized-velocity index of joint dof d
inline int gidx(const MV& m, int d) { return (m.floating ? 6 : 0) + d; }

// Jacobian rows (linear velocity of world point P, angular velocity) of body b (0 = base,
// l+1 = link l) w.r.t. the generalized velocity; written densely into Jv[3][NDOF], Jw[3][NDOF].
template <class T> void point_jacobian(const MV& m, const KinT<T>& k, int b, V3T<T> P, T Jv[3][MAXD], T Jw[3][MAXD]) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < m.NDOF; j++) Jv[i][j] = Jw[i][j] = T(0);
  if (m.floating) {
    V3T<T> r = P - k.x[0];
    for (int e = 0; e < 3; e++) {
      V3T<T> ax = v3(T(e == 0), T(e == 1), T(e == 2));
      Jv[e][e] = T(1);
      V3T<T> lin = cross(ax, r);
      Jv[0][3 + e] = lin.x; Jv[1][3 + e] = lin.y; Jv[2][3 + e] = lin.z;
      Jw[e][3 + e] = T(1);
    }
  }
  int l = b - 1;
  while (l >= 0) {
    int d = m.link_dof[l];
    if (d >= 0) {
      int g = gidx(m, d);
      V3T<T> a = k.ja[d];
      if (m.link_jtype[l] == 0) {
        V3T<T> lin = cross(a, P - k.jo[d]);
        Jv[0][g] = lin.x; Jv[1][g] = lin.y; Jv[2][g] = lin.z;
        Jw[0][g] = a.x; Jw[1][g] = a.y; Jw[2][g] = a.z;
      } else {
        Jv[0][g] = a.x; Jv[1][g] = a.y; Jv[2][g] = a.z;
      }
    }
    l = m.link_parent[l];
  }
}

// ------------------------------------------------------------------ dynamics
// M (NDOF x NDOF) and bias C (Coriolis/centrifugal/gyroscopic + gravity + body damping).
template <class T> void mass_and_bias(const MV& m, const KinT<T>& k, T M[MAXD][MAXD], T* C, const T* s = nullptr) {
  int n = m.NDOF;
  if (m.harder) {  // the cube's block: diag(m, m, m, I, I, I) (isotropic inertia), decoupled
    const int n6 = n_total(m);
    for (int i = n; i < n6; i++) {
      C[i] = T(0);
      for (int j = 0; j < n6; j++) M[i][j] = M[j][i] = T(0);
    }
  }
  for (int i = 0; i < n; i++) {
    C[i] = T(0);
    for (int j = 0; j < n; j++) M[i][j] = T(0);
  }
  const V3T<T> g = v3(T(0), T(0), T((g_flags & 16) ? 0.0 : -g_opt[OPT_GRAVITY]));
  const T kd_lin((g_flags & 4) ? 0.0 : PBG_LINEAR_DAMPING);
  const T kd_ang((g_flags & 4) ? 0.0 : PBG_ANGULAR_DAMPING);
  T Jv[3][MAXD], Jw[3][MAXD];
  int nb = m.NL + 1;
  for (int b = 0; b < nb; b++) {
    const T mass(b == 0 ? m.base_mass : m.mass[b - 1]);
    const double* I6 = b == 0 ? m.base_inertia : m.inertia[b - 1];
    if (b == 0 && !m.floating) continue;
    M3T<T> Iw = world_inertia(k.R[b], I6);
    point_jacobian(m, k, b, k.c[b], Jv, Jw);
    for (int i = 0; i < n; i++) {
      V3T<T> jvi = v3(Jv[0][i], Jv[1][i], Jv[2][i]);
      V3T<T> jwi = v3(Jw[0][i], Jw[1][i], Jw[2][i]);
      V3T<T> Ijwi = mul(Iw, jwi);
      for (int j = 0; j < n; j++) {
        V3T<T> jvj = v3(Jv[0][j], Jv[1][j], Jv[2][j]);
        V3T<T> jwj = v3(Jw[0][j], Jw[1][j], Jw[2][j]);
        M[i][j] = M[i][j] + (mass * dot(jvi, jvj) + dot(Ijwi, jwj));
      }
    }
    V3T<T> w = k.w[b], v = k.v[b];
    V3T<T> Iw_w = mul(Iw, w);
    V3T<T> f = mass * (k.ac[b] - g) + (mass * (kd_lin + kd_lin * norm(v))) * v;
    V3T<T> tq = mul(Iw, k.al[b]) + cross(w, Iw_w) + (kd_ang + kd_ang * norm(w)) * Iw_w;
    for (int i = 0; i < n; i++) {
      C[i] = C[i] + (Jv[0][i] * f.x + Jv[1][i] * f.y + Jv[2][i] * f.z + Jw[0][i] * tq.x + Jw[1][i] * tq.y + Jw[2][i] * tq.z);
    }
  }
  for (int d = 0; d < m.NJ; d++) M[gidx(m, d)][gidx(m, d)] = M[gidx(m, d)][gidx(m, d)] + T(m.armature[d]);
  if (m.harder && s) {
    // free-body bias as for the robot's base (ac = al = 0): f = m (-g) + m (k1 + k2 |v|) v,
    // tq = w x (I w) + (k1 + k2 |w|) I w, whose gyroscopic term vanishes for the isotropic cube
    const T* cs = s + cube_word(m);
    const T mc(PBG_CUBE_MASS), Ic(PBG_CUBE_INERTIA);
    const V3T<T> v = v3p(cs + 7), w = v3p(cs + 10);
    const V3T<T> f = mc * (vzero<T>() - g) + (mc * (kd_lin + kd_lin * norm(v))) * v;
    const V3T<T> tq = ((kd_ang + kd_ang * norm(w)) * Ic) * w;
    const int c0 = m.NDOF;
    for (int i = 0; i < 3; i++) { M[c0 + i][c0 + i] = mc; M[c0 + 3 + i][c0 + 3 + i] = Ic; }
    C[c0] = f.x; C[c0 + 1] = f.y; C[c0 + 2] = f.z; C[c0 + 3] = tq.x; C[c0 + 4] = tq.y; C[c0 + 5] = tq.z;
  }
}

// The kernels' formulation of the same M and C (pbg_step.hip dyn_mass, pbg_gang.hip
// gang_dyn_mass, pbg_team.hip): every body's inertia and wrench taken about one reference point
// O (the base COM, or the robot body's COM for a fixed base) and projected on the motion vectors
// (sw_i, sv_i) of the generalized coordinates about O,
//   M_ij += sw_i.(J sw_j + m r x sv_j) + sv_i.(m sv_j - m r x sw_j),  C_i += sw_i.(n + r x f) + sv_i.f
// with J = Iw + m (r.r 1 - r r^T), r = c_b - O, over the bodies both coordinates move.  Equal to
// mass_and_bias in exact arithmetic; in float32 its parallel-axis terms (m r^2 ~ 1 kg m^2 for an
// arm tip a metre from O) cancel down to the tip's ~1e-3 kg m^2 entries, which point Jacobians at
// each COM do not.  The float32 instantiations (precision 32 / 33: the conditioning and
// outlier-explanation envelopes of the parity tests) use it, so that they carry the kernels'
// rounding; the float64 oracle keeps mass_and_bias.
template <class T> void mass_and_bias_ref(const MV& m, const KinT<T>& k, T M[MAXD][MAXD], T* C, const T* s = nullptr) {
  const int n = m.NDOF;
  if (m.harder) {
    mass_and_bias(m, k, M, C, s);  // the cube block (decoupled); the robot's entries rebuilt below
  }
  for (int i = 0; i < n; i++) {
    C[i] = T(0);
    for (int j = 0; j < n; j++) M[i][j] = T(0);
  }
  const V3T<T> g = v3(T(0), T(0), T((g_flags & 16) ? 0.0 : -g_opt[OPT_GRAVITY]));
  const T kd_lin((g_flags & 4) ? 0.0 : PBG_LINEAR_DAMPING);
  const T kd_ang((g_flags & 4) ? 0.0 : PBG_ANGULAR_DAMPING);
  const int rb = m.floating ? 0 : m.robot_body + 1;
  const V3T<T> O = k.c[rb];
  // motion vectors about O of every generalized coordinate
  V3T<T> sw[MAXD], sv[MAXD];
  if (m.floating) {
    const V3T<T> ob = O - k.x[0];
    for (int e = 0; e < 3; e++) {
      const V3T<T> ax = v3(T(e == 0), T(e == 1), T(e == 2));
      sw[e] = vzero<T>(); sv[e] = ax;
      sw[3 + e] = ax; sv[3 + e] = cross(ax, ob);
    }
  }
  for (int l = 0; l < m.NL; l++) {
    const int d = m.link_dof[l];
    if (d < 0) continue;
    const int gi = gidx(m, d);
    if (m.link_jtype[l] == 0) { sw[gi] = k.ja[d]; sv[gi] = cross(k.ja[d], O - k.jo[d]); }
    else { sw[gi] = vzero<T>(); sv[gi] = k.ja[d]; }
  }
  for (int b = 0; b < m.NL + 1; b++) {
    if (b == 0 && !m.floating) continue;
    const double mb = b == 0 ? m.base_mass : m.mass[b - 1];
    if (!(mb > 0.0)) continue;
    const T mass(mb);
    const M3T<T> Iw = world_inertia(k.R[b], b == 0 ? m.base_inertia : m.inertia[b - 1]);
    const V3T<T> r = k.c[b] - O;
    const T rr = dot(r, r);
    M3T<T> J = Iw;
    const T rv[3] = {r.x, r.y, r.z};
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) J.m[i][j] = J.m[i][j] + mass * ((i == j ? rr : T(0)) - rv[i] * rv[j]);
    const V3T<T> w = k.w[b], v = k.v[b];
    const V3T<T> Iw_w = mul(Iw, w);
    const V3T<T> f = mass * (k.ac[b] - g) + (mass * (kd_lin + kd_lin * norm(v))) * v;
    const V3T<T> tq = mul(Iw, k.al[b]) + cross(w, Iw_w) + (kd_ang + kd_ang * norm(w)) * Iw_w;
    const V3T<T> pr = mass * r, Nn = tq + cross(r, f);
    // the coordinates that move body b: the base's and the joints on its chain
    int S[MAXD], ns = 0;
    if (m.floating)
      for (int e = 0; e < 6; e++) S[ns++] = e;
    for (int l = b - 1; l >= 0; l = m.link_parent[l])
      if (m.link_dof[l] >= 0) S[ns++] = gidx(m, m.link_dof[l]);
    for (int a = 0; a < ns; a++) {
      const int i = S[a];
      C[i] = C[i] + (dot(sw[i], Nn) + dot(sv[i], f));
      for (int c = 0; c < ns; c++) {
        const int j = S[c];
        const V3T<T> Jw_ = mul(J, sw[j]) + cross(pr, sv[j]);
        const V3T<T> Fv = mass * sv[j] - cross(pr, sw[j]);
        M[i][j] = M[i][j] + (dot(sw[i], Jw_) + dot(sv[i], Fv));
      }
    }
  }
  for (int d = 0; d < m.NJ; d++) M[gidx(m, d)][gidx(m, d)] = M[gidx(m, d)][gidx(m, d)] + T(m.armature[d]);
}

// in-place Cholesky M = L L^T (lower)
template <class T> void cholesky(int n, T A[MAXD][MAXD]) {
  for (int j = 0; j < n; j++) {
    T s = A[j][j];
    for (int k = 0; k < j; k++) s = s - A[j][k] * A[j][k];
    T ljj = sqrt(s);
    A[j][j] = ljj;
    for (int i = j + 1; i < n; i++) {
      T t = A[i][j];
      for (int k = 0; k < j; k++) t = t - A[i][k] * A[j][k];
      A[i][j] = t / ljj;
    }
  }
}
template <class T> void chol_solve(int n, const T L[MAXD][MAXD], const T* b, T* x) {
  T y[MAXD];
  for (int i = 0; i < n; i++) {
    T t = b[i];
    for (int k = 0; k < i; k++) t = t - L[i][k] * y[k];
    y[i] = t / L[i][i];
  }
  for (int i = n - 1; i >= 0; i--) {
    T t = y[i];
    for (int k = i + 1; k < n; k++) t = t - L[k][i] * x[k];
    x[i] = t / L[i][i];
  }
}

// ------------------------------------------------------------------ contacts + PGS
template <class T> struct RowT {
  T J[MAXD], W[MAXD];
  T meff, target, lo, hi, lambda, mu;
  int normal;  // friction rows: index of their normal row; else -1
};

template <class T> inline void plane_space(V3T<T> n, V3T<T>& p, V3T<T>& q) {  // btPlaneSpace1
  if (fabs(n.z) > T(0.7071067811865476)) {
    T a = n.y * n.y + n.z * n.z, k = T(1) / sqrt(a);
    p = v3(T(0), T(0) - n.z * k, n.y * k);
    q = v3(a * k, T(0) - n.x * p.z, n.x * p.y);
  } else {
    T a = n.x * n.x + n.y * n.y, k = T(1) / sqrt(a);
    p = v3(T(0) - n.y * k, n.x * k, T(0));
    q = v3(T(0) - n.z * p.y, n.z * p.x, a * k);
  }
}

// closest points between segments p0-p1 and q0-q1
template <class T> void segment_closest(V3T<T> p0, V3T<T> p1, V3T<T> q0, V3T<T> q1, V3T<T>& cp, V3T<T>& cq) {
  V3T<T> d1 = p1 - p0, d2 = q1 - q0, r = p0 - q0;
  T a = dot(d1, d1), e = dot(d2, d2), f = dot(d2, r);
  T s, t;
  const T eps(1e-12), zero(0), one(1);
  if (a <= eps && e <= eps) { s = t = zero; }
  else if (a <= eps) { s = zero; t = tmin(tmax(f / e, zero), one); }
  else {
    T c = dot(d1, r);
    if (e <= eps) { t = zero; s = tmin(tmax((zero - c) / a, zero), one); }
    else {
      T b = dot(d1, d2), den = a * e - b * b;
      s = den > eps ? tmin(tmax((b * f - c * e) / den, zero), one) : zero;
      t = (b * s + f) / e;
      if (t < zero) { t = zero; s = tmin(tmax((zero - c) / a, zero), one); }
      else if (t > one) { t = one; s = tmin(tmax((b - c) / a, zero), one); }
    }
  }
  cp = p0 + s * d1;
  cq = q0 + t * d2;
}

template <class T> struct ContactT {
  int cand;            // collision candidate: floor slot s, or NS + self pair p
  int body_a, body_b;  // body_b = -1: floor
  V3T<T> pa, pb, n;    // points on A / B, normal pointing from B into A
  T dist, mu;
};

// HumanoidFlagrunHarder's cube (a box of half extent h) against the floor and the robot's
// geoms.  Candidates after the floor slots and self pairs: NS + NPAIR + k for cube corner k
// (k bit 0/1/2: -/+ h along the cube's x/y/z), NS + NPAIR + 8 + g for robot geom g
// (cgeom_*).  [EXT] Bullet's box-plane algorithm keeps the deepest vertices of the box in its
// manifold (up to 4 with the multipoint iterations pybullet enables) -- here every corner
// within the contact threshold is a point, normal +z.  Box-capsule: Bullet's GJK/EPA returns
// the closest (or deepest) points of the two convex shapes; here the same points are found
// on the capsule's segment by minimising the box's signed distance function along it (convex
// in the segment parameter: golden-section search, CUBE_GS_ITERS fixed rounds, then the box
// point and normal of the minimiser).  Normal from the cube (B) into the robot link (A).
#define CUBE_GS_ITERS 24
template <class T> inline T box_sd(V3T<T> p, T h) {  // signed distance of a box-local point
  const T qx = fabs(p.x) - h, qy = fabs(p.y) - h, qz = fabs(p.z) - h;
  const T ox = tmax(qx, T(0)), oy = tmax(qy, T(0)), oz = tmax(qz, T(0));
  return sqrt(ox * ox + oy * oy + oz * oz) + tmin(tmax(qx, tmax(qy, qz)), T(0));
}
template <class T>
int detect_cube_contacts(const MV& m, const KinT<T>& k, ContactT<T>* out, int nc, int sub, uint32_t* sig) {
  const T thr(g_opt[OPT_CONTACT_THR]), h(PBG_CUBE_HALF);
  const M3T<T>& Rc = k.Rc;
  const V3T<T> xc = k.xc;
  for (int c = 0; c < 8; c++) {  // corners vs floor
    const V3T<T> lc = v3((c & 1) ? h : T(0) - h, (c & 2) ? h : T(0) - h, (c & 4) ? h : T(0) - h);
    const V3T<T> p = xc + mul(Rc, lc);
    if (!(p.z < thr)) continue;
    if (sig) *sig += pbg_contact_hash((uint32_t)sub, (uint32_t)(m.NS + m.NPAIR + c));
    ContactT<T>& ct = out[nc++];
    ct.cand = m.NS + m.NPAIR + c;
    ct.body_a = CUBE_BODY; ct.body_b = -1;
    ct.pa = p; ct.pb = v3(p.x, p.y, T(0));
    ct.n = v3(T(0), T(0), T(1)); ct.dist = p.z; ct.mu = T(m.cube_floor_mu);
  }
  // R^T: robot geom endpoints into the cube frame
  M3T<T> Rt;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) Rt.m[i][j] = Rc.m[j][i];
  const T bound(0.5 * 1.7320508075688772 * 2.0 * PBG_CUBE_HALF);  // cube circumradius
  for (int g = 0; g < m.NCG; g++) {
    const int b = m.cg_link[g] + 1;
    const V3T<T> e0 = k.x[b] + mul(k.R[b], v3c<T>(m.cg_p0[g])), e1 = k.x[b] + mul(k.R[b], v3c<T>(m.cg_p1[g]));
    const T r(m.cg_r[g]);
    // broad phase: the segment's distance to the cube centre vs circumradius + radius + threshold
    const V3T<T> p0 = mul(Rt, e0 - xc), p1 = mul(Rt, e1 - xc), d = p1 - p0;
    const T dd = dot(d, d);
    T t0 = dd > T(1e-12) ? tmin(tmax((T(0) - dot(p0, d)) / dd, T(0)), T(1)) : T(0);
    const V3T<T> pc = p0 + t0 * d;
    if (!(norm(pc) < bound + r + thr)) continue;
    T t = T(0);
    if (dd > T(1e-12)) {  // golden-section minimisation of box_sd(p0 + t d) over [0, 1]
      const T phi(0.6180339887498949);
      T a(0), bb(1);
      T x1 = bb - phi * (bb - a), x2 = a + phi * (bb - a);
      T f1 = box_sd(p0 + x1 * d, h), f2 = box_sd(p0 + x2 * d, h);
      for (int it = 0; it < CUBE_GS_ITERS; it++) {
        if (f1 <= f2) { bb = x2; x2 = x1; f2 = f1; x1 = bb - phi * (bb - a); f1 = box_sd(p0 + x1 * d, h); }
        else { a = x1; x1 = x2; f1 = f2; x2 = a + phi * (bb - a); f2 = box_sd(p0 + x2 * d, h); }
      }
      t = T(0.5) * (a + bb);
    }
    const V3T<T> ps = p0 + t * d;
    const T sd = box_sd(ps, h);
    const T dist = sd - r;
    if (!(dist < thr)) continue;
    // box point and outward normal (cube frame)
    V3T<T> nb, qb;
    const T qx = fabs(ps.x) - h, qy = fabs(ps.y) - h, qz = fabs(ps.z) - h;
    if (tmax(qx, tmax(qy, qz)) > T(0)) {  // outside: the nearest point of the box
      qb = v3(tmin(tmax(ps.x, T(0) - h), h), tmin(tmax(ps.y, T(0) - h), h), tmin(tmax(ps.z, T(0) - h), h));
      const V3T<T> dv = ps - qb;
      const T l = norm(dv);
      nb = l > T(1e-9) ? (T(1) / l) * dv : v3(T(0), T(0), T(1));
    } else {  // inside: through the nearest face
      const int ax = (qx >= qy && qx >= qz) ? 0 : (qy >= qz ? 1 : 2);
      const T c = ax == 0 ? ps.x : (ax == 1 ? ps.y : ps.z);
      const T sg = c < T(0) ? T(-1) : T(1);
      nb = v3(ax == 0 ? sg : T(0), ax == 1 ? sg : T(0), ax == 2 ? sg : T(0));
      qb = v3(ax == 0 ? sg * h : ps.x, ax == 1 ? sg * h : ps.y, ax == 2 ? sg * h : ps.z);
    }
    const V3T<T> n = mul(Rc, nb);
    if (sig) *sig += pbg_contact_hash((uint32_t)sub, (uint32_t)(m.NS + m.NPAIR + 8 + g));
    ContactT<T>& ct = out[nc++];
    ct.cand = m.NS + m.NPAIR + 8 + g;
    ct.body_a = b; ct.body_b = CUBE_BODY;
    ct.pa = xc + mul(Rc, ps) - r * n;
    ct.pb = xc + mul(Rc, qb);
    ct.n = n; ct.dist = dist; ct.mu = T(m.cg_mu[g]);
  }
  return nc;
}

// sig (nullable): adds pbg_contact_hash(sub, candidate) of every active candidate
template <class T>
int detect_contacts(const MV& m, const KinT<T>& k, ContactT<T>* out, uint8_t* slot_active, int sub, uint32_t* sig) {
  int nc = 0;
  const T thr(g_opt[OPT_CONTACT_THR]);
  const double margin = g_opt[OPT_MARGIN];
  for (int s = 0; s < m.NS; s++) {
    int b = m.slot_link[s] + 1;
    V3T<T> c = k.x[b] + mul(k.R[b], v3c<T>(m.slot_point[s]));
    T r(m.slot_radius[s] + margin);
    T dist = c.z - r;
    slot_active[s] = dist < thr;
    if (slot_active[s]) {
      if (sig) *sig += pbg_contact_hash((uint32_t)sub, (uint32_t)s);
      ContactT<T>& ct = out[nc++];
      ct.cand = s;
      ct.body_a = b; ct.body_b = -1;
      ct.pa = c - r * v3(T(0), T(0), T(1));
      ct.pb = v3(c.x, c.y, T(0));
      ct.n = v3(T(0), T(0), T(1));
      ct.dist = dist; ct.mu = T(m.slot_mu[s]);
    }
  }
  for (int p = 0; p < (g_opt[OPT_SELF_COLLISION] != 0.0 ? m.NPAIR : 0); p++) {
    int ba = m.pair_a[p] + 1, bb = m.pair_b[p] + 1;
    V3T<T> a0 = k.x[ba] + mul(k.R[ba], v3c<T>(m.pa0[p])), a1 = k.x[ba] + mul(k.R[ba], v3c<T>(m.pa1[p]));
    V3T<T> b0 = k.x[bb] + mul(k.R[bb], v3c<T>(m.pb0[p])), b1 = k.x[bb] + mul(k.R[bb], v3c<T>(m.pb1[p]));
    V3T<T> ca, cb;
    segment_closest(a0, a1, b0, b1, ca, cb);
    V3T<T> dvec = ca - cb;
    T d = norm(dvec);
    T dist = d - T(m.pra[p] + margin) - T(m.prb[p] + margin);
    if (dist < thr) {
      if (sig) *sig += pbg_contact_hash((uint32_t)sub, (uint32_t)(m.NS + p));
      V3T<T> n = d > T(1e-9) ? (T(1) / d) * dvec : v3(T(0), T(0), T(1));
      ContactT<T>& ct = out[nc++];
      ct.cand = m.NS + p;
      ct.body_a = ba; ct.body_b = bb;
      ct.pa = ca - T(m.pra[p] + margin) * n;
      ct.pb = cb + T(m.prb[p] + margin) * n;
      ct.n = n; ct.dist = dist; ct.mu = T(m.pmu[p]);
    }
  }
  if (m.harder) nc = detect_cube_contacts(m, k, out, nc, sub, sig);
  return nc;
}

// the cube's columns of a row along dir at world point P (v . dir + w . (r x dir)), scaled by sg
template <class T> void cube_row_jacobian(const MV& m, const KinT<T>& k, V3T<T> P, V3T<T> dir, T sg, T* J) {
  const V3T<T> rx = cross(P - k.xc, dir);
  const int c0 = m.NDOF;
  J[c0] = sg * dir.x; J[c0 + 1] = sg * dir.y; J[c0 + 2] = sg * dir.z;
  J[c0 + 3] = sg * rx.x; J[c0 + 4] = sg * rx.y; J[c0 + 5] = sg * rx.z;
}
template <class T> void contact_row_jacobian(const MV& m, const KinT<T>& k, const ContactT<T>& c, V3T<T> dir, T* J) {
  T Jv[3][MAXD], Jw[3][MAXD];
  if (m.harder)
    for (int j = m.NDOF; j < n_total(m); j++) J[j] = T(0);
  if (c.body_a == CUBE_BODY) {  // cube vs floor
    for (int j = 0; j < m.NDOF; j++) J[j] = T(0);
    cube_row_jacobian(m, k, c.pa, dir, T(1), J);
    return;
  }
  point_jacobian(m, k, c.body_a, c.pa, Jv, Jw);
  for (int j = 0; j < m.NDOF; j++) J[j] = dir.x * Jv[0][j] + dir.y * Jv[1][j] + dir.z * Jv[2][j];
  if (c.body_b == CUBE_BODY) {
    cube_row_jacobian(m, k, c.pb, dir, T(-1), J);
  } else if (c.body_b >= 0) {
    point_jacobian(m, k, c.body_b, c.pb, Jv, Jw);
    for (int j = 0; j < m.NDOF; j++) J[j] = J[j] - (dir.x * Jv[0][j] + dir.y * Jv[1][j] + dir.z * Jv[2][j]);
  }
}

// angular row: relative angular velocity of body A w.r.t. body B about dir (rolling / spinning
// friction, rule study)
template <class T> void contact_angular_jacobian(const MV& m, const KinT<T>& k, const ContactT<T>& c, V3T<T> dir, T* J) {
  T Jv[3][MAXD], Jw[3][MAXD];
  point_jacobian(m, k, c.body_a, c.pa, Jv, Jw);
  for (int j = 0; j < m.NDOF; j++) J[j] = dir.x * Jw[0][j] + dir.y * Jw[1][j] + dir.z * Jw[2][j];
  if (c.body_b >= 0) {
    point_jacobian(m, k, c.body_b, c.pb, Jv, Jw);
    for (int j = 0; j < m.NDOF; j++) J[j] = J[j] - (dir.x * Jw[0][j] + dir.y * Jw[1][j] + dir.z * Jw[2][j]);
  }
}

template <class T> inline T dotn(int n, const T* a, const T* b) {
  T s(0);
  for (int i = 0; i < n; i++) s = s + a[i] * b[i];
  return s;
}

// Row setup: W = M^-1 J^T, m_eff, and the target of J nu_new.  Positional rows (contact
// normals, joint limits) use Bullet's rhs (btMultiBodyConstraintSolver::
// setupMultiBodyContactConstraint: velocityError = -rel_vel, minus pos/dt when separated;
// positionalError = -erp pos/dt when penetrating), i.e. J nu_new >= -pos/dt (separated,
// speculative) or >= -erp pos/dt (penetrating); erp < 0: no positional term (J nu_new >= 0).  sep_abs = false
// is the round-1 relative form J dnu >= -pos/dt (kept for the rule study).
template <class T>
void setup_row(int n, const T L[MAXD][MAXD], const T* nu, RowT<T>& r, T pos, int positional, double erp, T dt,
               bool sep_abs, double cfm = 0.0) {
  chol_solve(n, L, r.J, r.W);
  T D = dotn(n, r.J, r.W) + T(cfm);
  r.meff = D > T(1e-12) ? T(1) / D : T(0);
  T vJ = dotn(n, r.J, nu);
  if (!positional) r.target = T(0);                                       // friction
  else if (pos > T(0)) r.target = (sep_abs ? T(0) : vJ) - pos / dt;         // [EXT] separated
  else if (erp < 0) r.target = T(0);                                      // velocity only: J nu_new >= 0
  else r.target = T(0) - T(erp) * pos / dt;                               // Baumgarte push-out
  r.lambda = T(0);
}

// returns the clamp code of the update (sim_params.h pbg_clamp_code)
template <class T> inline uint32_t solve_row(int n, RowT<T>& r, T* nu) {
  T delta = r.meff * (r.target - dotn(n, r.J, nu));
  T nl = r.lambda + delta;
  const uint32_t code = pbg_clamp_code(nl, r.lo, r.hi);
  if (nl < r.lo) nl = r.lo;
  if (nl > r.hi) nl = r.hi;
  delta = nl - r.lambda;
  r.lambda = nl;
  for (int i = 0; i < n; i++) nu[i] = nu[i] + r.W[i] * delta;
  return code;
}

template <class T> inline T clampv(T v) {
  const T mx(g_opt[OPT_MAX_COORD_VEL]);  // PBG_MAX_COORD_VELOCITY unless the rule study changes it
  return v > mx ? mx : (v < T(0) - mx ? T(0) - mx : v);
}

// Free body (the floating base, the cube): record words [pos 3 | quat 4 | v 3 | w 3] from its
// generalized velocity nu = [v, w]; semi-implicit Euler, exponential-map quaternion update
// with the world angular velocity  [EXT] btMultiBody pQuatUpdateFun
template <class T> void integrate_free_body(T* s, const T* nu, T dt) {
  for (int i = 0; i < 3; i++) { s[7 + i] = nu[i]; s[10 + i] = nu[3 + i]; s[i] = s[i] + dt * nu[i]; }
  V3T<T> w = v3p(s + 10);
  T ang = norm(w);
  const T thr(PBG_ANGULAR_MOTION_THRESHOLD), half(0.5);
  if (ang * dt > thr) ang = thr / dt;
  V3T<T> ax;
  if (ang < T(0.001)) ax = (half * dt - (dt * dt * dt) * T(0.020833333333) * ang * ang) * w;
  else ax = (sin(half * ang * dt) / ang) * w;
  T dw = cos(half * ang * dt);
  T* qt = s + 3;
  T x = qt[0], y = qt[1], z = qt[2], ww = qt[3];
  // dq * q (Hamilton, xyzw)
  T nx = dw * x + ax.x * ww + ax.y * z - ax.z * y;
  T ny = dw * y - ax.x * z + ax.y * ww + ax.z * x;
  T nz = dw * z + ax.x * y - ax.y * x + ax.z * ww;
  T nw = dw * ww - ax.x * x - ax.y * y - ax.z * z;
  T inv = T(1) / sqrt(nx * nx + ny * ny + nz * nz + nw * nw);
  qt[0] = nx * inv; qt[1] = ny * inv; qt[2] = nz * inv; qt[3] = nw * inv;
}

// ------------------------------------------------------------------ one sub-step
// s: the env's state record in T.  tau: motor torque on joint dofs, held over the env step
// (robot_locomotors.py:26-29).  qd_step: joint velocities at the start of the env step
// (rule study: damping once per step).  cache (nullable, T = double only): warm-start store.
// Returns the number of contacts; slot_active receives the floor-slot flags.
// asig (nullable): adds the solver active-set events (sim_params.h pbg_solver_event).
template <class T>
int substep(const MV& m, T* s, const T* tau, uint8_t* slot_active, int sub, uint32_t* sig, double* cache,
            const T* qd_step, uint32_t* asig) {
  const T dt(sim_dt(m));
  const int n = n_total(m);  // the robot's generalized velocity (+ the cube's 6)
  static thread_local KinT<T> k;
  static thread_local T M[MAXD][MAXD];
  static thread_local RowT<T> rows[MAXROWS];
  static thread_local ContactT<T> cts[MAXCAND];
  T C[MAXD], rhs[MAXD], qdd[MAXD], nu[MAXD];
  forward_kinematics(m, s, k);
  if constexpr (std::is_same<T, double>::value) mass_and_bias(m, k, M, C, s);
  else mass_and_bias_ref(m, k, M, C, s);  // float32 envelopes: the kernels' formulation
  // joint damping tau = -d*qd from this sub-step's velocity (explicit; [EXT] pybullet
  // applyJointDamping -- applied per sub-step here, the stable choice at dt/4)
  const T* qd0 = s + PBG_BASE_WORDS + m.NJ;
  for (int i = 0; i < n; i++) rhs[i] = T(0) - C[i];
  const T* qdd_src = g_opt[OPT_DAMP_MODE] != 0.0 ? qd_step : qd0;  // applyJointDamping once per step
  for (int d = 0; d < m.NJ; d++)
    rhs[gidx(m, d)] = rhs[gidx(m, d)] + (tau[d] - ((g_flags & 8) ? T(0) : T(m.damping[d]) * qdd_src[d]));
  // joint springs tau = -k*q (mjcf.py B7: MJCF <joint stiffness>, explicit per sub-step like the
  // damping; the rule study scales k by OPT_SPRINGS, 0 = none)
  if (g_opt[OPT_SPRINGS] != 0.0)
    for (int d = 0; d < m.NJ; d++)
      if (m.stiffness[d] != 0.0)
        rhs[gidx(m, d)] = rhs[gidx(m, d)] - T(g_opt[OPT_SPRINGS] * m.stiffness[d]) * s[PBG_BASE_WORDS + d];
  cholesky(n, M);
  chol_solve(n, M, rhs, qdd);
  // generalized velocity nu = [v_base, w_base, qd]
  T* q = s + PBG_BASE_WORDS;
  T* qd = q + m.NJ;
  if (m.floating) {
    for (int i = 0; i < 3; i++) { nu[i] = s[7 + i]; nu[3 + i] = s[10 + i]; }
  }
  for (int d = 0; d < m.NJ; d++) nu[gidx(m, d)] = qd[d];
  T* cs = s + cube_word(m);  // HumanoidFlagrunHarder's cube (n_total)
  if (m.harder)
    for (int i = 0; i < 3; i++) { nu[m.NDOF + i] = cs[7 + i]; nu[m.NDOF + 3 + i] = cs[10 + i]; }
  for (int i = 0; i < n; i++) nu[i] = clampv(nu[i] + dt * qdd[i]);

  // constraint rows, Bullet order: joint limits, contact normals, frictions
  int nr = 0;
  for (int d = 0; d < m.NJ; d++) {
    if (!m.limited[d] || (g_flags & 1)) continue;
    for (int side = 0; side < 2; side++) {
      T pos = side == 0 ? q[d] - T(m.lower[d]) : T(m.upper[d]) - q[d];
      if (g_opt[OPT_LIMIT_MODE] != 0.0 && pos > T(0)) continue;  // btMultiBodyJointLimitConstraint: violated only
      RowT<T>& r = rows[nr++];
      for (int i = 0; i < n; i++) r.J[i] = T(0);
      r.J[gidx(m, d)] = side == 0 ? T(1) : T(-1);
      double lerp = g_opt[OPT_LIMIT_ERP];
      if (g_opt[OPT_LIM_DEEP_MODE] != 0.0 && pos <= T(g_opt[OPT_DEEP_THR]))
        lerp = g_opt[OPT_LIM_DEEP_MODE] == 1.0 ? -1.0 : 0.9;
      setup_row(n, M, nu, r, pos, 1, lerp, dt, g_opt[OPT_LIM_SEP_ABS] != 0.0, g_opt[OPT_LIMIT_CFM]);
      r.lo = T(0); r.hi = T(PBG_LIMIT_MAX_IMPULSE); r.normal = -1;
    }
  }
  int nc = detect_contacts(m, k, cts, slot_active, sub, sig);
  if (g_flags & 2) nc = 0;
  // contact -> collision candidate (the warm-start cache key): slots in order, then pairs
  int cand[MAXCAND];
  for (int c = 0; c < nc; c++) cand[c] = cts[c].cand;
  if (g_opt[OPT_SEP_MODE] != 0.0) {  // drop separated contacts (no speculative rows)
    int w = 0;
    for (int c = 0; c < nc; c++)
      if (cts[c].dist + T(g_opt[OPT_SLOP]) <= T(0)) { cts[w] = cts[c]; cand[w] = cand[c]; w++; }
    nc = w;
  }
  int first_normal = nr;
  const double erp = g_opt[OPT_CONTACT_ERP] < 0 ? m.contact_erp : g_opt[OPT_CONTACT_ERP];
  const double deep_erp = g_opt[OPT_DEEP_ERP] < 0 ? erp : g_opt[OPT_DEEP_ERP];
  for (int c = 0; c < nc; c++) {
    RowT<T>& r = rows[nr++];
    contact_row_jacobian(m, k, cts[c], cts[c].n, r.J);
    const T dist = cts[c].dist + T(g_opt[OPT_SLOP]);
    const bool deep = dist <= T(g_opt[OPT_DEEP_THR]);
    const double e = deep ? (g_opt[OPT_DEEP_MODE] != 0.0 ? -1.0 : deep_erp) : erp;
    setup_row(n, M, nu, r, dist, 1, e, dt, g_opt[OPT_SEP_ABS] != 0.0, g_opt[OPT_CONTACT_CFM]);
    // restitution of a robot-floor contact (HalfCheetahMuJoCo: 0.5 x 0.5): [EXT]
    // btMultiBodyConstraintSolver::setupMultiBodyContactConstraint takes restitutionCurve(rel_vel) of
    // the pre-solve normal velocity -- e * (-v_n) when |v_n| >= the threshold, clamped at 0 -- into
    // velocityError = restitution - rel_vel, i.e. the target of J nu_new rises by it
    if (m.restitution > 0.0 && cts[c].body_b == -1 && cts[c].body_a != CUBE_BODY) {
      const T vn = dotn(n, r.J, nu);
      const T av = vn < T(0) ? T(0) - vn : vn;
      const T rest = av < T(PBG_RESTITUTION_VELOCITY_THRESHOLD) ? T(0) : T(m.restitution) * (T(0) - vn);
      if (rest > T(0)) r.target = r.target + rest;
    }
    r.lo = T(0); r.hi = T(1e30); r.normal = -1; r.mu = cts[c].mu;
  }
  // spinning (about the normal) and rolling (about the two tangents) friction: angular rows of
  // the robot-floor contacts, bounded by +-mu_t lambda_n under a positive normal impulse, solved
  // after the normals and before the lateral friction ([EXT] btMultiBodyConstraintSolver's
  // torsional friction constraints, addMultiBodyTorsionalFrictionConstraint: angular Jacobian,
  // zero target).  mu_t: the model's combined coefficients (HalfCheetahMuJoCo 0.1 x 0.8); the rule
  // study's OPT_SPIN_MU / OPT_ROLL_MU override them for every robot.
  const double spin = g_opt[OPT_SPIN_MU] > 0.0 ? g_opt[OPT_SPIN_MU] : m.spin_mu;
  const double roll = g_opt[OPT_ROLL_MU] > 0.0 ? g_opt[OPT_ROLL_MU] : m.roll_mu;
  const int first_torsion = nr;
  if (spin > 0.0 || roll > 0.0) {
    for (int c = 0; c < nc; c++) {
      V3T<T> t1, t2;
      plane_space(cts[c].n, t1, t2);
      for (int a = 0; a < 3; a++) {
        const double mu = a == 0 ? spin : roll;
        if (!(mu > 0.0)) continue;
        RowT<T>& r = rows[nr++];
        contact_angular_jacobian(m, k, cts[c], a == 0 ? cts[c].n : (a == 1 ? t1 : t2), r.J);
        setup_row(n, M, nu, r, T(0), 0, 0.0, dt, false, g_opt[OPT_CONTACT_CFM]);
        r.normal = first_normal + c; r.mu = T(mu); r.lo = r.hi = T(0);
      }
    }
  }
  int first_friction = nr;
  const int fric_dirs = g_opt[OPT_FRIC_MODE] == 2.0 ? 1 : 2;
  for (int c = 0; c < nc; c++) {
    V3T<T> t1, t2;
    plane_space(cts[c].n, t1, t2);
    for (int f = 0; f < fric_dirs; f++) {
      RowT<T>& r = rows[nr++];
      contact_row_jacobian(m, k, cts[c], f == 0 ? t1 : t2, r.J);
      setup_row(n, M, nu, r, T(0), 0, 0.0, dt, false, g_opt[OPT_CONTACT_CFM]);
      r.normal = first_normal + c; r.mu = cts[c].mu; r.lo = r.hi = T(0);
    }
  }
  // warm start: last sub-step's impulses of the same candidates (Bullet's persistent
  // manifold points carry m_appliedImpulse), scaled by the warm-start factor
  const T wf(g_opt[OPT_WARM]);
  if (cache && g_opt[OPT_WARM] != 0.0) {
    for (int c = 0; c < nc; c++) {
      if (cand[c] < 0) continue;
      const double* cc = cache + 4 * cand[c];
      if (cc[3] == 0.0) continue;
      RowT<T>& rn = rows[first_normal + c];
      rn.lambda = wf * T(cc[0]);
      for (int i = 0; i < n; i++) nu[i] = nu[i] + rn.W[i] * rn.lambda;
      if (g_opt[OPT_WARM_FRIC] != 0.0)
        for (int f = 0; f < fric_dirs; f++) {
          RowT<T>& rf = rows[first_friction + fric_dirs * c + f];
          rf.lambda = wf * T(cc[1 + f]);
          for (int i = 0; i < n; i++) nu[i] = nu[i] + rf.W[i] * rf.lambda;
        }
    }
  }
  const int iters = (int)g_opt[OPT_ITERS];
  const bool cone = g_opt[OPT_FRIC_MODE] == 1.0;
  // solver-event row ids: limits 2 li + side (first_normal rows), contact c 2 NLIM + 3 c + dir
  auto event = [&](int it, int row, uint32_t code) {
    if (asig && code) *asig += pbg_solver_event((uint32_t)sub, (uint32_t)it, (uint32_t)row, code);
  };
  auto crow = [&](int i) {  // the event row id of constraint row i
    if (i < first_normal) return i;
    if (i < first_torsion) return first_normal + 3 * (i - first_normal);
    const int c = (i - first_friction) / fric_dirs;
    return first_normal + 3 * c + 1 + (i - first_friction - fric_dirs * c);
  };
  for (int it = 0; it < iters; it++) {
    for (int i = 0; i < first_torsion; i++) event(it, crow(i), solve_row(n, rows[i], nu));
    for (int i = first_torsion; i < first_friction; i++) {  // torsional rows (no solver events)
      const T ln = rows[rows[i].normal].lambda;
      if (!(ln > T(0))) continue;
      rows[i].lo = T(0) - rows[i].mu * ln;
      rows[i].hi = rows[i].mu * ln;
      solve_row(n, rows[i], nu);
    }
    for (int i = first_friction; i < nr; i += (cone ? 2 : 1)) {
      T ln = rows[rows[i].normal].lambda;
      if (!(ln > T(0)) && (i - first_friction) % fric_dirs == 0) event(it, crow(i), 3u);
      if (ln > T(0)) {  // [EXT] Bullet solves a friction row only under a positive normal impulse
        if (cone) {  // btMultiBodyConstraintSolver::resolveConeFrictionConstraintRows
          RowT<T>& a = rows[i];
          RowT<T>& b = rows[i + 1];
          const T lim = a.mu * ln;
          T da = a.meff * (a.target - dotn(n, a.J, nu));
          T db = b.meff * (b.target - dotn(n, b.J, nu));
          T na = a.lambda + da, nb = b.lambda + db;
          const T mag = sqrt(na * na + nb * nb);
          if (mag > lim && mag > T(0)) { na = na * (lim / mag); nb = nb * (lim / mag); }
          da = na - a.lambda; db = nb - b.lambda;
          a.lambda = na; b.lambda = nb;
          for (int k2 = 0; k2 < n; k2++) nu[k2] = nu[k2] + (a.W[k2] * da + b.W[k2] * db);
        } else {
          rows[i].lo = T(0) - rows[i].mu * ln;
          rows[i].hi = rows[i].mu * ln;
          event(it, crow(i), solve_row(n, rows[i], nu));
        }
      }
    }
  }
  if (g_diag) {  // contact diagnostics (rule study)
    for (int c = 0; c < nc && g_diag_n < g_diag_cap; c++) {
      double* o = g_diag + 10 * g_diag_n++;
      const RowT<T>& rn = rows[first_normal + c];
      o[0] = sub; o[1] = cts[c].cand; o[2] = (double)cts[c].dist; o[3] = (double)rn.lambda;
      o[6] = (double)cts[c].mu; o[7] = (double)dotn(n, rn.J, nu);
      for (int f = 0; f < 2; f++) {
        const bool have = f < fric_dirs;
        const RowT<T>& rf = rows[first_friction + fric_dirs * c + (have ? f : 0)];
        o[4 + f] = have ? (double)rf.lambda : 0.0;
        o[8 + f] = have ? (double)dotn(n, rf.J, nu) : 0.0;
      }
    }
  }
  if (cache) {
    for (int i = 0; i < MAXCAND; i++) cache[4 * i + 3] = 0.0;
    for (int c = 0; c < nc; c++) {
      if (cand[c] < 0) continue;
      double* cc = cache + 4 * cand[c];
      cc[0] = (double)rows[first_normal + c].lambda;
      cc[1] = (double)rows[first_friction + fric_dirs * c].lambda;
      cc[2] = fric_dirs > 1 ? (double)rows[first_friction + fric_dirs * c + 1].lambda : 0.0;
      cc[3] = 1.0;
    }
  }
  for (int i = 0; i < n; i++) nu[i] = clampv(nu[i]);

  // integrate positions (semi-implicit Euler)
  for (int d = 0; d < m.NJ; d++) {
    qd[d] = nu[gidx(m, d)];
    q[d] = q[d] + dt * qd[d];
  }
  if (m.floating) integrate_free_body(s, nu, dt);
  if (m.harder) integrate_free_body(cs, nu + m.NDOF, dt);
  return nc;
}

// The env step's physics in T: apply_action's torques (from the float32 action, as the
// kernels: act_gain * clip(a) in double, rounded to T), `substeps` sub-steps.  state: the
// env's float64 record, read into T and written back (T = double: in place).
template <class T>
int physics_step(const MV& m, double* state, const float* ac, uint8_t* slot_active, uint32_t* sig, double* cache,
                 uint32_t* asig = nullptr) {
  T s[PBG_BASE_WORDS + 2 * MAXD + PBG_CUBE_WORDS], tau[MAXD], qd_step[MAXD];
  const int SD = PBG_STATE_WORDS(m.NJ, m.harder);
  for (int i = 0; i < SD; i++) s[i] = T(state[i]);
  for (int d = 0; d < m.NJ; d++) tau[d] = T(0);
  for (int i = 0; i < m.NA; i++) {  // robot_locomotors.py:26-29
    float c = ac[i] < -1.0f ? -1.0f : (ac[i] > 1.0f ? 1.0f : ac[i]);
    tau[m.act_dof[i]] = tau[m.act_dof[i]] + T(m.act_gain[i] * (double)c);
  }
  for (int d = 0; d < m.NJ; d++) qd_step[d] = s[PBG_BASE_WORDS + m.NJ + d];
  int nc = 0;
  // apply_action's torques in the first OPT_TORQUE_SUBSTEPS sub-steps (default: all; rule study)
  const int tsub = g_opt[OPT_TORQUE_SUBSTEPS] < 0 ? sim_substeps(m) : (int)g_opt[OPT_TORQUE_SUBSTEPS];
  T zero_tau[MAXD];
  for (int d = 0; d < m.NJ; d++) zero_tau[d] = T(0);
  for (int sub = 0; sub < sim_substeps(m); sub++)
    nc = substep<T>(m, s, sub < tsub ? tau : zero_tau, slot_active, sub, sig, cache, qd_step, asig);
  for (int i = 0; i < SD; i++) state[i] = (double)s[i];
  return nc;
}
