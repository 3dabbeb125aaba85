// pbg_oracle.cpp -- CPU restatement of the reference's hot path.  TEST INFRASTRUCTURE ONLY.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
// library, and only as the checker / the timed CPU baseline.  The product path
// (pybullet-gym_amd/csrc, libpbg_amd.so) never links or calls it.
//
// What it restates (file:line relative to /root/reference):
//   * WalkerBaseBulletEnv._step        pybulletgym/envs/roboschool/gym_locomotion_envs.py:54-114
//   * WalkerBase.apply_action          pybulletgym/envs/roboschool/robot_locomotors.py:26-29
//   * WalkerBase.calc_state/potential  robot_locomotors.py:31-79, robot_bases.py:209-325
//   * alive bonuses                    robot_locomotors.py:89-90,116-118,137-138,191-192
//   * WalkerBaseBulletEnv._reset       gym_locomotion_envs.py:22-39 + robot_locomotors.py:16-24
//   * InvertedPendulumBulletEnv        gym_pendulum_envs.py:16-39, robot_pendula.py:11-51
//   * World.step -> stepSimulation     scene_bases.py:47-52,58-76  [EXT: Bullet btMultiBody]
//
// The physics inside stepSimulation() is Bullet's (third-party, not in /root/reference,
// not installed here): it is restated from Bullet's published algorithm -- joint-space
// Featherstone dynamics (composite-rigid-body mass matrix + recursive Newton-Euler bias,
// Cholesky solve; equal to the articulated-body algorithm's result), Bullet-style body
// damping, sequential-impulse PGS over joint-limit / contact-normal / friction rows with
// Baumgarte ERP, semi-implicit Euler with exponential-map base rotation.  PHYSICS PARITY
// WITH PYBULLET IS UNPINNED (nothing in this container can run pybullet).  The
// observation/reward/done pack (pbg_oracle_pack) IS pinned: tests/golden/ holds vectors
// produced by the reference's own Python (tests/golden/make_golden.py).
//
// Plain double-precision scalar code; loops at run time over the model tables of
// csrc/models_gen.h.  Build: oracle/Makefile.
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

#include "../pybullet-gym_amd/csrc/models_gen.h"
#include "../pybullet-gym_amd/csrc/sim_params.h"

#define MAXL 24
#define MAXD 32
#define MAXS 32
#define MAXPAIR 72
#define MAXROWS (2 * MAXD + 3 * (MAXS + MAXPAIR))

namespace {

// Test switches (pbg_oracle_set_flags): bit0 no joint limits, bit1 no contacts, bit2 no body
// damping, bit3 no joint damping, bit4 no gravity.  0 in every product-parity comparison.
int g_flags = 0;

// ------------------------------------------------------------------ model view
struct MV {
  int robot_id, kind, floating, NL, NJ, NDOF, NA, NO, NR, NF, NP, NS, NPAIR, OBS, alive, substeps,
      floor, max_steps, robot_body, tip_link, flagrun;
  double power, elec, stall, jal, z0fixed, dt_sub, base_mass, power_cost, qvel_clip;
  const double *base_inertia, *base_pos, *base_quat;
  const int *link_parent, *link_jtype, *link_dof;
  const double (*off_pos)[3], (*axis)[3], (*anchor)[3], (*com)[3], (*off_quat)[4], (*inertia)[6];
  const double* mass;
  const double *lower, *upper, *damping, *armature;
  const int *limited, *dof_jtype;
  const int* act_dof; const double* act_gain;
  const int* obs_dof; const double* obs_vel_scale; const int* reset_dof; const double* reset_offset;
  const int* part_link; const int* foot_link;
  const int* slot_link; const double (*slot_point)[3]; const double *slot_radius, *slot_mu;
  const int *pair_a, *pair_b; const double (*pa0)[3], (*pa1)[3], (*pb0)[3], (*pb1)[3];
  const double *pra, *prb, *pmu;
};

template <class R>
MV view() {
  MV m;
  m.robot_id = R::robot_id; m.kind = R::kind; m.floating = R::floating; m.NL = R::NL; m.NJ = R::NJ;
  m.NDOF = R::NDOF; m.NA = R::NA; m.NO = R::NO; m.NR = R::NR; m.NF = R::NF; m.NP = R::NP;
  m.NS = R::NS; m.NPAIR = R::NPAIR; m.OBS = R::OBS; m.alive = R::alive; m.substeps = R::substeps;
  m.floor = R::floor; m.max_steps = R::max_episode_steps; m.robot_body = R::robot_body; m.tip_link = R::tip_link;
  m.flagrun = R::flagrun;
  m.power = R::power; m.elec = R::electricity_cost; m.stall = R::stall_torque_cost;
  m.jal = R::joints_at_limit_cost; m.z0fixed = R::initial_z_fixed; m.dt_sub = R::dt_sub;
  m.base_mass = R::base_mass; m.power_cost = R::power_cost; m.qvel_clip = R::qvel_clip; m.base_inertia = R::base_inertia; m.base_pos = R::base_pos;
  m.base_quat = R::base_quat; m.link_parent = R::link_parent; m.link_jtype = R::link_jtype;
  m.link_dof = R::link_dof; m.off_pos = R::link_offset_pos; m.axis = R::link_axis;
  m.anchor = R::link_anchor; m.com = R::link_com; m.off_quat = R::link_offset_quat;
  m.inertia = R::link_inertia; m.mass = R::link_mass; m.lower = R::dof_lower; m.upper = R::dof_upper;
  m.damping = R::dof_damping; m.armature = R::dof_armature; m.limited = R::dof_limited;
  m.dof_jtype = R::dof_jtype; m.act_dof = R::act_dof; m.act_gain = R::act_gain;
  m.obs_dof = R::obs_dof; m.obs_vel_scale = R::obs_vel_scale; m.reset_dof = R::reset_dof;
  m.reset_offset = R::reset_offset;
  m.part_link = R::part_link; m.foot_link = R::foot_link; m.slot_link = R::slot_link;
  m.slot_point = R::slot_point; m.slot_radius = R::slot_radius; m.slot_mu = R::slot_mu;
  m.pair_a = R::pair_link_a; m.pair_b = R::pair_link_b; m.pa0 = R::pair_a0; m.pa1 = R::pair_a1;
  m.pb0 = R::pair_b0; m.pb1 = R::pair_b1; m.pra = R::pair_ra; m.prb = R::pair_rb; m.pmu = R::pair_mu;
  return m;
}

const MV* model(int robot) {
  static MV views[15] = {view<pbg_models::Pendulum>(), view<pbg_models::Hopper>(),
                         view<pbg_models::HalfCheetah>(), view<pbg_models::Ant>(),
                         view<pbg_models::Humanoid>(), view<pbg_models::Walker2D>(),
                         view<pbg_models::PendulumSwingup>(), view<pbg_models::DoublePendulum>(),
                         view<pbg_models::HumanoidFlagrun>(), view<pbg_models::HopperMuJoCo>(),
                         view<pbg_models::Walker2DMuJoCo>(), view<pbg_models::HalfCheetahMuJoCo>(),
                         view<pbg_models::AntMuJoCo>(), view<pbg_models::HumanoidMuJoCo>(),
                         view<pbg_models::DoublePendulumMuJoCo>()};
  if (robot < 0 || robot > 14) return nullptr;
  return &views[robot];
}

// ------------------------------------------------------------------ small linear algebra
struct V3 { double x, y, z; };
inline V3 v3(double x, double y, double z) { V3 r = {x, y, z}; return r; }
inline V3 v3(const double* p) { return v3(p[0], p[1], p[2]); }
inline V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator*(double s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
inline double norm(V3 a) { return sqrt(dot(a, a)); }

struct M3 { double m[3][3]; };
inline V3 mul(const M3& A, V3 v) {
  return v3(A.m[0][0] * v.x + A.m[0][1] * v.y + A.m[0][2] * v.z,
            A.m[1][0] * v.x + A.m[1][1] * v.y + A.m[1][2] * v.z,
            A.m[2][0] * v.x + A.m[2][1] * v.y + A.m[2][2] * v.z);
}
inline M3 mul(const M3& A, const M3& B) {
  M3 C;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) C.m[i][j] = A.m[i][0] * B.m[0][j] + A.m[i][1] * B.m[1][j] + A.m[i][2] * B.m[2][j];
  return C;
}
inline M3 quat_to_m3(const double* q) {  // q = (x, y, z, w)
  double x = q[0], y = q[1], z = q[2], w = q[3];
  M3 R;
  R.m[0][0] = 1 - 2 * (y * y + z * z); R.m[0][1] = 2 * (x * y - w * z); R.m[0][2] = 2 * (x * z + w * y);
  R.m[1][0] = 2 * (x * y + w * z); R.m[1][1] = 1 - 2 * (x * x + z * z); R.m[1][2] = 2 * (y * z - w * x);
  R.m[2][0] = 2 * (x * z - w * y); R.m[2][1] = 2 * (y * z + w * x); R.m[2][2] = 1 - 2 * (x * x + y * y);
  return R;
}
inline M3 axis_angle_m3(V3 a, double ang) {  // unit axis
  double c = cos(ang), s = sin(ang), t = 1 - c;
  M3 R;
  R.m[0][0] = t * a.x * a.x + c;       R.m[0][1] = t * a.x * a.y - s * a.z; R.m[0][2] = t * a.x * a.z + s * a.y;
  R.m[1][0] = t * a.x * a.y + s * a.z; R.m[1][1] = t * a.y * a.y + c;       R.m[1][2] = t * a.y * a.z - s * a.x;
  R.m[2][0] = t * a.x * a.z - s * a.y; R.m[2][1] = t * a.y * a.z + s * a.x; R.m[2][2] = t * a.z * a.z + c;
  return R;
}
// world inertia R I R^T from the 6-vector (xx,yy,zz,xy,xz,yz)
inline M3 world_inertia(const M3& R, const double* I6) {
  M3 I = {{{I6[0], I6[3], I6[4]}, {I6[3], I6[1], I6[5]}, {I6[4], I6[5], I6[2]}}};
  M3 RI = mul(R, I), W;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) W.m[i][j] = RI.m[i][0] * R.m[j][0] + RI.m[i][1] * R.m[j][1] + RI.m[i][2] * R.m[j][2];
  return W;
}
// M3 -> quaternion (x,y,z,w)
inline void m3_to_quat(const M3& m, double* q) {
  double t = m.m[0][0] + m.m[1][1] + m.m[2][2];
  if (t > 0) {
    double s = sqrt(t + 1.0) * 2;
    q[3] = 0.25 * s; q[0] = (m.m[2][1] - m.m[1][2]) / s; q[1] = (m.m[0][2] - m.m[2][0]) / s; q[2] = (m.m[1][0] - m.m[0][1]) / s;
  } else if (m.m[0][0] > m.m[1][1] && m.m[0][0] > m.m[2][2]) {
    double s = sqrt(1.0 + m.m[0][0] - m.m[1][1] - m.m[2][2]) * 2;
    q[3] = (m.m[2][1] - m.m[1][2]) / s; q[0] = 0.25 * s; q[1] = (m.m[0][1] + m.m[1][0]) / s; q[2] = (m.m[0][2] + m.m[2][0]) / s;
  } else if (m.m[1][1] > m.m[2][2]) {
    double s = sqrt(1.0 + m.m[1][1] - m.m[0][0] - m.m[2][2]) * 2;
    q[3] = (m.m[0][2] - m.m[2][0]) / s; q[0] = (m.m[0][1] + m.m[1][0]) / s; q[1] = 0.25 * s; q[2] = (m.m[1][2] + m.m[2][1]) / s;
  } else {
    double s = sqrt(1.0 + m.m[2][2] - m.m[0][0] - m.m[1][1]) * 2;
    q[3] = (m.m[1][0] - m.m[0][1]) / s; q[0] = (m.m[0][2] + m.m[2][0]) / s; q[1] = (m.m[1][2] + m.m[2][1]) / s; q[2] = 0.25 * s;
  }
}

// ------------------------------------------------------------------ kinematics
struct Kin {
  M3 R[MAXL + 1];      // index 0 = base, l+1 = link l
  V3 x[MAXL + 1];      // frame origin (base: COM)
  V3 c[MAXL + 1];      // COM world
  V3 w[MAXL + 1], v[MAXL + 1];      // angular velocity, COM linear velocity
  V3 al[MAXL + 1], ac[MAXL + 1];    // bias angular / COM linear acceleration
  V3 ja[MAXD], jo[MAXD];            // per joint dof: world axis, world anchor
};

void forward_kinematics(const MV& m, const double* s, Kin& k) {
  const double* q = s + PBG_BASE_WORDS;
  const double* qd = q + m.NJ;
  k.R[0] = quat_to_m3(s + 3);
  k.x[0] = v3(s);
  k.c[0] = k.x[0];
  k.w[0] = m.floating ? v3(s + 10) : v3(0, 0, 0);
  k.v[0] = m.floating ? v3(s + 7) : v3(0, 0, 0);
  k.al[0] = v3(0, 0, 0);
  k.ac[0] = v3(0, 0, 0);
  for (int l = 0; l < m.NL; l++) {
    int p = m.link_parent[l] + 1;
    M3 Ro = quat_to_m3(m.off_quat[l]);
    M3 R0 = mul(k.R[p], Ro);
    V3 x0 = k.x[p] + mul(k.R[p], v3(m.off_pos[l]));
    V3 axl = v3(m.axis[l]), anl = v3(m.anchor[l]);
    int jt = m.link_jtype[l], d = m.link_dof[l];
    M3 R = R0;
    V3 x = x0;
    if (jt == 0) {
      M3 Rj = axis_angle_m3(axl, q[d]);
      R = mul(R0, Rj);
      x = x0 + mul(R0, anl - mul(Rj, anl));
    } else if (jt == 1) {
      x = x0 + mul(R0, q[d] * axl);
    }
    k.R[l + 1] = R;
    k.x[l + 1] = x;
    k.c[l + 1] = x + mul(R, v3(m.com[l]));
    V3 cp = k.c[p], wp = k.w[p], vp = k.v[p], alp = k.al[p], acp = k.ac[p];
    V3 c = k.c[l + 1];
    if (jt == 0) {
      V3 a = mul(R0, axl), o = x0 + mul(R0, anl);
      k.ja[d] = a; k.jo[d] = o;
      V3 ro = o - cp;
      V3 vo = vp + cross(wp, ro);
      V3 ao = acp + cross(alp, ro) + cross(wp, cross(wp, ro));
      V3 w = wp + qd[d] * a;
      V3 al = alp + qd[d] * cross(wp, a);
      V3 rc = c - o;
      k.w[l + 1] = w; k.al[l + 1] = al;
      k.v[l + 1] = vo + cross(w, rc);
      k.ac[l + 1] = ao + cross(al, rc) + cross(w, cross(w, rc));
    } else if (jt == 1) {
      V3 a = mul(R0, axl);
      k.ja[d] = a; k.jo[d] = x0;
      V3 r = c - cp;
      k.w[l + 1] = wp; k.al[l + 1] = alp;
      k.v[l + 1] = vp + cross(wp, r) + qd[d] * a;
      k.ac[l + 1] = acp + cross(alp, r) + cross(wp, cross(wp, r)) + (2.0 * qd[d]) * cross(wp, a);
    } else {
      V3 r = c - cp;
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
void point_jacobian(const MV& m, const Kin& k, int b, V3 P, double Jv[3][MAXD], double Jw[3][MAXD]) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < m.NDOF; j++) Jv[i][j] = Jw[i][j] = 0.0;
  if (m.floating) {
    V3 r = P - k.x[0];
    for (int e = 0; e < 3; e++) {
      V3 ax = v3(e == 0, e == 1, e == 2);
      Jv[e][e] = 1.0;
      V3 lin = cross(ax, r);
      Jv[0][3 + e] = lin.x; Jv[1][3 + e] = lin.y; Jv[2][3 + e] = lin.z;
      Jw[e][3 + e] = 1.0;
    }
  }
  int l = b - 1;
  while (l >= 0) {
    int d = m.link_dof[l];
    if (d >= 0) {
      int g = gidx(m, d);
      V3 a = k.ja[d];
      if (m.link_jtype[l] == 0) {
        V3 lin = cross(a, P - k.jo[d]);
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
void mass_and_bias(const MV& m, const Kin& k, double M[MAXD][MAXD], double* C) {
  int n = m.NDOF;
  for (int i = 0; i < n; i++) {
    C[i] = 0;
    for (int j = 0; j < n; j++) M[i][j] = 0;
  }
  const V3 g = v3(0, 0, (g_flags & 16) ? 0.0 : -PBG_GRAVITY);
  const double kd_lin = (g_flags & 4) ? 0.0 : PBG_LINEAR_DAMPING;
  const double kd_ang = (g_flags & 4) ? 0.0 : PBG_ANGULAR_DAMPING;
  double Jv[3][MAXD], Jw[3][MAXD];
  int nb = m.NL + 1;
  for (int b = 0; b < nb; b++) {
    double mass = b == 0 ? m.base_mass : m.mass[b - 1];
    const double* I6 = b == 0 ? m.base_inertia : m.inertia[b - 1];
    if (b == 0 && !m.floating) continue;
    M3 Iw = world_inertia(k.R[b], I6);
    point_jacobian(m, k, b, k.c[b], Jv, Jw);
    for (int i = 0; i < n; i++) {
      V3 jvi = v3(Jv[0][i], Jv[1][i], Jv[2][i]);
      V3 jwi = v3(Jw[0][i], Jw[1][i], Jw[2][i]);
      V3 Ijwi = mul(Iw, jwi);
      for (int j = 0; j < n; j++) {
        V3 jvj = v3(Jv[0][j], Jv[1][j], Jv[2][j]);
        V3 jwj = v3(Jw[0][j], Jw[1][j], Jw[2][j]);
        M[i][j] += mass * dot(jvi, jvj) + dot(Ijwi, jwj);
      }
    }
    V3 w = k.w[b], v = k.v[b];
    V3 Iw_w = mul(Iw, w);
    V3 f = mass * (k.ac[b] - g) + (mass * (kd_lin + kd_lin * norm(v))) * v;
    V3 tq = mul(Iw, k.al[b]) + cross(w, Iw_w) + (kd_ang + kd_ang * norm(w)) * Iw_w;
    for (int i = 0; i < n; i++) {
      C[i] += Jv[0][i] * f.x + Jv[1][i] * f.y + Jv[2][i] * f.z + Jw[0][i] * tq.x + Jw[1][i] * tq.y + Jw[2][i] * tq.z;
    }
  }
  for (int d = 0; d < m.NJ; d++) M[gidx(m, d)][gidx(m, d)] += m.armature[d];
}

// in-place Cholesky M = L L^T (lower)
void cholesky(int n, double A[MAXD][MAXD]) {
  for (int j = 0; j < n; j++) {
    double s = A[j][j];
    for (int k = 0; k < j; k++) s -= A[j][k] * A[j][k];
    double ljj = sqrt(s);
    A[j][j] = ljj;
    for (int i = j + 1; i < n; i++) {
      double t = A[i][j];
      for (int k = 0; k < j; k++) t -= A[i][k] * A[j][k];
      A[i][j] = t / ljj;
    }
  }
}
void chol_solve(int n, const double L[MAXD][MAXD], const double* b, double* x) {
  double y[MAXD];
  for (int i = 0; i < n; i++) {
    double t = b[i];
    for (int k = 0; k < i; k++) t -= L[i][k] * y[k];
    y[i] = t / L[i][i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double t = y[i];
    for (int k = i + 1; k < n; k++) t -= L[k][i] * x[k];
    x[i] = t / L[i][i];
  }
}

// ------------------------------------------------------------------ contacts + PGS
struct Row {
  double J[MAXD], W[MAXD];
  double meff, target, lo, hi, lambda, mu;
  int normal;  // friction rows: index of their normal row; else -1
};

inline void plane_space(V3 n, V3& p, V3& q) {  // btPlaneSpace1
  if (fabs(n.z) > 0.7071067811865476) {
    double a = n.y * n.y + n.z * n.z, k = 1.0 / sqrt(a);
    p = v3(0, -n.z * k, n.y * k);
    q = v3(a * k, -n.x * p.z, n.x * p.y);
  } else {
    double a = n.x * n.x + n.y * n.y, k = 1.0 / sqrt(a);
    p = v3(-n.y * k, n.x * k, 0);
    q = v3(-n.z * p.y, n.z * p.x, a * k);
  }
}

// closest points between segments p0-p1 and q0-q1
void segment_closest(V3 p0, V3 p1, V3 q0, V3 q1, V3& cp, V3& cq) {
  V3 d1 = p1 - p0, d2 = q1 - q0, r = p0 - q0;
  double a = dot(d1, d1), e = dot(d2, d2), f = dot(d2, r);
  double s, t;
  const double eps = 1e-12;
  if (a <= eps && e <= eps) { s = t = 0; }
  else if (a <= eps) { s = 0; t = fmin(fmax(f / e, 0.0), 1.0); }
  else {
    double c = dot(d1, r);
    if (e <= eps) { t = 0; s = fmin(fmax(-c / a, 0.0), 1.0); }
    else {
      double b = dot(d1, d2), den = a * e - b * b;
      s = den > eps ? fmin(fmax((b * f - c * e) / den, 0.0), 1.0) : 0.0;
      t = (b * s + f) / e;
      if (t < 0) { t = 0; s = fmin(fmax(-c / a, 0.0), 1.0); }
      else if (t > 1) { t = 1; s = fmin(fmax((b - c) / a, 0.0), 1.0); }
    }
  }
  cp = p0 + s * d1;
  cq = q0 + t * d2;
}

struct Contact {
  int body_a, body_b;  // body_b = -1: floor
  V3 pa, pb, n;        // points on A / B, normal pointing from B into A
  double dist, mu;
};

int detect_contacts(const MV& m, const Kin& k, Contact* out, uint8_t* slot_active) {
  int nc = 0;
  for (int s = 0; s < m.NS; s++) {
    int b = m.slot_link[s] + 1;
    V3 c = k.x[b] + mul(k.R[b], v3(m.slot_point[s]));
    double r = m.slot_radius[s];
    double dist = c.z - r;
    slot_active[s] = dist < PBG_CONTACT_THRESHOLD;
    if (slot_active[s]) {
      Contact& ct = out[nc++];
      ct.body_a = b; ct.body_b = -1;
      ct.pa = c - r * v3(0, 0, 1);
      ct.pb = v3(c.x, c.y, 0.0);
      ct.n = v3(0, 0, 1);
      ct.dist = dist; ct.mu = m.slot_mu[s];
    }
  }
  for (int p = 0; p < m.NPAIR; p++) {
    int ba = m.pair_a[p] + 1, bb = m.pair_b[p] + 1;
    V3 a0 = k.x[ba] + mul(k.R[ba], v3(m.pa0[p])), a1 = k.x[ba] + mul(k.R[ba], v3(m.pa1[p]));
    V3 b0 = k.x[bb] + mul(k.R[bb], v3(m.pb0[p])), b1 = k.x[bb] + mul(k.R[bb], v3(m.pb1[p]));
    V3 ca, cb;
    segment_closest(a0, a1, b0, b1, ca, cb);
    V3 dvec = ca - cb;
    double d = norm(dvec);
    double dist = d - m.pra[p] - m.prb[p];
    if (dist < PBG_CONTACT_THRESHOLD) {
      V3 n = d > 1e-9 ? (1.0 / d) * dvec : v3(0, 0, 1);
      Contact& ct = out[nc++];
      ct.body_a = ba; ct.body_b = bb;
      ct.pa = ca - m.pra[p] * n;
      ct.pb = cb + m.prb[p] * n;
      ct.n = n; ct.dist = dist; ct.mu = m.pmu[p];
    }
  }
  return nc;
}

void contact_row_jacobian(const MV& m, const Kin& k, const Contact& c, V3 dir, double* J) {
  double Jv[3][MAXD], Jw[3][MAXD];
  point_jacobian(m, k, c.body_a, c.pa, Jv, Jw);
  for (int j = 0; j < m.NDOF; j++) J[j] = dir.x * Jv[0][j] + dir.y * Jv[1][j] + dir.z * Jv[2][j];
  if (c.body_b >= 0) {
    point_jacobian(m, k, c.body_b, c.pb, Jv, Jw);
    for (int j = 0; j < m.NDOF; j++) J[j] -= dir.x * Jv[0][j] + dir.y * Jv[1][j] + dir.z * Jv[2][j];
  }
}

inline double dotn(int n, const double* a, const double* b) {
  double s = 0;
  for (int i = 0; i < n; i++) s += a[i] * b[i];
  return s;
}

void setup_row(int n, const double L[MAXD][MAXD], const double* nu, Row& r, double pos, int positional, double erp, double dt) {
  chol_solve(n, L, r.J, r.W);
  double D = dotn(n, r.J, r.W);
  r.meff = D > 1e-12 ? 1.0 / D : 0.0;
  double vJ = dotn(n, r.J, nu);
  if (!positional) r.target = 0.0;                        // friction
  else if (pos > 0) r.target = vJ - pos / dt;             // [EXT] Bullet: velocityError = -pen/dt
  else r.target = -erp * pos / dt;                        // Baumgarte push-out
  r.lambda = 0.0;
}

inline void solve_row(int n, Row& r, double* nu) {
  double delta = r.meff * (r.target - dotn(n, r.J, nu));
  double nl = r.lambda + delta;
  if (nl < r.lo) nl = r.lo;
  if (nl > r.hi) nl = r.hi;
  delta = nl - r.lambda;
  r.lambda = nl;
  for (int i = 0; i < n; i++) nu[i] += r.W[i] * delta;
}

inline double clampv(double v) {
  return v > PBG_MAX_COORD_VELOCITY ? PBG_MAX_COORD_VELOCITY : (v < -PBG_MAX_COORD_VELOCITY ? -PBG_MAX_COORD_VELOCITY : v);
}

// ------------------------------------------------------------------ one sub-step
// tau: motor torque on joint dofs, held over the env step (robot_locomotors.py:26-29).
// Returns number of contacts detected; slot_active receives floor-slot flags.
int substep(const MV& m, double* s, const double* tau, uint8_t* slot_active) {
  const double dt = m.dt_sub;
  const int n = m.NDOF;
  static thread_local Kin k;
  static thread_local double M[MAXD][MAXD];
  static thread_local Row rows[MAXROWS];
  static thread_local Contact cts[MAXS + MAXPAIR];
  double C[MAXD], rhs[MAXD], qdd[MAXD], nu[MAXD];
  forward_kinematics(m, s, k);
  mass_and_bias(m, k, M, C);
  // joint damping tau = -d*qd from this sub-step's velocity (explicit; [EXT] pybullet
  // applyJointDamping -- applied per sub-step here, the stable choice at dt/4)
  const double* qd0 = s + PBG_BASE_WORDS + m.NJ;
  for (int i = 0; i < n; i++) rhs[i] = -C[i];
  for (int d = 0; d < m.NJ; d++)
    rhs[gidx(m, d)] += tau[d] - ((g_flags & 8) ? 0.0 : m.damping[d] * qd0[d]);
  cholesky(n, M);
  chol_solve(n, M, rhs, qdd);
  // generalized velocity nu = [v_base, w_base, qd]
  double* q = s + PBG_BASE_WORDS;
  double* qd = q + m.NJ;
  if (m.floating) {
    for (int i = 0; i < 3; i++) { nu[i] = s[7 + i]; nu[3 + i] = s[10 + i]; }
  }
  for (int d = 0; d < m.NJ; d++) nu[gidx(m, d)] = qd[d];
  for (int i = 0; i < n; i++) nu[i] = clampv(nu[i] + dt * qdd[i]);

  // constraint rows, Bullet order: joint limits, contact normals, frictions
  int nr = 0;
  for (int d = 0; d < m.NJ; d++) {
    if (!m.limited[d] || (g_flags & 1)) continue;
    for (int side = 0; side < 2; side++) {
      Row& r = rows[nr++];
      for (int i = 0; i < n; i++) r.J[i] = 0;
      r.J[gidx(m, d)] = side == 0 ? 1.0 : -1.0;
      double pos = side == 0 ? q[d] - m.lower[d] : m.upper[d] - q[d];
      setup_row(n, M, nu, r, pos, 1, PBG_LIMIT_ERP, dt);
      r.lo = 0; r.hi = PBG_LIMIT_MAX_IMPULSE; r.normal = -1;
    }
  }
  int nc = detect_contacts(m, k, cts, slot_active);
  if (g_flags & 2) nc = 0;
  int first_normal = nr;
  for (int c = 0; c < nc; c++) {
    Row& r = rows[nr++];
    contact_row_jacobian(m, k, cts[c], cts[c].n, r.J);
    setup_row(n, M, nu, r, cts[c].dist, 1, PBG_CONTACT_ERP, dt);
    r.lo = 0; r.hi = 1e30; r.normal = -1; r.mu = cts[c].mu;
  }
  int first_friction = nr;
  for (int c = 0; c < nc; c++) {
    V3 t1, t2;
    plane_space(cts[c].n, t1, t2);
    for (int f = 0; f < 2; f++) {
      Row& r = rows[nr++];
      contact_row_jacobian(m, k, cts[c], f == 0 ? t1 : t2, r.J);
      setup_row(n, M, nu, r, 0.0, 0, 0.0, dt);
      r.normal = first_normal + c; r.mu = cts[c].mu; r.lo = r.hi = 0;
    }
  }
  for (int it = 0; it < PBG_SOLVER_ITERATIONS; it++) {
    for (int i = 0; i < first_friction; i++) solve_row(n, rows[i], nu);
    for (int i = first_friction; i < nr; i++) {
      double ln = rows[rows[i].normal].lambda;
      if (ln > 0) {  // [EXT] Bullet solves a friction row only under a positive normal impulse
        rows[i].lo = -rows[i].mu * ln;
        rows[i].hi = rows[i].mu * ln;
        solve_row(n, rows[i], nu);
      }
    }
  }
  for (int i = 0; i < n; i++) nu[i] = clampv(nu[i]);

  // integrate positions (semi-implicit Euler)
  for (int d = 0; d < m.NJ; d++) {
    qd[d] = nu[gidx(m, d)];
    q[d] += dt * qd[d];
  }
  if (m.floating) {
    for (int i = 0; i < 3; i++) { s[7 + i] = nu[i]; s[10 + i] = nu[3 + i]; s[i] += dt * nu[i]; }
    // exponential-map quaternion update with world angular velocity  [EXT] pQuatUpdateFun
    V3 w = v3(s + 10);
    double ang = norm(w);
    if (ang * dt > PBG_ANGULAR_MOTION_THRESHOLD) ang = PBG_ANGULAR_MOTION_THRESHOLD / dt;
    V3 ax;
    if (ang < 0.001) ax = (0.5 * dt - (dt * dt * dt) * 0.020833333333 * ang * ang) * w;
    else ax = (sin(0.5 * ang * dt) / ang) * w;
    double dw = cos(0.5 * ang * dt);
    double* qt = s + 3;
    double x = qt[0], y = qt[1], z = qt[2], ww = qt[3];
    // dq * q (Hamilton, xyzw)
    double nx = dw * x + ax.x * ww + ax.y * z - ax.z * y;
    double ny = dw * y - ax.x * z + ax.y * ww + ax.z * x;
    double nz = dw * z + ax.x * y - ax.y * x + ax.z * ww;
    double nw = dw * ww - ax.x * x - ax.y * y - ax.z * z;
    double inv = 1.0 / sqrt(nx * nx + ny * ny + nz * nz + nw * nw);
    qt[0] = nx * inv; qt[1] = ny * inv; qt[2] = nz * inv; qt[3] = nw * inv;
  }
  return nc;
}

// ------------------------------------------------------------------ pack (numpy-exact)
// numpy pairwise summation (numpy/_core/src/umath/loops_utils.h.src) with the add
// identity 0 as the reduction's initial value; verified bit-exact against numpy 2.2.
double np_sum_f64(const double* a, int n, int stride) {
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; i++) res += a[i * stride];
    return 0.0 + res;
  }
  double r[8];
  for (int j = 0; j < 8; j++) r[j] = a[j * stride];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; j++) r[j] += a[(i + j) * stride];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; i++) res += a[i * stride];
  return 0.0 + res;
}
float np_sum_f32(const float* a, int n) {
  if (n < 8) {
    float res = 0.0f;
    for (int i = 0; i < n; i++) res += a[i];
    return 0.0f + res;
  }
  float r[8];
  for (int j = 0; j < 8; j++) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; j++) r[j] += a[i + j];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; i++) res += a[i];
  return 0.0f + res;
}

// pybullet.getEulerFromQuaternion (pybullet.c), q = (x, y, z, w)  [EXT, restated]
void euler_from_quat(const double* q, double* rpy) {
  double sqx = q[0] * q[0], sqy = q[1] * q[1], sqz = q[2] * q[2], squ = q[3] * q[3];
  rpy[0] = atan2(2 * (q[1] * q[2] + q[3] * q[0]), squ - sqx - sqy + sqz);
  double sarg = -2 * (q[0] * q[2] - q[3] * q[1]);
  rpy[1] = sarg <= -1.0 ? -0.5 * 3.141592538 : (sarg >= 1.0 ? 0.5 * 3.141592538 : asin(sarg));
  rpy[2] = atan2(2 * (q[0] * q[1] + q[3] * q[2]), squ + sqx - sqy - sqz);
}

inline float clip5(float v) { return v < -5.0f ? -5.0f : (v > 5.0f ? 5.0f : v); }  // NaN passes

// Philox4x32-10 (Salmon et al. 2011), as the kernels use it for their random draws.
void philox(uint32_t ctr[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; r++) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0], p1 = (uint64_t)0xCD9E8D57u * ctr[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ ctr[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ ctr[3] ^ k1;
    ctr[1] = (uint32_t)p1; ctr[3] = (uint32_t)p0; ctr[0] = n0; ctr[2] = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}
uint64_t g_seed = 0;
int g_env_offset = 0;

// HumanoidFlagrun walk target (robot_locomotors.py:195-226): flag_reposition draws
// U(+-halflen) x U(+-halfwidth) times 0.5 (here Philox, counter (global env, draw index)).
struct Flag { double tx, ty; int timeout, count; };
void flag_draw(int e, Flag& f) {
  uint32_t c[4] = {(uint32_t)(g_env_offset + e), (uint32_t)f.count, 0xF1A6u, 0x5EEDu};
  philox(c, (uint32_t)g_seed, (uint32_t)(g_seed >> 32));
  const double u0 = (double)(c[0] >> 8) * (1.0 / 16777216.0), u1 = (double)(c[1] >> 8) * (1.0 / 16777216.0);
  f.tx = (-PBG_STADIUM_HALFLEN + 2.0 * PBG_STADIUM_HALFLEN * u0) * PBG_FLAG_COMPACT;
  f.ty = (-PBG_STADIUM_HALFWIDTH + 2.0 * PBG_STADIUM_HALFWIDTH * u1) * PBG_FLAG_COMPACT;
  f.timeout = PBG_FLAG_TIMEOUT;
  f.count++;
}

}  // namespace

extern "C" {

// Pack inputs, i.e. what the reference reads back from pybullet after stepSimulation.
// part_xyz: [n_parts][3] COM positions in `parts` dict order (floor last when present).
typedef struct {
  const double* part_xyz; int n_parts;
  const double* body_quat;   // robot_body orientation (x,y,z,w)
  const double* body_pos;    // robot_body COM position
  const double* body_vel;    // robot_body COM linear velocity
  const double* jq;          // [NO] joint positions of obs joints (ordered_joints order)
  const double* jqd;         // [NO] joint velocities
  const float* feet_prev;    // [NF] feet_contact as of the previous step (goes into obs)
  const uint8_t* feet_new;   // [NF] contact with the floor after this step (nullable: reset)
  const float* act;          // [NA] raw action (nullable: reset)
  double potential_old;
  double initial_z;          // NaN: take it from this calc_state (robot_locomotors.py:44-45)
  double target_x, target_y; // robot.walk_target_x / _y (1e3, 0 except HumanoidFlagrun)
  const double* body_avel;   // base angular velocity (MuJoCo-observation Ant / Humanoid; nullable)
} pbg_pack_in;

typedef struct {
  float* obs; double reward; uint8_t done; double potential; double initial_z;
  float* feet_out;           // [NF]
  double rewards[5];         // alive, progress, electricity, joints_at_limit, feet_collision
  double dist;               // walk_target_dist
  double pitch;              // body_rpy[1]
  int at_limit;              // joints_at_limit
} pbg_pack_out;

void pbg_oracle_set_flags(int flags) { g_flags = flags; }

// Link frames at a state, for tests: R [NL+1][9] row-major, COM [NL+1][3] (base first).
int pbg_oracle_link_frames(int robot, const double* state, double* R_out, double* c_out) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  static thread_local Kin k;
  forward_kinematics(*mp, state, k);
  for (int b = 0; b <= mp->NL; b++) {
    for (int i = 0; i < 9; i++) R_out[9 * b + i] = k.R[b].m[i / 3][i % 3];
    c_out[3 * b] = k.c[b].x; c_out[3 * b + 1] = k.c[b].y; c_out[3 * b + 2] = k.c[b].z;
  }
  return 0;
}

// Link COM velocities / bias accelerations [NL+1][3] each (base first), for tests.
int pbg_oracle_link_vel(int robot, const double* state, double* v, double* w, double* ac, double* al) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  static thread_local Kin k;
  forward_kinematics(*mp, state, k);
  for (int b = 0; b <= mp->NL; b++) {
    V3* src[4] = {&k.v[b], &k.w[b], &k.ac[b], &k.al[b]};
    double* dst[4] = {v, w, ac, al};
    for (int t = 0; t < 4; t++) { dst[t][3 * b] = src[t]->x; dst[t][3 * b + 1] = src[t]->y; dst[t][3 * b + 2] = src[t]->z; }
  }
  return 0;
}

int pbg_oracle_info(int robot, int* out) {
  const MV* m = model(robot);
  if (!m) return -1;
  int v[] = {m->NL, m->NJ, m->NDOF, m->NA, m->NO, m->NR, m->NF, m->NP, m->NS, m->NPAIR, m->OBS,
             PBG_BASE_WORDS + 2 * m->NJ, PBG_AUX_WORDS + m->NF + (m->flagrun ? 4 : 0), m->floating, m->kind,
             m->substeps};
  memcpy(out, v, sizeof(v));
  return 0;
}

static void pendulum_obs(const MV& m, const double* jq, const double* jqd, const double* tip, float* obs,
                         double* rew, uint8_t* done);
static void mujoco_planar_obs(const MV& m, const double* jq, const double* jqd, double x_after, double x_before,
                              const float* act, pbg_pack_out* out);
static void mujoco3d_obs(const MV& m, const pbg_pack_in* in, pbg_pack_out* out);

// Walker pack: calc_state (robot_locomotors.py:31-64) + the reward/done part of
// WalkerBaseBulletEnv._step (gym_locomotion_envs.py:59-114).  With act == NULL only the
// calc_state half runs (reset path).
static int walker_pack_body(const MV& m, const pbg_pack_in* in, pbg_pack_out* out);

int pbg_oracle_pack(int robot, const pbg_pack_in* in, pbg_pack_out* out) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  const MV& m = *mp;
  if (m.kind == 3) {  // MuJoCo Ant / Humanoid: WalkerBase.calc_state side effects, then qpos/qvel obs
    pbg_pack_in w = *in;
    w.act = nullptr;
    walker_pack_body(m, &w, out);
    mujoco3d_obs(m, in, out);
    return 0;
  }
  if (m.kind == 2) {  // MuJoCo planar: jq/jqd all ordered joints, body_pos = robot_body, potential_old = x_before
    mujoco_planar_obs(m, in->jq, in->jqd, in->body_pos[0], in->potential_old, in->act, out);
    return 0;
  }
  if (m.kind == 1) {  // pendulums: jq/jqd = (hinge, [hinge2,] slider), pos = pole2 position
    pendulum_obs(m, in->jq, in->jqd, in->body_pos, out->obs, &out->reward, &out->done);
    if (!in->act) { out->reward = 0; out->done = 0; }
    return 0;
  }
  return walker_pack_body(m, in, out);
}

static int walker_pack_body(const MV& m, const pbg_pack_in* in, pbg_pack_out* out) {
  // joints: np.array([...], dtype=float32) of (pos_rel, vel_scaled) pairs  (robot_bases.py:306-321)
  float j[2 * MAXD];
  for (int i = 0; i < m.NO; i++) {
    int d = m.obs_dof[i];
    double pos = in->jq[i], vel = in->jqd[i];
    if (m.lower[d] < m.upper[d]) {
      double mid = 0.5 * (m.lower[d] + m.upper[d]);
      pos = 2 * (pos - mid) / (m.upper[d] - m.lower[d]);
    }
    vel *= m.obs_vel_scale[i];
    j[2 * i] = (float)pos;
    j[2 * i + 1] = (float)vel;
  }
  int at_limit = 0;
  for (int i = 0; i < m.NO; i++) at_limit += fabsf(j[2 * i]) > PBG_JOINT_AT_LIMIT;
  double bx = np_sum_f64(in->part_xyz + 0, in->n_parts, 3) / (double)in->n_parts;
  double by = np_sum_f64(in->part_xyz + 1, in->n_parts, 3) / (double)in->n_parts;
  double bz = in->body_pos[2];
  double rpy[3];
  euler_from_quat(in->body_quat, rpy);
  double z0 = isnan(in->initial_z) ? bz : in->initial_z;
  double theta = atan2(in->target_y - by, in->target_x - bx);
  double dy = in->target_y - by, dx = in->target_x - bx;
  double dist = sqrt(dy * dy + dx * dx);
  out->dist = dist;
  double ang = theta - rpy[2];
  double cy = cos(-rpy[2]), sy = sin(-rpy[2]);
  double vx = cy * in->body_vel[0] + -sy * in->body_vel[1] + 0.0 * in->body_vel[2];
  double vy = sy * in->body_vel[0] + cy * in->body_vel[1] + 0.0 * in->body_vel[2];
  double vz = 0.0 * in->body_vel[0] + 0.0 * in->body_vel[1] + 1.0 * in->body_vel[2];
  float more[8] = {(float)(bz - z0), (float)sin(ang), (float)cos(ang), (float)(0.3 * vx),
                   (float)(0.3 * vy), (float)(0.3 * vz), (float)rpy[0], (float)rpy[1]};
  int o = 0;
  for (int i = 0; i < 8; i++) out->obs[o++] = clip5(more[i]);
  for (int i = 0; i < 2 * m.NO; i++) out->obs[o++] = clip5(j[i]);
  for (int i = 0; i < m.NF; i++) out->obs[o++] = clip5(in->feet_prev[i]);
  out->initial_z = z0;
  out->pitch = rpy[1];
  out->at_limit = at_limit;
  double dt = m.dt_sub * m.substeps;  // scene.dt = timestep*frame_skip (scene_bases.py:17)
  out->potential = -dist / dt;         // robot_locomotors.py:79
  for (int i = 0; i < m.NF; i++) out->feet_out[i] = in->feet_prev[i];
  if (!in->act) {
    out->reward = 0; out->done = 0;
    return 0;
  }
  // --- _step: alive / done (gym_locomotion_envs.py:61-65)
  float s0 = out->obs[0];
  double alive;
  double pitch = rpy[1];
  switch (m.alive) {
    case 0: {  // Hopper: z (f64) > 0.8 and |pitch| < 1
      double z = (double)s0 + z0;
      alive = (z > 0.8 && fabs(pitch) < 1.0) ? 1.0 : -1.0;
      break;
    }
    case 1:  // HalfCheetah: previous-step feet_contact[1,2,4,5]
      alive = (fabs(pitch) < 1.0 && !(in->feet_prev[1] != 0) && !(in->feet_prev[2] != 0) &&
               !(in->feet_prev[4] != 0) && !(in->feet_prev[5] != 0)) ? 1.0 : -1.0;
      break;
    case 2: {  // Ant: z > 0.26
      double z = (double)s0 + z0;
      alive = z > 0.26 ? 1.0 : -1.0;
      break;
    }
    default: {  // Humanoid: np.float32 + python 0.8 stays float32 (NEP 50); z > 0.78 in f32
      float z = s0 + (float)z0;
      alive = z > 0.78f ? 2.0 : -1.0;
      break;
    }
  }
  uint8_t done = alive < 0;
  for (int i = 0; i < m.OBS; i++) if (isnan(out->obs[i])) done = 1;
  double progress = out->potential - in->potential_old;
  for (int i = 0; i < m.NF; i++) out->feet_out[i] = in->feet_new[i] ? 1.0f : 0.0f;
  // electricity: float32 arithmetic on the float32 action (gym_locomotion_envs.py:82-83)
  float tmp[MAXD];
  for (int i = 0; i < m.NA; i++) tmp[i] = fabsf(in->act[i] * j[2 * i + 1]);
  float mean_e = np_sum_f32(tmp, m.NA) / (float)m.NA;
  for (int i = 0; i < m.NA; i++) tmp[i] = in->act[i] * in->act[i];
  float mean_s = np_sum_f32(tmp, m.NA) / (float)m.NA;
  double elec = m.elec * (double)mean_e;
  elec += m.stall * (double)mean_s;
  double jal = m.jal * (double)at_limit;
  out->rewards[0] = alive; out->rewards[1] = progress; out->rewards[2] = elec;
  out->rewards[3] = jal; out->rewards[4] = 0.0;
  out->reward = ((((0.0 + alive) + progress) + elec) + jal) + 0.0;
  out->done = done;
  return 0;
}

// calc_state with HumanoidFlagrun's bookkeeping (robot_locomotors.py:219-226): timeout
// countdown, pack against the current flag, re-draw and pack again when the target is
// within 1 m or the timeout ran out.  `next` (nullable) replaces the draw (golden tests).
static void flag_pack(int robot, const MV& m, pbg_pack_in* in, pbg_pack_out* out, Flag& f, int e,
                      const double* next) {
  if (!m.flagrun) { pbg_oracle_pack(robot, in, out); return; }
  f.timeout -= 1;
  in->target_x = f.tx; in->target_y = f.ty;
  pbg_oracle_pack(robot, in, out);
  if (out->dist < 1.0 || f.timeout <= 0) {
    if (next) { f.tx = next[0]; f.ty = next[1]; f.timeout = PBG_FLAG_TIMEOUT; f.count++; }
    else flag_draw(e, f);
    in->target_x = f.tx; in->target_y = f.ty;
    pbg_oracle_pack(robot, in, out);
  }
}
static Flag load_flag(const MV& m, const double* a) {
  Flag f = {0.0, 0.0, 0, 0};
  if (m.flagrun) { f.tx = a[4 + m.NF]; f.ty = a[5 + m.NF]; f.timeout = (int)a[6 + m.NF]; f.count = (int)a[7 + m.NF]; }
  return f;
}
static void store_flag(const MV& m, double* a, const Flag& f) {
  if (m.flagrun) { a[4 + m.NF] = f.tx; a[5 + m.NF] = f.ty; a[6 + m.NF] = f.timeout; a[7 + m.NF] = f.count; }
}

// Flag RNG of the kernels: Philox key = seed, env ids offset by env_offset.
void pbg_oracle_set_rng(uint64_t seed, int env_offset) { g_seed = seed; g_env_offset = env_offset; }

// Golden-vector form: flag_in = [target x, y, flag_timeout, next draw x, y],
// flag_out = [target x, y, flag_timeout] after the calc_state.
int pbg_oracle_pack_flag(int robot, const pbg_pack_in* in, pbg_pack_out* out, const double* flag_in,
                         double* flag_out) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  pbg_pack_in in2 = *in;
  Flag f = {flag_in[0], flag_in[1], (int)flag_in[2], 0};
  flag_pack(robot, *mp, &in2, out, f, 0, flag_in + 3);
  flag_out[0] = f.tx; flag_out[1] = f.ty; flag_out[2] = f.timeout;
  return 0;
}

// MuJoCo-observation planar walkers (mujoco robot_locomotors.py:93-196, mujoco
// gym_locomotion_envs.py:121-252): obs float32 [qpos[1:], clip(qvel, +-10)] (HalfCheetah
// unclipped) over every ordered joint incl. the ignored root joints; potential =
// (x_after - x_before) / dt; reward = sum([potential, 1.0, c * sum(a^2) (float32)]).
static void mujoco_planar_obs(const MV& m, const double* jq, const double* jqd, double x_after, double x_before,
                              const float* act, pbg_pack_out* out) {
  const float c = (float)m.qvel_clip;
  int o = 0;
  for (int i = 1; i < m.NO; i++) out->obs[o++] = (float)jq[i];
  for (int i = 0; i < m.NO; i++) {
    const float v = (float)jqd[i];
    out->obs[o++] = c > 0.f ? (v < -c ? -c : (v > c ? c : v)) : v;
  }
  out->potential = x_after; out->initial_z = 0.0; out->dist = 0.0;
  for (int i = 0; i < 5; i++) out->rewards[i] = 0.0;
  if (!act) { out->reward = 0.0; out->done = 0; return; }
  const double potential = (x_after - x_before) / (m.dt_sub * m.substeps);
  float sq[MAXD];
  for (int i = 0; i < m.NA; i++) sq[i] = act[i] * act[i];
  const float power_cost = (float)m.power_cost * np_sum_f32(sq, m.NA);
  bool finite = true, small = true;
  for (int i = 0; i < m.OBS; i++) {
    finite = finite && isfinite(out->obs[i]);
    if (i >= 2) small = small && fabsf(out->obs[i]) < 100.f;
  }
  const float h = out->obs[0], ang = out->obs[1];
  if (m.alive == 12) {
    out->reward = (0.0 + potential) + (double)power_cost;
    out->done = 0;
  } else {
    out->reward = ((0.0 + potential) + 1.0) + (double)power_cost;
    out->done = m.alive == 10 ? !(finite && small && h > -0.3f && fabsf(ang) < 0.2f)
                              : !(finite && small && (1.0f > h && h > -0.2f) && (-1.0f < ang && ang < 1.0f));
  }
}

// MuJoCo-observation Ant / Humanoid (mujoco robot_locomotors.py:210-319, mujoco
// gym_locomotion_envs.py:53-114): obs [z, quat, joint q, v, w, joint qd, zeros] (float64 in
// the reference), reward sum([alive(state[0] + initial_z), progress, -0.1 at_limit, 0]).
static void mujoco3d_obs(const MV& m, const pbg_pack_in* in, pbg_pack_out* out) {
  double st[5 + 2 * MAXD + 6];
  int o = 0;
  st[o++] = in->body_pos[2];
  for (int i = 0; i < 4; i++) st[o++] = in->body_quat[i];
  for (int i = 0; i < m.NO; i++) st[o++] = in->jq[i];
  for (int i = 0; i < 3; i++) st[o++] = in->body_vel[i];
  for (int i = 0; i < 3; i++) st[o++] = in->body_avel ? in->body_avel[i] : 0.0;
  for (int i = 0; i < m.NO; i++) st[o++] = in->jqd[i];
  bool finite = true;
  for (int i = 0; i < o; i++) { out->obs[i] = (float)st[i]; finite = finite && isfinite(st[i]); }
  for (int i = o; i < m.OBS; i++) out->obs[i] = 0.f;
  for (int i = 0; i < m.NF; i++) out->feet_out[i] = in->feet_new ? (in->feet_new[i] ? 1.f : 0.f) : in->feet_prev[i];
  for (int i = 0; i < 5; i++) out->rewards[i] = 0.0;
  if (!in->act) { out->reward = 0.0; out->done = 0; return; }
  const double z = st[0] + out->initial_z;
  const double alive = m.alive == 2 ? (z > 0.26 ? 1.0 : -1.0) : (z > 0.78 ? 2.0 : -1.0);
  out->done = alive < 0 || !finite;
  const double progress = out->potential - in->potential_old;
  const double jal = -0.1 * (double)out->at_limit;
  out->rewards[0] = alive; out->rewards[1] = progress; out->rewards[2] = jal;  // [alive, progress, jal, 0]
  out->reward = (((0.0 + alive) + progress) + jal) + 0.0;
}

// Pendulum packs: calc_state + reward/done.  obs is float64 in the reference; written here
// as float32 (the C-ABI's obs dtype).
//  * InvertedPendulum / Swingup (robot_pendula.py:27-51, gym_pendulum_envs.py:26-39): non-finite
//    vx / theta / theta_dot are replaced by 0 (:32-46); balance: reward 1, done |theta| > .2;
//    swingup: reward cos(theta), never done.
//  * InvertedDoublePendulum (robot_pendula.py:76-88, gym_pendulum_envs.py:69-80): obs
//    [x, vx, pole2 x, cos th, sin th, th', cos g, sin g, g']; reward = sum([10, -dist_penalty, -0]),
//    dist_penalty = 0.01 x2^2 + (y2 + 0.3 - 2)^2 with (x2, _, y2) = pole2.pose().xyz();
//    done = y2 + 0.3 <= 1.
static void pendulum_obs(const MV& m, const double* jq, const double* jqd, const double* tip, float* obs,
                         double* rew, uint8_t* done) {
  if (m.alive == 7) {  // MuJoCo obs (mujoco robot_pendula.py:75-89, mujoco gym_pendulum_envs.py:60-72)
    const double th = jq[0], thd = jqd[0], g = jq[1], gd = jqd[1], x = jq[2], vx = jqd[2];
    const double px = tip[0], py = tip[2];
    auto clip10 = [](double v) { return v < -10.0 ? -10.0 : (v > 10.0 ? 10.0 : v); };
    const double o[11] = {x, sin(th), sin(g), cos(th), cos(g), clip10(vx), clip10(thd), clip10(gd), 0.0, 0.0, 0.0};
    for (int i = 0; i < 11; i++) obs[i] = (float)o[i];
    const double dist_penalty = 0.01 * (px * px) + ((py + 0.3) - 2) * ((py + 0.3) - 2);
    const double vel_penalty = 1e-3 * (thd * thd) + 5e-3 * (gd * gd);
    if (rew) *rew = ((0.0 + 10.0) + -dist_penalty) + -vel_penalty;
    if (done) *done = py + 0.3 <= 1;
    return;
  }
  if (m.alive == 6) {
    const double th = jq[0], thd = jqd[0], g = jq[1], gd = jqd[1], x = jq[2], vx = jqd[2];
    const double px = tip[0], py = tip[2];
    const double o[9] = {x, vx, px, cos(th), sin(th), thd, cos(g), sin(g), gd};
    for (int i = 0; i < 9; i++) obs[i] = (float)o[i];
    const double dist_penalty = 0.01 * (px * px) + ((py + 0.3) - 2) * ((py + 0.3) - 2);
    if (rew) *rew = ((0.0 + 10.0) + -dist_penalty) + 0.0;
    if (done) *done = py + 0.3 <= 1;
    return;
  }
  double theta = jq[0], theta_dot = jqd[0], x = jq[1], vx = jqd[1];
  if (!isfinite(vx)) vx = 0.0;
  if (!isfinite(theta)) theta = 0.0;
  if (!isfinite(theta_dot)) theta_dot = 0.0;
  obs[0] = (float)x; obs[1] = (float)vx; obs[2] = (float)cos(theta); obs[3] = (float)sin(theta);
  obs[4] = (float)theta_dot;
  if (rew) *rew = m.alive == 5 ? cos(theta) : 1.0;
  if (done) *done = m.alive == 5 ? 0 : fabs(theta) > 0.2;
}
static void pendulum_pack(const MV& m, const double* s, float* obs, double* rew, uint8_t* done) {
  const double* q = s + PBG_BASE_WORDS;
  const double* qd = q + m.NJ;
  double jq[MAXD], jqd[MAXD], tip[3] = {0, 0, 0};
  for (int i = 0; i < m.NO; i++) { jq[i] = q[m.obs_dof[i]]; jqd[i] = qd[m.obs_dof[i]]; }
  if (m.tip_link >= 0) {
    static thread_local Kin k;
    forward_kinematics(m, s, k);
    const V3 c = k.c[m.tip_link + 1];
    tip[0] = c.x; tip[1] = c.y; tip[2] = c.z;
  }
  pendulum_obs(m, jq, jqd, tip, obs, rew, done);
}

// MuJoCo planar pack from a physical state; returns x_after (robot_body COM x).
static double mujoco_planar_pack(const MV& m, const double* s, double x_before, const float* act, float* obs,
                                 double* rew, uint8_t* done) {
  const double* q = s + PBG_BASE_WORDS;
  const double* qd = q + m.NJ;
  double jq[MAXD], jqd[MAXD];
  for (int i = 0; i < m.NO; i++) { jq[i] = q[m.obs_dof[i]]; jqd[i] = qd[m.obs_dof[i]]; }
  static thread_local Kin k;
  forward_kinematics(m, s, k);
  const double x_after = k.c[m.robot_body + 1].x;
  float feet[8];
  pbg_pack_out out;
  out.obs = obs; out.feet_out = feet;
  mujoco_planar_obs(m, jq, jqd, x_after, x_before, act, &out);
  if (rew) *rew = out.reward;
  if (done) *done = out.done;
  return x_after;
}

// Gather the pack inputs from a physical state.
static void gather(const MV& m, const double* s, const double* aux, Kin& k, double* part_xyz,
                   int& n_parts, double* quat, double* pos, double* vel, double* jq, double* jqd) {
  forward_kinematics(m, s, k);
  n_parts = 0;
  for (int p = 0; p < m.NP; p++) {
    V3 c = k.c[m.part_link[p] + 1];
    part_xyz[3 * n_parts] = c.x; part_xyz[3 * n_parts + 1] = c.y; part_xyz[3 * n_parts + 2] = c.z;
    n_parts++;
  }
  if (m.floor && aux[3] != 0.0) {  // gym_locomotion_envs.py:30-31: floor joins robot.parts
    part_xyz[3 * n_parts] = part_xyz[3 * n_parts + 1] = part_xyz[3 * n_parts + 2] = 0.0;
    n_parts++;
  }
  int b = m.robot_body + 1;
  m3_to_quat(k.R[b], quat);
  pos[0] = k.c[b].x; pos[1] = k.c[b].y; pos[2] = k.c[b].z;
  vel[0] = k.v[b].x; vel[1] = k.v[b].y; vel[2] = k.v[b].z;
  const double* q = s + PBG_BASE_WORDS;
  for (int i = 0; i < m.NO; i++) { jq[i] = q[m.obs_dof[i]]; jqd[i] = q[m.NJ + m.obs_dof[i]]; }
}

// Reset envs to the load snapshot with the given ordered-joint positions qinit[n][NR]
// (gym_locomotion_envs.py:22-39, robot_locomotors.py:16-24).  Writes the reset obs.
int pbg_oracle_reset(int robot, int n, double* state, double* aux, const double* qinit, float* obs) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  const MV& m = *mp;
  int SD = PBG_BASE_WORDS + 2 * m.NJ, AD = PBG_AUX_WORDS + m.NF + (m.flagrun ? 4 : 0);
  for (int e = 0; e < n; e++) {
    double* s = state + (size_t)e * SD;
    double* a = aux + (size_t)e * AD;
    for (int i = 0; i < 3; i++) s[i] = m.base_pos[i];
    for (int i = 0; i < 4; i++) s[3 + i] = m.base_quat[i];
    for (int i = 7; i < PBG_BASE_WORDS + 2 * m.NJ; i++) s[i] = 0.0;
    // robot_pendula.py:16 (swingup: 3.1415 + u)
    for (int r = 0; r < m.NR; r++) s[PBG_BASE_WORDS + m.reset_dof[r]] = m.reset_offset[r] + qinit[(size_t)e * m.NR + r];
    float* ob = obs + (size_t)e * m.OBS;
    a[2] = 0.0;
    for (int i = 0; i < m.NF; i++) a[4 + i] = 0.0;
    if (m.kind == 1) { pendulum_pack(m, s, ob, nullptr, nullptr); a[3] = 1.0; continue; }
    if (m.kind == 2) { a[0] = mujoco_planar_pack(m, s, 0.0, nullptr, ob, nullptr, nullptr); a[3] = 1.0; continue; }
    static thread_local Kin k;
    double part_xyz[3 * (MAXL + 2)], quat[4], pos[3], vel[3], jq[MAXD], jqd[MAXD];
    int n_parts;
    gather(m, s, a, k, part_xyz, n_parts, quat, pos, vel, jq, jqd);
    float feet_prev[8] = {0}, feet_out[8];
    pbg_pack_in in = {part_xyz, n_parts, quat, pos, vel, jq, jqd, feet_prev, nullptr, nullptr, 0.0,
                      m.z0fixed, PBG_WALK_TARGET_X, PBG_WALK_TARGET_Y, s + 10};
    pbg_pack_out out;
    out.obs = ob; out.feet_out = feet_out;
    Flag fl = load_flag(m, a);
    if (m.flagrun) flag_draw(e, fl);  // robot_specific_reset -> flag_reposition (:199-201)
    flag_pack(robot, m, &in, &out, fl, e, nullptr);
    store_flag(m, a, fl);
    a[0] = out.potential;
    a[1] = out.initial_z;
    a[3] = 1.0;  // the floor is in robot.parts from now on
  }
  return 0;
}

// One env step for each of n envs: apply_action, stepSimulation (substeps), pack.
// ncontact (nullable): contacts detected in the last sub-step, per env.
int pbg_oracle_step(int robot, int n, double* state, double* aux, const float* act, float* obs,
                    double* rew, uint8_t* done, int32_t* ncontact, int nthreads) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  const MV& m = *mp;
  int SD = PBG_BASE_WORDS + 2 * m.NJ, AD = PBG_AUX_WORDS + m.NF + (m.flagrun ? 4 : 0);
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static)
  for (int e = 0; e < n; e++) {
    double* s = state + (size_t)e * SD;
    double* a = aux + (size_t)e * AD;
    const float* ac = act + (size_t)e * m.NA;
    double tau[MAXD];
    for (int d = 0; d < m.NJ; d++) tau[d] = 0.0;
    for (int i = 0; i < m.NA; i++) {                                  // robot_locomotors.py:26-29
      float c = ac[i] < -1.0f ? -1.0f : (ac[i] > 1.0f ? 1.0f : ac[i]);
      tau[m.act_dof[i]] += m.act_gain[i] * (double)c;
    }
    uint8_t slot_active[MAXS];
    int nc = 0;
    for (int sub = 0; sub < m.substeps; sub++) nc = substep(m, s, tau, slot_active);
    if (ncontact) ncontact[e] = nc;
    a[2] += 1.0;
    float* ob = obs + (size_t)e * m.OBS;
    if (m.kind == 1) { pendulum_pack(m, s, ob, rew + e, done + e); continue; }
    if (m.kind == 2) { a[0] = mujoco_planar_pack(m, s, a[0], ac, ob, rew + e, done + e); continue; }
    uint8_t feet_new[8];
    for (int f = 0; f < m.NF; f++) {
      feet_new[f] = 0;
      for (int sl = 0; sl < m.NS; sl++)
        if (m.slot_link[sl] == m.foot_link[f] && slot_active[sl]) feet_new[f] = 1;
    }
    static thread_local Kin k;
    double part_xyz[3 * (MAXL + 2)], quat[4], pos[3], vel[3], jq[MAXD], jqd[MAXD];
    int n_parts;
    gather(m, s, a, k, part_xyz, n_parts, quat, pos, vel, jq, jqd);
    float feet_prev[8], feet_out[8];
    for (int f = 0; f < m.NF; f++) feet_prev[f] = (float)a[4 + f];
    pbg_pack_in in = {part_xyz, n_parts, quat, pos, vel, jq, jqd, feet_prev, feet_new, ac,
                      a[0], a[1], PBG_WALK_TARGET_X, PBG_WALK_TARGET_Y, s + 10};
    pbg_pack_out out;
    out.obs = ob; out.feet_out = feet_out;
    Flag fl = load_flag(m, a);
    flag_pack(robot, m, &in, &out, fl, e, nullptr);
    store_flag(m, a, fl);
    rew[e] = out.reward;
    done[e] = out.done;
    a[0] = out.potential;
    for (int f = 0; f < m.NF; f++) a[4 + f] = feet_out[f];
  }
  return 0;
}

// Joint-space dynamics at a state, for tests: M (NDOF x NDOF, row-major) and bias C.
int pbg_oracle_dynamics(int robot, const double* state, double* M_out, double* C_out) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  static thread_local Kin k;
  static thread_local double M[MAXD][MAXD];
  forward_kinematics(*mp, state, k);
  mass_and_bias(*mp, k, M, C_out);
  for (int i = 0; i < mp->NDOF; i++)
    for (int j = 0; j < mp->NDOF; j++) M_out[i * mp->NDOF + j] = M[i][j];
  return 0;
}

// Link COM world positions [NL+1][3] (base first) at a state, for tests.
int pbg_oracle_link_com(int robot, const double* state, double* out) {
  const MV* mp = model(robot);
  if (!mp) return -1;
  static thread_local Kin k;
  forward_kinematics(*mp, state, k);
  for (int b = 0; b <= mp->NL; b++) { out[3 * b] = k.c[b].x; out[3 * b + 1] = k.c[b].y; out[3 * b + 2] = k.c[b].z; }
  return 0;
}

}  // extern "C"
