// pbg_step.hip -- batched locomotion-env step on MI355X (gfx950).
//
// Replaces, for N envs at once, the reference's per-env hot path
//   WalkerBaseBulletEnv._step (pybulletgym/envs/roboschool/gym_locomotion_envs.py:54-114)
//     -> robot.apply_action            (robot_locomotors.py:26-29; Humanoid :185-189)
//     -> scene.global_step -> World.step -> pybullet.stepSimulation  (scene_bases.py:47-52,75-76)
//     -> robot.calc_state / calc_potential / alive_bonus / feet contacts / costs  (:59-114)
// and the reset path WalkerBaseBulletEnv._reset (gym_locomotion_envs.py:22-39).
//
// Design: one lane per env, robot topology baked in at compile time
// (template on the generated tables of models_gen.h, every link/dof loop unrolled so
// link state stays in VGPRs), struct-of-arrays float32 state in HBM ([word][env],
// coalesced), float64 only for the numpy-exact observation/reward pack and the
// potential.  Physics per sub-step: joint-space Featherstone dynamics (composite
// rigid-body mass matrix about a robot-local reference point + recursive Newton-Euler
// bias), sparsity-preserving Cholesky (leaf-first dof order, no fill-in), Bullet-style
// sequential-impulse PGS run in Cholesky-transformed velocity space u = L^T nu (one
// vector per constraint row), semi-implicit Euler.  Same algorithm as the CPU oracle
// (oracle/pbg_oracle.cpp), which is the parity reference.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "models_gen.h"
#include "pbg_math.h"
#include "pbg_records.h"
#include "pbg_types.h"
#include "sim_params.h"

namespace pbg {

// Scheduling fence between phases: keeps the scheduler from interleaving whole phases
// (which stretches live ranges past the register file).
#ifndef PBG_NO_PHASE_BARRIERS
#define PBG_PHASE_BARRIER __builtin_amdgcn_sched_barrier(0);
#else
#define PBG_PHASE_BARRIER
#endif

// Diagnostic build only (-DPBG_STAMPS): per-phase wave-cycle sums (s_memtime), summed over
// waves into g_stamps by lane 0.  Never compiled into the product library.
#ifdef PBG_STAMPS
__device__ unsigned long long g_stamps[16];
#define STAMP_DECL unsigned long long _st_t = __builtin_amdgcn_s_memtime(), _st_acc[16] = {0};
#define STAMP(i) { __builtin_amdgcn_sched_barrier(0); unsigned long long _n = __builtin_amdgcn_s_memtime(); _st_acc[i] += _n - _st_t; _st_t = _n; __builtin_amdgcn_sched_barrier(0); }
#define STAMP_FLUSH if ((threadIdx.x & 63) == 0) { for (int _i = 0; _i < 16; _i++) atomicAdd(&g_stamps[_i], _st_acc[_i]); }
#define STAMPX(i) STAMP(i)  // finer split, diagnostic build only (no phase barrier in the product)
#else
#define STAMP_DECL
#define STAMP(i) PBG_PHASE_BARRIER
#define STAMPX(i)
#define STAMP_FLUSH
#endif

// ------------------------------------------------------------------ compile-time model facts
template <int A, int B>
struct BoolTab {
  bool v[A][B];
};
template <int A, int B>
struct FloatTab {
  float v[A][B];
};
template <int A, int B>
struct IntTab {
  int v[A][B];
};

// any joint spring (mjcf.py B7)?  Robots without one compile no spring term at all.
template <class R>
constexpr bool has_springs() {
  for (int d = 0; d < R::NJ; d++)
    if (R::dof_stiffness[d] != 0.0) return true;
  return false;
}

template <class R>
struct Dims {
  static constexpr int NL = R::NL, NJ = R::NJ, NB = R::NL + 1, NDOF = R::NDOF;
  static constexpr int SD = PBG_STATE_WORDS(R::NJ, R::harder);
  // contact capacity: floor slots, self pairs (+ HumanoidFlagrunHarder's cube: 8 corners, NCG geoms)
  static constexpr int NC = R::NS + R::NPAIR + (R::harder ? 8 + R::NCG : 0);
  // constraint-row length: the robot's generalized velocity (+ the cube's 6 in u-space)
  static constexpr int NY = R::NDOF + (R::harder ? 6 : 0);
  static constexpr int count_limited() {
    int c = 0;
    for (int d = 0; d < R::NJ; d++) c += R::dof_limited[d];
    return c;
  }
  static constexpr int NLIM = count_limited();
  // GPU generalized-velocity order: joint dofs leaf-first (reverse preorder), base last.
  static constexpr int gj(int d) { return NJ - 1 - d; }
  static constexpr int gb(int k) { return NJ + k; }
  // generalized index -> joint dof (or -1 for a base dof)
  static constexpr int dof_of(int g) { return g < NJ ? NJ - 1 - g : -1; }
  // joint dof d moves link l
  static constexpr bool moves_(int d, int l) { return l >= 0 && ((R::link_chain_mask[l] >> d) & 1u); }
  static constexpr bool coupled_(int i, int k) {
    int di = dof_of(i), dk = dof_of(k);
    if (di < 0 || dk < 0) return true;
    return moves_(di, R::dof_link[dk]) || moves_(dk, R::dof_link[di]);
  }
  static constexpr bool in_chain_(int g, int l) {
    int d = dof_of(g);
    if (d < 0) return true;
    return moves_(d, l);
  }
  static constexpr double body_mass(int b) { return b == 0 ? (R::floating ? R::base_mass : 0.0) : R::link_mass[b - 1]; }
  static constexpr bool anc_or_self_(int a, int b) {
    return a == b || a == 0 || (a > 0 && b > 0 && ((R::link_anc_mask[b - 1] >> (a - 1)) & 1u));
  }
  // ---- lookup tables, built at compile time (plain constant-array loads after unrolling;
  // a constexpr *function* with loops is not reliably folded in device code)
  static constexpr BoolTab<NDOF, NDOF> make_coupled() {
    BoolTab<NDOF, NDOF> t{};
    for (int i = 0; i < NDOF; i++)
      for (int k = 0; k < NDOF; k++) t.v[i][k] = coupled_(i, k);
    return t;
  }
  static constexpr BoolTab<NDOF, NB> make_in_chain() {
    BoolTab<NDOF, NB> t{};
    for (int i = 0; i < NDOF; i++)
      for (int l = -1; l < NL; l++) t.v[i][l + 1] = in_chain_(i, l);
    return t;
  }
  static constexpr BoolTab<NB, NB> make_anc() {
    BoolTab<NB, NB> t{};
    for (int a = 0; a < NB; a++)
      for (int b = 0; b < NB; b++) t.v[a][b] = anc_or_self_(a, b);
    return t;
  }
  static constexpr int count_nnz() {
    int c = 0;
    for (int i = 0; i < NDOF; i++)
      for (int k = 0; k <= i; k++) c += coupled_(i, k);
    return c;
  }
  static constexpr int NNZ = count_nnz();
  static constexpr IntTab<NDOF, NDOF> make_lidx() {
    IntTab<NDOF, NDOF> t{};
    int c = 0;
    for (int a = 0; a < NDOF; a++)
      for (int b = 0; b < NDOF; b++) t.v[a][b] = NNZ;
    for (int a = 0; a < NDOF; a++)
      for (int b = 0; b <= a; b++)
        if (coupled_(a, b)) t.v[a][b] = c++;
    return t;
  }
  static constexpr BoolTab<NDOF, NDOF> COUPLED = make_coupled();
  static constexpr BoolTab<NDOF, NB> IN_CHAIN = make_in_chain();
  static constexpr BoolTab<NB, NB> ANC = make_anc();
  static constexpr IntTab<NDOF, NDOF> LIDX = make_lidx();
  // generalized indices i, k coupled in M (one's link is an ancestor-or-self of the other's)
  static constexpr bool coupled(int i, int k) { return COUPLED.v[i][k]; }
  // generalized index g enters the Jacobian of a point on link l (-1 = base)
  static constexpr bool in_chain(int g, int l) { return IN_CHAIN.v[g][l + 1]; }
  // body a is body b or an ancestor of it (0 = base)
  static constexpr bool anc_or_self(int a, int b) { return ANC.v[a][b]; }
  static constexpr int lidx(int i, int k) { return LIDX.v[i][k]; }
  // reference point body: base COM (floating) or the robot_body link COM (fixed base)
  static constexpr int REF_BODY = R::floating ? 0 : R::robot_body + 1;
  // body b owns a composite: the floating base, or a link carrying a joint dof
  // body-frame inertia (xx, yy, zz, xy, xz, yz) of body b by value: a pointer into the
  // model table is loaded at run time
  struct Inertia6 { double v[6]; };
  template <int b>
  static constexpr Inertia6 inertia() {
    Inertia6 I{};
    for (int i = 0; i < 6; i++) I.v[i] = b == 0 ? R::base_inertia[i] : R::link_inertia[b > 0 ? b - 1 : 0][i];
    return I;
  }
  // squared (2 x bounding distance) per self-collision pair, for the broad phase
  static constexpr FloatTab<(R::NPAIR > 0 ? R::NPAIR : 1), 1> make_pair_bound() {
    FloatTab<(R::NPAIR > 0 ? R::NPAIR : 1), 1> t{};
    for (int pp = 0; pp < R::NPAIR; pp++) {
      const int ga = R::pair_ga[pp], gb = R::pair_gb[pp];
      double ha = 0, hb = 0;
      for (int c = 0; c < 3; c++) {
        ha += (R::geom_p1[ga][c] - R::geom_p0[ga][c]) * (R::geom_p1[ga][c] - R::geom_p0[ga][c]);
        hb += (R::geom_p1[gb][c] - R::geom_p0[gb][c]) * (R::geom_p1[gb][c] - R::geom_p0[gb][c]);
      }
      // sqrt by Newton (constexpr); generous margin keeps the cull conservative in float32
      auto csqrt = [](double x) { double r = x > 1 ? x : 1; for (int i = 0; i < 60; i++) r = 0.5 * (r + x / r); return x > 0 ? r : 0.0; };
      const double bound = 0.5 * csqrt(ha) + 0.5 * csqrt(hb) + R::geom_r[ga] + R::geom_r[gb] + PBG_CONTACT_THRESHOLD + 0.01;
      t.v[pp][0] = (float)(4.0 * bound * bound);
    }
    return t;
  }
  static constexpr FloatTab<(R::NPAIR > 0 ? R::NPAIR : 1), 1> PAIR_BOUND2 = make_pair_bound();
  static constexpr bool is_owner(int b) { return b == 0 ? R::floating : R::link_dof[b - 1] >= 0; }
  // every body with mass comes after the reference body in DFS order (O is set first)
  static constexpr bool ref_first() {
    for (int b = 0; b < REF_BODY; b++)
      if (body_mass(b) > 0.0) return false;
    return true;
  }
  static_assert(ref_first(), "massive body before the reference body");
  // ---- joint-limit rows: limited dofs in dof order, sparse pattern of y = L^-1 e_g
  static constexpr IntTab<(NLIM > 0 ? NLIM : 1), NDOF + 3> make_lim() {
    // row li: [0] dof, [1] pattern size, [2] LDS word offset, [3..] generalized indices
    IntTab<(NLIM > 0 ? NLIM : 1), NDOF + 3> t{};
    int li = 0, off = 0;
    for (int d = 0; d < NJ; d++) {
      if (!R::dof_limited[d]) continue;
      const int g = gj(d);
      int np = 0;
      for (int i = g; i < NDOF; i++)
        if (coupled_(i, g)) t.v[li][3 + np++] = i;
      t.v[li][0] = d;
      t.v[li][1] = np;
      t.v[li][2] = off;
      off += np + 5;  // y | meff | target_lo | target_hi | lambda_lo | lambda_hi
      li++;
    }
    return t;
  }
  static constexpr IntTab<(NLIM > 0 ? NLIM : 1), NDOF + 3> LIM = make_lim();
  static constexpr int limw() {
    int w = 0;
    for (int li = 0; li < NLIM; li++) w += LIM.v[li][1] + 5;
    return w;
  }
  static constexpr int LIMW = limw();
  // pattern membership / position by generalized index (fixed-trip loops unroll reliably)
  static constexpr IntTab<(NLIM > 0 ? NLIM : 1), NDOF> make_limpos() {
    IntTab<(NLIM > 0 ? NLIM : 1), NDOF> t{};
    for (int li = 0; li < (NLIM > 0 ? NLIM : 1); li++)
      for (int i = 0; i < NDOF; i++) t.v[li][i] = -1;
    for (int li = 0; li < NLIM; li++)
      for (int j = 0; j < LIM.v[li][1]; j++) t.v[li][LIM.v[li][3 + j]] = j;
    return t;
  }
  static constexpr IntTab<(NLIM > 0 ? NLIM : 1), NDOF> LIMPOS = make_limpos();
};

// ------------------------------------------------------------------ state record in registers
// HumanoidFlagrunHarder's cube: a second free body (words after the robot's, sim_params.h)
template <class T>
struct CubeState {
  T p[3], q[4], v[3], w[3];
};
struct NoCube {};
template <class R>
struct State {
  using T = real_t<R>;
  T bp[3], bq[4], bv[3], bw[3];
  T q[R::NJ > 0 ? R::NJ : 1], qd[R::NJ > 0 ? R::NJ : 1];
  std::conditional_t<(R::harder != 0), CubeState<T>, NoCube> cube;
};

// The handle's state / initial_z buffers and scene in R's precision (pbg_types.h real_t)
template <class R>
PBG_DEV real_t<R>* st_of(const Buffers& B) { return static_cast<real_t<R>*>(B.st); }
template <class R>
PBG_DEV real_t<R>* z0_of(const Buffers& B) { return static_cast<real_t<R>*>(B.z0); }
template <class R>
PBG_DEV const SimPT<real_t<R>>& sp_of(const Buffers& B) {
  if constexpr (std::is_same<real_t<R>, double>::value) return B.sp64;
  else return B.sp;
}
// precision-generic libm pieces (float: the f-suffixed calls the float32 kernels always made)
PBG_DEV float tabs(float x) { return fabsf(x); }
PBG_DEV double tabs(double x) { return fabs(x); }
template <class S>
PBG_DEV S tmin(S a, nd<S> b) {
  if constexpr (std::is_same<S, float>::value) return fminf(a, b);
  else return fmin(a, b);
}
template <class S>
PBG_DEV S tmax(S a, nd<S> b) {
  if constexpr (std::is_same<S, float>::value) return fmaxf(a, b);
  else return fmax(a, b);
}
PBG_DEV float tsqrt(float x) { return sqrtf(x); }
PBG_DEV double tsqrt(double x) { return sqrt(x); }

// XCD-aware block order for the step kernels: the dispatcher deals workgroups round-robin over the
// 8 XCDs (workgroup b -> XCD b % 8), each with its own L2, so consecutive env blocks -- which share
// the 128-byte lines of every SoA word (16 envs = 64 bytes) -- landed on different XCDs and each
// fetched the whole line.  Block b processes env block (b % 8) * (G / 8) + b / 8: every XCD walks
// one contiguous range of env blocks (a permutation when G % 8 == 0; identity otherwise).
PBG_DEV int xcd_block() {
  const int G = (int)gridDim.x, b = (int)blockIdx.x;
  if (G & 7) return b;
  return (b & 7) * (G >> 3) + (b >> 3);
}

template <class R>
PBG_DEV void load_state(State<R>& s, const real_t<R>* __restrict__ st, int n, int e) {
#pragma unroll
  for (int i = 0; i < 3; i++) s.bp[i] = st[(size_t)i * n + e];
#pragma unroll
  for (int i = 0; i < 4; i++) s.bq[i] = st[(size_t)(3 + i) * n + e];
#pragma unroll
  for (int i = 0; i < 3; i++) s.bv[i] = st[(size_t)(7 + i) * n + e];
#pragma unroll
  for (int i = 0; i < 3; i++) s.bw[i] = st[(size_t)(10 + i) * n + e];
#pragma unroll
  for (int d = 0; d < R::NJ; d++) s.q[d] = st[(size_t)(PBG_BASE_WORDS + d) * n + e];
#pragma unroll
  for (int d = 0; d < R::NJ; d++) s.qd[d] = st[(size_t)(PBG_BASE_WORDS + R::NJ + d) * n + e];
  if constexpr (R::harder) {
    constexpr int c0 = PBG_BASE_WORDS + 2 * R::NJ;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      s.cube.p[i] = st[(size_t)(c0 + i) * n + e];
      s.cube.v[i] = st[(size_t)(c0 + 7 + i) * n + e];
      s.cube.w[i] = st[(size_t)(c0 + 10 + i) * n + e];
    }
#pragma unroll
    for (int i = 0; i < 4; i++) s.cube.q[i] = st[(size_t)(c0 + 3 + i) * n + e];
  }
}
template <class R>
PBG_DEV void store_state(const State<R>& s, real_t<R>* __restrict__ st, int n, int e) {
#pragma unroll
  for (int i = 0; i < 3; i++) st[(size_t)i * n + e] = s.bp[i];
#pragma unroll
  for (int i = 0; i < 4; i++) st[(size_t)(3 + i) * n + e] = s.bq[i];
#pragma unroll
  for (int i = 0; i < 3; i++) st[(size_t)(7 + i) * n + e] = s.bv[i];
#pragma unroll
  for (int i = 0; i < 3; i++) st[(size_t)(10 + i) * n + e] = s.bw[i];
#pragma unroll
  for (int d = 0; d < R::NJ; d++) st[(size_t)(PBG_BASE_WORDS + d) * n + e] = s.q[d];
#pragma unroll
  for (int d = 0; d < R::NJ; d++) st[(size_t)(PBG_BASE_WORDS + R::NJ + d) * n + e] = s.qd[d];
  if constexpr (R::harder) {
    constexpr int c0 = PBG_BASE_WORDS + 2 * R::NJ;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      st[(size_t)(c0 + i) * n + e] = s.cube.p[i];
      st[(size_t)(c0 + 7 + i) * n + e] = s.cube.v[i];
      st[(size_t)(c0 + 10 + i) * n + e] = s.cube.w[i];
    }
#pragma unroll
    for (int i = 0; i < 4; i++) st[(size_t)(c0 + 3 + i) * n + e] = s.cube.q[i];
  }
}

// Stores of a value replicated over T cooperating lanes (gang / quad kernels), dealt over
// them: lane t stores elements t, t+T, ... -- each element picked by selects, so the
// register arrays are never indexed at run time.
template <int T, int M, int W, class V>
PBG_DEV V lanes_pick(const V (&v)[W], int t) {  // v[M*T + t] by selects (no indexed registers)
  V r = v[M * T];
  static_for<1, T>([&](auto k_c) {
    constexpr int k = decltype(k_c)::value;
    if constexpr (M * T + k < W) r = t == k ? v[M * T + k] : r;
  });
  return r;
}
template <class R, int T>
PBG_DEV void lanes_store_row(const float (&obs)[R::OBS], float* __restrict__ out, int e, int t) {  // out[e][:]
  static_for<0, (R::OBS + T - 1) / T>([&](auto m_c) {
    constexpr int m = decltype(m_c)::value;
    const float v = lanes_pick<T, m, R::OBS>(obs, t);
    if (m * T + t < R::OBS) out[(size_t)e * R::OBS + m * T + t] = v;
  });
}
// load snapshot (gym_locomotion_envs.py:23-25 restoreState) + reset noise on reset dofs
template <class R>
PBG_DEV void snapshot_state(State<R>& s) {
  using T = real_t<R>;
#pragma unroll
  for (int i = 0; i < 3; i++) s.bp[i] = (T)R::base_pos[i];
#pragma unroll
  for (int i = 0; i < 4; i++) s.bq[i] = (T)R::base_quat[i];
#pragma unroll
  for (int i = 0; i < 3; i++) { s.bv[i] = 0.f; s.bw[i] = 0.f; }
#pragma unroll
  for (int d = 0; d < R::NJ; d++) { s.q[d] = 0.f; s.qd[d] = 0.f; }
  if constexpr (R::harder) {  // restoreState + resetBasePositionAndOrientation(cube, (-1.5, 0, 0.05)) (:241)
    s.cube.p[0] = (T)PBG_CUBE_X0; s.cube.p[1] = (T)PBG_CUBE_Y0; s.cube.p[2] = (T)PBG_CUBE_Z0;
    s.cube.q[0] = 0.f; s.cube.q[1] = 0.f; s.cube.q[2] = 0.f; s.cube.q[3] = 1.f;
#pragma unroll
    for (int i = 0; i < 3; i++) { s.cube.v[i] = 0.f; s.cube.w[i] = 0.f; }
  }
}

// ------------------------------------------------------------------ kinematics
template <class R>
struct Kin {
  static constexpr int NB = R::NL + 1;
  M3<real_t<R>> Rm[NB];
  V3<real_t<R>> x[NB], c[NB];
};
template <class R>
struct KinVel {
  static constexpr int NB = R::NL + 1;
  V3<real_t<R>> w[NB], v[NB], al[NB], ac[NB];
};

// Forward kinematics (positions; optionally the world axis / anchor of every joint dof).
template <class R, bool AXES = false>
PBG_DEV void fk_pos(const State<R>& s, Kin<R>& k, V3<real_t<R>>* ja = nullptr, V3<real_t<R>>* jo = nullptr) {
  using T = real_t<R>;
  using f3 = V3<T>;
  using m3 = M3<T>;
  k.Rm[0] = quat_to_m3(s.bq[0], s.bq[1], s.bq[2], s.bq[3]);
  k.x[0] = mk3<T>(s.bp[0], s.bp[1], s.bp[2]);
  k.c[0] = k.x[0];
  static_for<0, R::NL>([&](auto l_c) {
    constexpr int l = decltype(l_c)::value;
    constexpr int p = R::link_parent[l] + 1;
    const m3 Ro = quat_to_m3c<T>(R::link_offset_quat[l][0], R::link_offset_quat[l][1], R::link_offset_quat[l][2], R::link_offset_quat[l][3]);
    const m3 R0 = mulc(k.Rm[p], Ro);
    const f3 x0 = k.x[p] + mulc(k.Rm[p], (T)R::link_offset_pos[l][0], (T)R::link_offset_pos[l][1], (T)R::link_offset_pos[l][2]);
    const f3 axl = mk3<T>((T)R::link_axis[l][0], (T)R::link_axis[l][1], (T)R::link_axis[l][2]);
    const f3 anl = mk3<T>((T)R::link_anchor[l][0], (T)R::link_anchor[l][1], (T)R::link_anchor[l][2]);
    constexpr int jt = R::link_jtype[l], d = R::link_dof[l];
    if constexpr (jt == 0) {
      const m3 Rj = axis_angle_m3c<T, lib_trig_v<R>>(axl.x, axl.y, axl.z, s.q[d]);
      k.Rm[l + 1] = mul(R0, Rj);
      k.x[l + 1] = x0 + mul(R0, anl - mulc(Rj, anl));
      if constexpr (AXES) { ja[d] = mulc(R0, axl); jo[d] = x0 + mulc(R0, anl); }
    } else if constexpr (jt == 1) {
      k.Rm[l + 1] = R0;
      k.x[l + 1] = x0 + s.q[d] * mulc(R0, axl);
      if constexpr (AXES) { ja[d] = mulc(R0, axl); jo[d] = x0; }
    } else {
      k.Rm[l + 1] = R0;
      k.x[l + 1] = x0;
    }
    k.c[l + 1] = k.x[l + 1] + mulc(k.Rm[l + 1], (T)R::link_com[l][0], (T)R::link_com[l][1], (T)R::link_com[l][2]);
  });
}

// Opaque copy of the positional state: forces a recomputation instead of keeping values
// of an earlier phase live across the solve (register pressure).
template <class R>
PBG_DEV State<R> opaque_positions(const State<R>& s) {
  State<R> t = s;
#pragma unroll
  for (int i = 0; i < 3; i++) asm volatile("" : "+v"(t.bp[i]));
#pragma unroll
  for (int i = 0; i < 4; i++) asm volatile("" : "+v"(t.bq[i]));
#pragma unroll
  for (int d = 0; d < R::NJ; d++) asm volatile("" : "+v"(t.q[d]));
  return t;
}

// ------------------------------------------------------------------ per-substep scratch
// Constraint rows, per lane in LDS (dynamic shared memory, [word][lane]: conflict-free):
//   [joint-limit block | contact rows 0..cap-1 | mu per contact]
// Joint-limit rows are compile-time: one block per limited dof holding the sparse
// y = L^-1 e_g (only the dof and its ancestors + base are non-zero), m_eff and the
// lower/upper targets and impulses -- the two rows of a joint share y and are solved
// back to back.  Contact c owns rows 3c + {normal, t1, t2}, y dense; contact rows beyond
// the LDS capacity (rare: many simultaneous contacts) go to a device workspace laid out
// [word][env] (coalesced).
typedef __attribute__((address_space(3))) float lds_float;  // explicit LDS pointers
typedef __attribute__((address_space(3))) double lds_double;
template <class T>
using lds_t = std::conditional_t<std::is_same<T, double>::value, lds_double, lds_float>;

template <class R, int LS = 64>
struct Rows {
  using D = Dims<R>;
  using T = real_t<R>;
  static constexpr int N = D::NY, W = N + 3;  // contact row: y | meff | target | lambda (N: robot [+ cube])
  // rows per contact: normal, 2 lateral friction (+ spinning, 2 rolling: robots whose links carry
  // torsional friction, HalfCheetahMuJoCo); contact c's rows are NRC c + dir
  static constexpr int NRC = (R::spin_mu > 0.0 || R::roll_mu > 0.0) ? 6 : 3;
  static_assert(NRC == 3 || (!R::harder && R::NPAIR == 0), "torsional rows: robot-floor contacts only");
  static constexpr int MR = NRC * D::NC > 0 ? NRC * D::NC : 1;
  static constexpr int NC = D::NC > 0 ? D::NC : 1;
  static constexpr int WORDS = MR * W;  // global workspace words per env
  static constexpr int ls = LS;  // LDS stride = lanes per workgroup
  static constexpr int LIMW = D::LIMW;
  lds_t<T>* lds;   // LDS base + lane
  T* gbl;          // global workspace base + env
  int n;       // global stride (envs)
  int cap;     // contact rows resident in LDS
  PBG_DEV lds_t<T>& lim(int w) const { return lds[(size_t)w * ls]; }
  PBG_DEV lds_t<T>& mu(int c) const { return lds[(size_t)(LIMW + cap * W + c) * ls]; }
  template <class P>
  static PBG_DEV void put_at(P p, size_t st, const T* y, T meff, T target) {
#pragma unroll
    for (int i = 0; i < N; i++) p[i * st] = y[i];
    p[N * st] = meff;
    p[(N + 1) * st] = target;
    p[(N + 2) * st] = 0.f;
  }
  template <class P>
  static PBG_DEV void solve_at(P p, size_t st, T* u, T lo, T hi) {
    T yv[N];
#pragma unroll
    for (int i = 0; i < N; i++) yv[i] = p[i * st];
    const T meff = p[N * st], tgt = p[(N + 1) * st], lam0 = p[(N + 2) * st];
    T acc[4] = {0.f, 0.f, 0.f, 0.f};  // 4 partial sums: shorter dependency chain
#pragma unroll
    for (int i = 0; i < N; i++) acc[i & 3] += yv[i] * u[i];
    const T yu = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    const T nl = clampf(lam0 + meff * (tgt - yu), lo, hi);
    const T dl = nl - lam0;
    p[(N + 2) * st] = nl;
#pragma unroll
    for (int i = 0; i < N; i++) u[i] += yv[i] * dl;
  }
  PBG_DEV void put(int r, const T* y, T meff, T target) const {
    if (r < cap) put_at(lds + (size_t)(LIMW + r * W) * ls, (size_t)ls, y, meff, target);
    else put_at(gbl + (size_t)r * W * n, (size_t)n, y, meff, target);
  }
  PBG_DEV T lam(int r) const {
    if (r < cap) return lds[(size_t)(LIMW + r * W + N + 2) * ls];
    return gbl[((size_t)r * W + N + 2) * n];
  }
  // one projected Gauss-Seidel update of contact row r in u-space, bounds [lo, hi]
  PBG_DEV void solve(int r, T* u, T lo, T hi) const {
    if (r < cap) solve_at(lds + (size_t)(LIMW + r * W) * ls, (size_t)ls, u, lo, hi);
    else solve_at(gbl + (size_t)r * W * n, (size_t)n, u, lo, hi);
  }
};

// ------------------------------------------------------------------ one physics sub-step
// Target of J nu_new for a positional row (contact normal, joint limit), Bullet's rhs
// (btMultiBodyConstraintSolver::setupMultiBodyContactConstraint; velocityError = -rel_vel,
// minus pos/dt when separated, positionalError = -erp pos/dt when penetrating) in absolute form:
// a separated row admits an approach of at most pos/dt (speculative contact), a penetrating
// one pushes out at erp * pos / dt.  Continuous at pos = 0.
// k_pen / k_sep: the slopes -erp/dt and -1/dt of SimP (pbg_types.h), pre-formed on the host.
template <class S>
PBG_DEV S pos_target(S pos, nd<S> k_pen, nd<S> k_sep) { return (pos > S(0) ? k_sep : k_pen) * pos; }

// tau: motor torque per joint dof, held over the env step.  slot_active: floor-slot flags
// of this sub-step's collision pass (feet contacts come from the last sub-step).
// dof motion vectors (angular, linear-at-O) in generalized order
template <class R>
PBG_DEV void motion_vectors(const V3<real_t<R>>* ja, const V3<real_t<R>>* jo, V3<real_t<R>> O, V3<real_t<R>>* sw,
                            V3<real_t<R>>* sv) {
  using D = Dims<R>;
  using T = real_t<R>;
  using f3 = V3<T>;
#pragma unroll
  for (int gi = 0; gi < R::NDOF; gi++) {
    const int d = D::dof_of(gi);
    if (d >= 0) {
      if (R::dof_jtype[d] == 0) { sw[gi] = ja[d]; sv[gi] = cross3(jo[d] - O, ja[d]); }
      else { sw[gi] = mk3<T>(0, 0, 0); sv[gi] = ja[d]; }
    } else {
      const int kk = gi - R::NJ;  // 0..2 linear, 3..5 angular
      const f3 e = mk3<T>(kk % 3 == 0, kk % 3 == 1, kk % 3 == 2);
      if (kk < 3) { sw[gi] = mk3<T>(0, 0, 0); sv[gi] = e; }
      else { sw[gi] = e; sv[gi] = mk3<T>(0, 0, 0); }
    }
  }
}

// Link frames and dof motion vectors about the reference point O, recomputed from the
// positions (cheaper than keeping phase A's copies live through the factorisation).
template <class R>
PBG_DEV void kin_motion(const State<R>& s, Kin<R>& k, V3<real_t<R>>* sw, V3<real_t<R>>* sv, V3<real_t<R>>& O) {
  using D = Dims<R>;
  using f3 = V3<real_t<R>>;
  constexpr int NJ = R::NJ;
  const State<R> sp = opaque_positions<R>(s);
  f3 ja2[NJ > 0 ? NJ : 1], jo2[NJ > 0 ? NJ : 1];
  fk_pos<R, true>(sp, k, ja2, jo2);
  O = k.c[D::REF_BODY];
  motion_vectors<R>(ja2, jo2, O, sw, sv);
}

#ifdef PBG_STAMPS
#define SUB_STAMP_ARGS , unsigned long long& _st_t, unsigned long long* _st_acc
#define SUB_STAMP_PASS , _st_t, _st_acc
#else
#define SUB_STAMP_ARGS
#define SUB_STAMP_PASS
#endif
// Unconstrained joint-space dynamics of one sub-step (phase A .. u): composites, mass
// matrix and bias, its sparse Cholesky factor L (Ld = 1/diag), the predicted velocity
// nu = clamp(nu + dt M^-1 (tau - C)) and u = L^T nu.  Shared by the lane and gang kernels.
template <class R>
PBG_DEV void dyn_mass(const State<R>& s, const real_t<R>* tau, real_t<R>* L, real_t<R>* rhs,
                      const SimPT<real_t<R>>& P SUB_STAMP_ARGS) {
  using D = Dims<R>;
  using T = real_t<R>;
  using f3 = V3<T>;
  using m3 = M3<T>;
  using s6 = S6<T>;
  constexpr int NJ = R::NJ, NB = D::NB, N = R::NDOF;
  const T g = P.gravity;

  // --- phase A: one forward pass over the bodies: kinematics, velocities, bias
  // accelerations, and each body's inertia + wrench about the reference point O added
  // straight into the composites of its dof-owning ancestors.  No per-body array
  // survives the pass (register pressure); positions are recomputed for contacts.
  f3 ja[NJ > 0 ? NJ : 1], jo[NJ > 0 ? NJ : 1];
  T cm[NB];
  f3 cp1[NB], cF[NB], cN[NB];
  s6 cJ[NB];
  static_for<0, NB>([&](auto b_c) {
    constexpr int b = decltype(b_c)::value;
    if constexpr (D::is_owner(b)) {
      cm[b] = 0.f; cp1[b] = mk3<T>(0, 0, 0); cF[b] = mk3<T>(0, 0, 0); cN[b] = mk3<T>(0, 0, 0);
#pragma unroll
      for (int i = 0; i < 6; i++) cJ[b].a[i] = 0.f;
    }
  });
  f3 O = mk3<T>(s.bp[0], s.bp[1], s.bp[2]);
  {
    Kin<R> k;
    f3 w[NB], v[NB], al[NB], ac[NB];
    k.Rm[0] = quat_to_m3(s.bq[0], s.bq[1], s.bq[2], s.bq[3]);
    k.x[0] = mk3<T>(s.bp[0], s.bp[1], s.bp[2]);
    k.c[0] = k.x[0];
    w[0] = R::floating ? mk3<T>(s.bw[0], s.bw[1], s.bw[2]) : mk3<T>(0, 0, 0);
    v[0] = R::floating ? mk3<T>(s.bv[0], s.bv[1], s.bv[2]) : mk3<T>(0, 0, 0);
    al[0] = mk3<T>(0, 0, 0);
    ac[0] = mk3<T>(0, 0, 0);
    static_for<0, NB>([&](auto b_c) {
      constexpr int b = decltype(b_c)::value;
      if constexpr (b > 0) {
        constexpr int l = b - 1;
        constexpr int p = R::link_parent[l] + 1;
        constexpr int jt = R::link_jtype[l], d = R::link_dof[l];
        const m3 Ro = quat_to_m3c<T>(R::link_offset_quat[l][0], R::link_offset_quat[l][1], R::link_offset_quat[l][2], R::link_offset_quat[l][3]);
        const m3 R0 = mulc(k.Rm[p], Ro);
        const f3 x0 = k.x[p] + mulc(k.Rm[p], (T)R::link_offset_pos[l][0], (T)R::link_offset_pos[l][1], (T)R::link_offset_pos[l][2]);
        const f3 axl = mk3<T>((T)R::link_axis[l][0], (T)R::link_axis[l][1], (T)R::link_axis[l][2]);
        const f3 anl = mk3<T>((T)R::link_anchor[l][0], (T)R::link_anchor[l][1], (T)R::link_anchor[l][2]);
        if constexpr (jt == 0) {
          const m3 Rj = axis_angle_m3c<T, lib_trig_v<R>>(axl.x, axl.y, axl.z, s.q[d]);
          k.Rm[b] = mul(R0, Rj);
          k.x[b] = x0 + mul(R0, anl - mulc(Rj, anl));
        } else if constexpr (jt == 1) {
          k.Rm[b] = R0;
          k.x[b] = x0 + s.q[d] * mulc(R0, axl);
        } else {
          k.Rm[b] = R0;
          k.x[b] = x0;
        }
        k.c[b] = k.x[b] + mulc(k.Rm[b], (T)R::link_com[l][0], (T)R::link_com[l][1], (T)R::link_com[l][2]);
        const f3 cp = k.c[p], wp = w[p], vp = v[p], alp = al[p], acp = ac[p];
        const f3 c = k.c[b];
        if constexpr (jt == 0 || jt == 1) {
          const f3 a = mulc(R0, axl);
          ja[d] = a;
          if constexpr (jt == 0) {
            const f3 o = x0 + mulc(R0, anl);
            jo[d] = o;
            const f3 ro = o - cp;
            const f3 vo = vp + cross3(wp, ro);
            const f3 ao = acp + cross3(alp, ro) + cross3(wp, cross3(wp, ro));
            const f3 wl = wp + s.qd[d] * a;
            const f3 all = alp + s.qd[d] * cross3(wp, a);
            const f3 rc = c - o;
            w[b] = wl;
            al[b] = all;
            v[b] = vo + cross3(wl, rc);
            ac[b] = ao + cross3(all, rc) + cross3(wl, cross3(wl, rc));
          } else {
            jo[d] = x0;
            const f3 r = c - cp;
            w[b] = wp;
            al[b] = alp;
            v[b] = vp + cross3(wp, r) + s.qd[d] * a;
            ac[b] = acp + cross3(alp, r) + cross3(wp, cross3(wp, r)) + (T(2) * s.qd[d]) * cross3(wp, a);
          }
        } else {
          const f3 r = c - cp;
          w[b] = wp;
          al[b] = alp;
          v[b] = vp + cross3(wp, r);
          ac[b] = acp + cross3(alp, r) + cross3(wp, cross3(wp, r));
        }
      }
      if (b == D::REF_BODY) O = k.c[b];
      if constexpr (D::body_mass(b) > 0.0) {
        const T m = (T)D::body_mass(b);
        constexpr typename D::Inertia6 I6 = D::template inertia<b>();
        const s6 Iw = rotate_inertia(k.Rm[b], I6.v);
        const f3 r = k.c[b] - O;
        const T rr = dot3(r, r);
        s6 J;
        J.a[0] = Iw.a[0] + m * (rr - r.x * r.x);
        J.a[1] = Iw.a[1] + m * (rr - r.y * r.y);
        J.a[2] = Iw.a[2] + m * (rr - r.z * r.z);
        J.a[3] = Iw.a[3] - m * r.x * r.y;
        J.a[4] = Iw.a[4] - m * r.x * r.z;
        J.a[5] = Iw.a[5] - m * r.y * r.z;
        const f3 Iww = mul(Iw, w[b]);
        const f3 f = m * (ac[b] - mk3<T>(0, 0, -g)) +
                     (m * ((T)PBG_LINEAR_DAMPING + (T)PBG_LINEAR_DAMPING * norm3(v[b]))) * v[b];
        const f3 n = mul(Iw, al[b]) + cross3(w[b], Iww) +
                     ((T)PBG_ANGULAR_DAMPING + (T)PBG_ANGULAR_DAMPING * norm3(w[b])) * Iww;
        const f3 pr = m * r, Nn = n + cross3(r, f);
        static_for<0, NB>([&](auto a_c) {
          constexpr int a = decltype(a_c)::value;
          if constexpr (D::is_owner(a) && D::anc_or_self(a, b)) {
            cm[a] += m;
            cp1[a] += pr;
            cF[a] += f;
            cN[a] += Nn;
#pragma unroll
            for (int i = 0; i < 6; i++) cJ[a].a[i] += J.a[i];
          }
        });
      }
      PBG_PHASE_BARRIER
    });
  }

  STAMP(0)
  // --- mass matrix (lower triangle, gi >= gk) and bias -----------------------------------
  {
  f3 sw[N], sv[N];
  motion_vectors<R>(ja, jo, O, sw, sv);
#pragma unroll
  for (int gi = 0; gi < N; gi++) {
    // composite body owning dof gi (its link); base dofs use the whole-robot composite
    const int di = D::dof_of(gi);
    const int bi = di >= 0 ? R::dof_link[di] + 1 : 0;
    // bias: C_gi = s_gi . (N, F) of its composite
    rhs[gi] = -(dot3(sw[gi], cN[bi]) + dot3(sv[gi], cF[bi]));
#pragma unroll
    for (int gk = 0; gk <= gi; gk++) {
      if (!D::coupled(gi, gk)) continue;
      // deeper dof of the pair owns the composite: joints come leaf-first, so the smaller
      // generalized index is the deeper (or equal) one; base dofs are the root.
      const int dk = D::dof_of(gk);
      const int bk = dk >= 0 ? R::dof_link[dk] + 1 : 0;
      const f3 Jw_ = mul(cJ[bk], sw[gk]) + cross3(cp1[bk], sv[gk]);
      const f3 Fv = cm[bk] * sv[gk] - cross3(cp1[bk], sw[gk]);
      L[D::lidx(gi, gk)] = dot3(sw[gi], Jw_) + dot3(sv[gi], Fv);
    }
  }
  }
  // joint damping -d qd and springs -k q (mjcf.py B6 / B7), explicit from this sub-step's state
  static_for<0, NJ>([&](auto d_c) {
    constexpr int d = decltype(d_c)::value;
    L[D::lidx(D::gj(d), D::gj(d))] += (T)R::dof_armature[d];
    T r = tau[d];
    if constexpr (R::dof_damping[d] != 0.0) r -= (T)R::dof_damping[d] * s.qd[d];
    if constexpr (R::dof_stiffness[d] != 0.0) r -= (T)R::dof_stiffness[d] * s.q[d];
    rhs[D::gj(d)] += r;
  });
  STAMP(1)
}

// Cholesky of the mass matrix held in L (in place, no fill-in in leaf-first order; Ld =
// 1 / diag(L)), nu = clamp(nu + dt M^-1 rhs), u = L^T nu.
template <class R>
PBG_DEV void dyn_solve(const State<R>& s, real_t<R>* L, const real_t<R>* rhs, real_t<R>* Ld, real_t<R>* nu, real_t<R>* u,
                       const SimPT<real_t<R>>& P) {
  using D = Dims<R>;
  using T = real_t<R>;
  constexpr int NJ = R::NJ, N = R::NDOF;
  const T dt = P.dt;
#pragma unroll
  for (int j = 0; j < N; j++) {
    T sjj = L[D::lidx(j, j)];
#pragma unroll
    for (int kk = 0; kk < j; kk++)
      if (D::coupled(j, kk)) sjj -= L[D::lidx(j, kk)] * L[D::lidx(j, kk)];
    const T ljj = fast_sqrt(sjj);
    const T inv = fast_rcp(ljj);
    Ld[j] = inv;
    L[D::lidx(j, j)] = ljj;
#pragma unroll
    for (int i = j + 1; i < N; i++) {
      if (!D::coupled(i, j)) continue;
      T t = L[D::lidx(i, j)];
#pragma unroll
      for (int kk = 0; kk < j; kk++)
        if (D::coupled(i, kk) && D::coupled(j, kk)) t -= L[D::lidx(i, kk)] * L[D::lidx(j, kk)];
      L[D::lidx(i, j)] = t * inv;
    }
  }

  // --- unconstrained velocity: nu_pred = nu + dt * M^-1 (tau - C) ------------------------
#pragma unroll
  for (int d = 0; d < NJ; d++) nu[D::gj(d)] = s.qd[d];
  if (R::floating) {
#pragma unroll
    for (int i = 0; i < 3; i++) { nu[NJ + i] = s.bv[i]; nu[NJ + 3 + i] = s.bw[i]; }
  }
  T yv[N];
#pragma unroll
  for (int i = 0; i < N; i++) {  // forward: L y = rhs
    T t = rhs[i];
#pragma unroll
    for (int kk = 0; kk < i; kk++)
      if (D::coupled(i, kk)) t -= L[D::lidx(i, kk)] * yv[kk];
    yv[i] = t * Ld[i];
  }
  T qdd[N];
#pragma unroll
  for (int i = N - 1; i >= 0; i--) {  // backward: L^T x = y
    T t = yv[i];
#pragma unroll
    for (int kk = i + 1; kk < N; kk++)
      if (D::coupled(kk, i)) t -= L[D::lidx(kk, i)] * qdd[kk];
    qdd[i] = t * Ld[i];
  }
  // u = L^T nu_pred
#pragma unroll
  for (int i = 0; i < N; i++) {
    T t = nu[i] + dt * qdd[i];
    nu[i] = clampf(t, -(T)PBG_MAX_COORD_VELOCITY, (T)PBG_MAX_COORD_VELOCITY);
  }
#pragma unroll
  for (int i = 0; i < N; i++) {
    T t = 0.f;
#pragma unroll
    for (int kk = i; kk < N; kk++)
      if (D::coupled(kk, i)) t += L[D::lidx(kk, i)] * nu[kk];
    u[i] = t;
  }
}

template <class R>
PBG_DEV void dynamics(const State<R>& s, const real_t<R>* tau, real_t<R>* L, real_t<R>* Ld, real_t<R>* nu, real_t<R>* u,
                      const SimPT<real_t<R>>& P SUB_STAMP_ARGS) {
  real_t<R> rhs[R::NDOF];
  dyn_mass<R>(s, tau, L, rhs, P SUB_STAMP_PASS);
  dyn_solve<R>(s, L, rhs, Ld, nu, u, P);
}

// exponential-map quaternion update of a free body (the floating base, the cube) with its
// world angular velocity  [EXT] btMultiBody pQuatUpdateFun
template <bool LIB = false, class S>
PBG_DEV void free_body_quat(S* q, V3<S> wv, const SimPT<S>& P) {
  const S dt = P.dt;
  S ang = norm3(wv);
  if (ang * dt > (S)PBG_ANGULAR_MOTION_THRESHOLD) ang = P.ang_max;
  S sh, dw;
  sincos_phys<LIB>(S(0.5f) * ang * dt, &sh, &dw);
  V3<S> ax;
  if (ang < S(0.001)) ax = (S(0.5f) * dt - P.dt3c * ang * ang) * wv;
  else ax = (sh / ang) * wv;
  const S x = q[0], y = q[1], z = q[2], ww = q[3];
  const S nx = dw * x + ax.x * ww + ax.y * z - ax.z * y;
  const S ny = dw * y - ax.x * z + ax.y * ww + ax.z * x;
  const S nz = dw * z + ax.x * y - ax.y * x + ax.z * ww;
  const S nw = dw * ww - ax.x * x - ax.y * y - ax.z * z;
  const S inv = fast_rsq(nx * nx + ny * ny + nz * nz + nw * nw);
  q[0] = nx * inv; q[1] = ny * inv; q[2] = nz * inv; q[3] = nw * inv;
}

// HumanoidFlagrunHarder's cube (a free body with isotropic inertia, block-diagonal to the robot):
// its Cholesky factor is diag(sqrt m x3, sqrt I x3), so u_c = L_c^T nu_c and y_c = L_c^-1 J_c are
// plain scalings.  Unconstrained velocity: the free-body bias of the oracle's mass_and_bias
// (f = m (-g) + m (k1 + k2 |v|) v, tq = (k1 + k2 |w|) I w; the gyroscopic term of an isotropic
// body vanishes), nu_c = clamp(nu_c - dt M_c^-1 (f, tq)), then u_c.
template <class S>
struct CubeK {
  static PBG_DEV S sm() { return tsqrt((S)PBG_CUBE_MASS); }
  static PBG_DEV S sI() { return tsqrt((S)PBG_CUBE_INERTIA); }
};
template <class R>
PBG_DEV void cube_unconstrained(const State<R>& s, real_t<R>* uc, const SimPT<real_t<R>>& P) {
  using T = real_t<R>;
  using f3 = V3<T>;
  using CK = CubeK<T>;
  if constexpr (R::harder) {
    const f3 v = mk3<T>(s.cube.v[0], s.cube.v[1], s.cube.v[2]), w = mk3<T>(s.cube.w[0], s.cube.w[1], s.cube.w[2]);
    const T kl = (T)PBG_LINEAR_DAMPING + (T)PBG_LINEAR_DAMPING * norm3(v);
    const T ka = (T)PBG_ANGULAR_DAMPING + (T)PBG_ANGULAR_DAMPING * norm3(w);
    const T vmax = (T)PBG_MAX_COORD_VELOCITY;
    const T vv[3] = {v.x, v.y, v.z}, wv[3] = {w.x, w.y, w.z};
#pragma unroll
    for (int i = 0; i < 3; i++) {
      const T acc = -(kl * vv[i]) - (i == 2 ? P.gravity : T(0));
      uc[i] = CK::sm() * clampf(vv[i] + P.dt * acc, -vmax, vmax);
      uc[3 + i] = CK::sI() * clampf(wv[i] + P.dt * (-(ka * wv[i])), -vmax, vmax);
    }
  } else {
    (void)s; (void)uc; (void)P;
  }
}
// nu_c = L_c^-T u_c, clamp, semi-implicit Euler
template <class R>
PBG_DEV void cube_integrate(State<R>& s, const real_t<R>* uc, const SimPT<real_t<R>>& P) {
  using T = real_t<R>;
  using CK = CubeK<T>;
  if constexpr (R::harder) {
    const T vmax = (T)PBG_MAX_COORD_VELOCITY;
    const T rm = T(1) / CK::sm(), rI = T(1) / CK::sI();
#pragma unroll
    for (int i = 0; i < 3; i++) {
      s.cube.v[i] = clampf(uc[i] * rm, -vmax, vmax);
      s.cube.w[i] = clampf(uc[3 + i] * rI, -vmax, vmax);
      s.cube.p[i] += P.dt * s.cube.v[i];
    }
    free_body_quat<lib_trig_v<R>>(s.cube.q, mk3<T>(s.cube.w[0], s.cube.w[1], s.cube.w[2]), P);
  } else {
    (void)s; (void)uc; (void)P;
  }
}
// signed distance of a cube-local point to the box of half extent h (oracle box_sd)
template <class S>
PBG_DEV S box_sd(V3<S> p, S h) {
  const S qx = tabs(p.x) - h, qy = tabs(p.y) - h, qz = tabs(p.z) - h;
  const S ox = tmax(qx, S(0)), oy = tmax(qy, S(0)), oz = tmax(qz, S(0));
  return tsqrt(ox * ox + oy * oy + oz * oz) + tmin(tmax(qx, tmax(qy, qz)), S(0));
}

// nu = L^-T u, clamp, semi-implicit Euler (exponential-map base rotation).  nu: scratch.
template <class R>
PBG_DEV void integrate(State<R>& s, const real_t<R>* L, const real_t<R>* Ld, const real_t<R>* u, real_t<R>* nu,
                       const SimPT<real_t<R>>& P) {
  using D = Dims<R>;
  using T = real_t<R>;
  constexpr int NJ = R::NJ, N = R::NDOF;
  const T dt = P.dt;
  // --- back to nu = L^-T u; clamp; integrate positions ----------------------------------
#pragma unroll
  for (int i = N - 1; i >= 0; i--) {
    T t = u[i];
#pragma unroll
    for (int kk = i + 1; kk < N; kk++)
      if (D::coupled(kk, i)) t -= L[D::lidx(kk, i)] * nu[kk];
    nu[i] = t * Ld[i];
  }
#pragma unroll
  for (int i = 0; i < N; i++) nu[i] = clampf(nu[i], -(T)PBG_MAX_COORD_VELOCITY, (T)PBG_MAX_COORD_VELOCITY);
#pragma unroll
  for (int d = 0; d < NJ; d++) {
    s.qd[d] = nu[D::gj(d)];
    s.q[d] += dt * s.qd[d];
  }
  if (R::floating) {
#pragma unroll
    for (int i = 0; i < 3; i++) {
      s.bv[i] = nu[NJ + i];
      s.bw[i] = nu[NJ + 3 + i];
      s.bp[i] += dt * s.bv[i];
    }
    free_body_quat<lib_trig_v<R>>(s.bq, mk3<T>(s.bw[0], s.bw[1], s.bw[2]), P);
  }
}

// HumanoidFlagrunHarder's cube against the floor and the robot (oracle detect_cube_contacts):
// candidates NS + NPAIR + corner (8), then NS + NPAIR + 8 + geom; a corner within the contact
// threshold of the floor is a point (normal +z, cube = body A), a robot geom against the box
// takes the minimiser of the box's signed distance along its segment (golden section,
// PBG_CUBE_GS_ITERS rounds; robot link = A, cube = B).  Rows: the robot part y_h = L^-1 J_h as
// for the self pairs, the cube part y_c = +-(n / sqrt m, (r x n) / sqrt I).  Returns nc.
#define PBG_CUBE_GS_ITERS 24
template <class R, int LS>
PBG_DEV int cube_contacts(const State<R>& s, const Kin<R>& k, const V3<real_t<R>>* sw, const V3<real_t<R>>* sv,
                          V3<real_t<R>> O, const real_t<R>* L, const real_t<R>* Ld, const Rows<R, LS>& rw, uint32_t sub,
                          uint32_t& csig, const SimPT<real_t<R>>& P, int nc) {
  using D = Dims<R>;
  using T = real_t<R>;
  using f3 = V3<T>;
  using m3 = M3<T>;
  using CK = CubeK<T>;
  constexpr int N = R::NDOF, NY = D::NY;
  const T h = (T)PBG_CUBE_HALF, thr = (T)PBG_CONTACT_THRESHOLD;
  const T rm = T(1) / CK::sm(), rI = T(1) / CK::sI();
  const m3 Rc = quat_to_m3(s.cube.q[0], s.cube.q[1], s.cube.q[2], s.cube.q[3]);
  const f3 xc = mk3<T>(s.cube.p[0], s.cube.p[1], s.cube.p[2]);
  // --- corners vs floor
  static_for<0, 8>([&](auto c_c) {
    constexpr int c = decltype(c_c)::value;
    const f3 lc = mk3<T>((c & 1) ? h : -h, (c & 2) ? h : -h, (c & 4) ? h : -h);
    const f3 p = xc + mul(Rc, lc);
    if (!(p.z < thr)) return;
    csig += pbg_contact_hash(sub, (uint32_t)(R::NS + R::NPAIR + c));
    const f3 rc = p - xc;
#pragma unroll
    for (int dir = 0; dir < 3; dir++) {
      const f3 nd = dir == 0 ? mk3<T>(0, 0, 1) : (dir == 1 ? mk3<T>(0, -1, 0) : mk3<T>(1, 0, 0));
      const f3 mm = cross3(rc, nd);
      T y[NY];
#pragma unroll
      for (int i = 0; i < N; i++) y[i] = 0.f;
      y[N] = nd.x * rm; y[N + 1] = nd.y * rm; y[N + 2] = nd.z * rm;
      y[N + 3] = mm.x * rI; y[N + 4] = mm.y * rI; y[N + 5] = mm.z * rI;
      T D2 = 0.f;
#pragma unroll
      for (int i = N; i < NY; i++) D2 += y[i] * y[i];
      rw.put(Rows<R, LS>::NRC * nc + dir, y, D2 > T(1e-12) ? fast_rcp(D2) : T(0), dir == 0 ? pos_target(p.z, P.k_contact, P.k_sep) : T(0));
    }
    rw.mu(nc) = (T)R::cube_floor_mu;
    nc++;
  });
  // --- robot geoms vs the box
  f3 G0[R::NCG], G1[R::NCG];
#pragma unroll
  for (int g = 0; g < R::NCG; g++) {
    const int b = R::cgeom_link[g] + 1;
    G0[g] = k.x[b] + mulc(k.Rm[b], (T)R::cgeom_p0[g][0], (T)R::cgeom_p0[g][1], (T)R::cgeom_p0[g][2]);
    G1[g] = k.x[b] + mulc(k.Rm[b], (T)R::cgeom_p1[g][0], (T)R::cgeom_p1[g][1], (T)R::cgeom_p1[g][2]);
  }
  m3 Rt;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) Rt.m[3 * i + j] = Rc.m[3 * j + i];
  const T bound = (T)(1.7320508075688772 * PBG_CUBE_HALF);  // circumradius
#pragma unroll 1
  for (int g = 0; g < R::NCG; g++) {
    const T r = (T)R::cgeom_r[g];
    const f3 p0 = mul(Rt, G0[g] - xc), p1 = mul(Rt, G1[g] - xc), d = p1 - p0;
    const T dd = dot3(d, d);
    const T t0 = dd > T(1e-12) ? tmin(tmax(-dot3(p0, d) / dd, T(0)), T(1)) : T(0);
    if (!(norm3(p0 + t0 * d) < bound + r + thr)) continue;
    T t = 0.f;
    if (dd > T(1e-12)) {
      const T phi = T(0.6180339887498949);
      T a = 0.f, bb = 1.f;
      T x1 = bb - phi * (bb - a), x2 = a + phi * (bb - a);
      T f1 = box_sd(p0 + x1 * d, h), f2 = box_sd(p0 + x2 * d, h);
#pragma unroll 1
      for (int it = 0; it < PBG_CUBE_GS_ITERS; it++) {
        if (f1 <= f2) { bb = x2; x2 = x1; f2 = f1; x1 = bb - phi * (bb - a); f1 = box_sd(p0 + x1 * d, h); }
        else { a = x1; x1 = x2; f1 = f2; x2 = a + phi * (bb - a); f2 = box_sd(p0 + x2 * d, h); }
      }
      t = T(0.5f) * (a + bb);
    }
    const f3 ps = p0 + t * d;
    const T dist = box_sd(ps, h) - r;
    if (!(dist < thr)) continue;
    f3 nb, qb;
    const T qx = tabs(ps.x) - h, qy = tabs(ps.y) - h, qz = tabs(ps.z) - h;
    if (tmax(qx, tmax(qy, qz)) > T(0)) {
      qb = mk3<T>(tmin(tmax(ps.x, -h), h), tmin(tmax(ps.y, -h), h), tmin(tmax(ps.z, -h), h));
      const f3 dv = ps - qb;
      const T l = norm3(dv);
      nb = l > T(1e-9) ? (T(1) / l) * dv : mk3<T>(0, 0, 1);
    } else {
      const int ax = (qx >= qy && qx >= qz) ? 0 : (qy >= qz ? 1 : 2);
      const T cc = ax == 0 ? ps.x : (ax == 1 ? ps.y : ps.z);
      const T sg = cc < T(0) ? T(-1) : T(1);
      nb = mk3<T>(ax == 0 ? sg : T(0), ax == 1 ? sg : T(0), ax == 2 ? sg : T(0));
      qb = mk3<T>(ax == 0 ? sg * h : ps.x, ax == 1 ? sg * h : ps.y, ax == 2 ? sg * h : ps.z);
    }
    csig += pbg_contact_hash(sub, (uint32_t)(R::NS + R::NPAIR + 8 + g));
    const f3 nrm = mul(Rc, nb);
    const f3 PA = xc + mul(Rc, ps) - r * nrm, PB = xc + mul(Rc, qb);
    f3 t1, t2;  // btPlaneSpace1(nrm)
    if (tabs(nrm.z) > T(0.7071067811865476)) {
      const T a2 = nrm.y * nrm.y + nrm.z * nrm.z, kinv = fast_rsq(a2);
      t1 = mk3<T>(0, -nrm.z * kinv, nrm.y * kinv);
      t2 = mk3<T>(a2 * kinv, -nrm.x * t1.z, nrm.x * t1.y);
    } else {
      const T a2 = nrm.x * nrm.x + nrm.y * nrm.y, kinv = fast_rsq(a2);
      t1 = mk3<T>(-nrm.y * kinv, nrm.x * kinv, 0);
      t2 = mk3<T>(-nrm.z * t1.y, nrm.z * t1.x, a2 * kinv);
    }
    const int lnk = R::cgeom_link[g];
    const uint32_t ma = lnk >= 0 ? R::link_chain_mask[lnk] : 0u;
    const f3 rA = PA - O, rB = PB - xc;
#pragma unroll 1
    for (int dir = 0; dir < 3; dir++) {
      const f3 nd = dir == 0 ? nrm : (dir == 1 ? t1 : t2);
      const f3 mA = cross3(rA, nd), mB = cross3(rB, nd);
      T y[NY];
      T D2 = 0.f;
#pragma unroll
      for (int i = 0; i < N; i++) {
        const int di = D::dof_of(i);
        const bool inA = di < 0 || ((ma >> di) & 1u);
        T tt = inA ? dot3(nd, sv[i]) + dot3(mA, sw[i]) : T(0);
#pragma unroll
        for (int kk = 0; kk < i; kk++)
          if (D::coupled(i, kk)) tt -= L[D::lidx(i, kk)] * y[kk];
        y[i] = tt * Ld[i];
        D2 += y[i] * y[i];
      }
      y[N] = -nd.x * rm; y[N + 1] = -nd.y * rm; y[N + 2] = -nd.z * rm;
      y[N + 3] = -mB.x * rI; y[N + 4] = -mB.y * rI; y[N + 5] = -mB.z * rI;
#pragma unroll
      for (int i = N; i < NY; i++) D2 += y[i] * y[i];
      rw.put(Rows<R, LS>::NRC * nc + dir, y, D2 > T(1e-12) ? fast_rcp(D2) : T(0), dir == 0 ? pos_target(dist, P.k_contact, P.k_sep) : T(0));
    }
    rw.mu(nc) = (T)R::cgeom_mu[g];
    nc++;
  }
  return nc;
}

template <class R, int LS>
PBG_DEV int substep(State<R>& s, const real_t<R>* tau, uint32_t* slot_active, const Rows<R, LS>& rw, uint32_t sub,
                    uint32_t& csig, const SimPT<real_t<R>>& P SUB_STAMP_ARGS) {
  using D = Dims<R>;
  using T = real_t<R>;
  using f3 = V3<T>;
  constexpr int NJ = R::NJ, N = R::NDOF;
  constexpr int NY = D::NY;  // rows and u: the robot's N (+ HumanoidFlagrunHarder's cube 6)
  T L[D::NNZ];  // coupled lower-triangle entries only (packed, compile-time indexed)
  T Ld[N], nu[N], u[NY];
  dynamics<R>(s, tau, L, Ld, nu, u, P SUB_STAMP_PASS);
  cube_unconstrained<R>(s, u + N, P);
  f3 O;
  STAMP(2)
  // --- constraint rows: joint limits, contact normals, frictions (Bullet order) ---------
  static_for<0, D::NLIM>([&](auto li_c) {
    constexpr int li = decltype(li_c)::value;
    constexpr int d = D::LIM.v[li][0], np = D::LIM.v[li][1], off = D::LIM.v[li][2];
    constexpr int gd = D::gj(d);
    // y = L^-1 e_gd, non-zero only on the pattern (the dof, its ancestors, the base)
    T y[N];
#pragma unroll
    for (int i = 0; i < N; i++) {
      if (i < gd || !D::coupled(i, gd)) { y[i] = 0.f; continue; }
      T t = i == gd ? 1.f : 0.f;
#pragma unroll
      for (int kk = gd; kk < i; kk++)
        if (D::coupled(i, kk) && D::coupled(kk, gd)) t -= L[D::lidx(i, kk)] * y[kk];
      y[i] = t * Ld[i];
    }
    T D2 = 0.f;
#pragma unroll
    for (int i = 0; i < N; i++) { D2 += y[i] * y[i]; }
    const T meff = D2 > T(1e-12) ? fast_rcp(D2) : T(0);
    // lower row J = +e_d (pos = q - lo), upper row J = -e_d (pos = hi - q)
    const T plo = s.q[d] - (T)R::dof_lower[d], phi = (T)R::dof_upper[d] - s.q[d];
    const T tlo = pos_target(plo, P.k_limit, P.k_sep);
    const T thi = pos_target(phi, P.k_limit, P.k_sep);
#pragma unroll
    for (int i = 0; i < N; i++)
      if (D::LIMPOS.v[li][i] >= 0) rw.lim(off + D::LIMPOS.v[li][i]) = y[i];
    rw.lim(off + np) = meff;
    rw.lim(off + np + 1) = tlo;
    rw.lim(off + np + 2) = thi;
    rw.lim(off + np + 3) = 0.f;
    rw.lim(off + np + 4) = 0.f;
  });
  STAMP(3)
  constexpr int first_normal = 0;
  constexpr int NRC = Rows<R, LS>::NRC;  // rows per contact
  static_assert(R::restitution == 0.0 || (R::NPAIR == 0 && !R::harder), "restitution: robot-floor contacts only");
  int nc = 0;
  // positions, joint axes and motion vectors again: recomputing them is cheaper than
  // keeping phase A's copies live through the factorisation
  Kin<R> k;
  f3 sw[N], sv[N];
  kin_motion<R>(s, k, sw, sv, O);
  // contact rows are staged: normals first (in contact order), frictions after.
  // Each contact stores its normal row now and its two friction rows at MAXROWS-space
  // offsets after all normals; friction rows are compacted once nc is known.
  static_for<0, R::NS>([&](auto sl_c) {
    constexpr int sl = decltype(sl_c)::value;
    constexpr int b = R::slot_link[sl] + 1;
    const f3 cc = k.x[b] + mulc(k.Rm[b], (T)R::slot_point[sl][0], (T)R::slot_point[sl][1], (T)R::slot_point[sl][2]);
    const T rad = (T)R::slot_radius[sl];
    const T dist = cc.z - rad;
    const bool act = dist < (T)PBG_CONTACT_THRESHOLD;
    slot_active[sl] = act;
    if (!act) return;
    csig += pbg_contact_hash(sub, (uint32_t)sl);
    const f3 cp = mk3<T>(cc.x, cc.y, cc.z - rad);
    const f3 rP = cp - O;
    const int lnk = R::slot_link[sl];
#pragma unroll
    for (int dir = 0; dir < NRC; dir++) {
      // n = +z, t1 = (0,-1,0), t2 = (1,0,0)  (btPlaneSpace1 of +z); rows 3-5 (NRC = 6): the
      // spinning and rolling rows about n, t1, t2, an angular Jacobian
      const int ax = dir < 3 ? dir : dir - 3;
      const f3 nd = ax == 0 ? mk3<T>(0, 0, 1) : (ax == 1 ? mk3<T>(0, -1, 0) : mk3<T>(1, 0, 0));
      const f3 mm = cross3(rP, nd);
      T Jr[N];
#pragma unroll
      for (int i = 0; i < N; i++)
        Jr[i] = !D::in_chain(i, lnk) ? T(0) : (dir < 3 ? dot3(nd, sv[i]) + dot3(mm, sw[i]) : dot3(nd, sw[i]));
      T y[NY];
#pragma unroll
      for (int i = N; i < NY; i++) y[i] = 0.f;
#pragma unroll
      for (int i = 0; i < N; i++) {
        if (!D::in_chain(i, lnk)) { y[i] = 0.f; continue; }
        T t = Jr[i];
#pragma unroll
        for (int kk = 0; kk < i; kk++)
          if (D::coupled(i, kk) && D::in_chain(kk, lnk)) t -= L[D::lidx(i, kk)] * y[kk];
        y[i] = t * Ld[i];
      }
      T D2 = 0.f;
#pragma unroll
      for (int i = 0; i < N; i++) { D2 += y[i] * y[i]; }
      T tgt = dir == 0 ? (pos_target(dist, P.k_contact, P.k_sep)) : T(0);
      if constexpr (R::restitution > 0.0) {
        // restitution (sim_params.h): e (-v_n) when |v_n| >= the threshold, v_n = J nu = y.u before the solve
        if (dir == 0) {
          T vn = 0.f;
#pragma unroll
          for (int i = 0; i < N; i++) vn += y[i] * u[i];
          const T rest = tabs(vn) < T(PBG_RESTITUTION_VELOCITY_THRESHOLD) ? T(0) : T(R::restitution) * -vn;
          tgt += rest > T(0) ? rest : T(0);
        }
      }
      rw.put(first_normal + NRC * nc + dir, y, D2 > T(1e-12) ? fast_rcp(D2) : T(0), tgt);
    }
    rw.mu(nc) = (T)R::slot_mu[sl];
    nc++;
  });
  // self-collision pairs (capsule-capsule / sphere) -- Humanoid.  World endpoints per
  // geom are computed once (unrolled); the pair loop itself runs at run time.
  if constexpr (R::NPAIR > 0) {
    f3 G0[R::NG], G1[R::NG];
#pragma unroll
    for (int gg = 0; gg < R::NG; gg++) {
      const int b = R::geom_link[gg] + 1;
      G0[gg] = k.x[b] + mulc(k.Rm[b], (T)R::geom_p0[gg][0], (T)R::geom_p0[gg][1], (T)R::geom_p0[gg][2]);
      G1[gg] = k.x[b] + mulc(k.Rm[b], (T)R::geom_p1[gg][0], (T)R::geom_p1[gg][1], (T)R::geom_p1[gg][2]);
    }
#pragma unroll 1
    for (int pp = 0; pp < R::NPAIR; pp++) {
      const int ga = R::pair_ga[pp], gb = R::pair_gb[pp];
      const f3 a0 = G0[ga], a1 = G1[ga], b0 = G0[gb], b1 = G1[gb];
      // broad phase: capsules whose bounding spheres are beyond the contact threshold
      // cannot touch (bound = half lengths + radii + threshold, compile-time per pair)
      const f3 dc = (a0 + a1) - (b0 + b1);  // twice the centre distance
      if (dot3(dc, dc) > D::PAIR_BOUND2.v[pp][0]) continue;
      const f3 d1 = a1 - a0, d2 = b1 - b0, r0 = a0 - b0;
      const T aa = dot3(d1, d1), ee = dot3(d2, d2), ff = dot3(d2, r0);
      T ss, tt;
      const T eps = T(1e-12);
      if (aa <= eps && ee <= eps) { ss = tt = 0.f; }
      else if (aa <= eps) { ss = 0.f; tt = tmin(tmax(ff / ee, T(0)), T(1)); }
      else {
        const T cc2 = dot3(d1, r0);
        if (ee <= eps) { tt = 0.f; ss = tmin(tmax(-cc2 / aa, T(0)), T(1)); }
        else {
          const T bb2 = dot3(d1, d2), den = aa * ee - bb2 * bb2;
          ss = den > eps ? tmin(tmax((bb2 * ff - cc2 * ee) / den, T(0)), T(1)) : T(0);
          tt = (bb2 * ss + ff) / ee;
          if (tt < T(0)) { tt = 0.f; ss = tmin(tmax(-cc2 / aa, T(0)), T(1)); }
          else if (tt > T(1)) { tt = 1.f; ss = tmin(tmax((bb2 - cc2) / aa, T(0)), T(1)); }
        }
      }
      const f3 ca = a0 + ss * d1, cb = b0 + tt * d2;
      const f3 dv = ca - cb;
      const T dd = norm3(dv);
      const T ra = (T)R::geom_r[ga], rb = (T)R::geom_r[gb];
      const T dist = dd - ra - rb;
      if (!(dist < (T)PBG_CONTACT_THRESHOLD)) continue;
      csig += pbg_contact_hash(sub, (uint32_t)(R::NS + pp));
      const f3 nrm = dd > T(1e-9) ? fast_rcp(dd) * dv : mk3<T>(0, 0, 1);
      const f3 PA = ca - ra * nrm, PB = cb + rb * nrm;
      f3 t1, t2;  // btPlaneSpace1(nrm)
      if (tabs(nrm.z) > T(0.7071067811865476)) {
        const T a2 = nrm.y * nrm.y + nrm.z * nrm.z, kinv = fast_rsq(a2);
        t1 = mk3<T>(0, -nrm.z * kinv, nrm.y * kinv);
        t2 = mk3<T>(a2 * kinv, -nrm.x * t1.z, nrm.x * t1.y);
      } else {
        const T a2 = nrm.x * nrm.x + nrm.y * nrm.y, kinv = fast_rsq(a2);
        t1 = mk3<T>(-nrm.y * kinv, nrm.x * kinv, 0);
        t2 = mk3<T>(-nrm.z * t1.y, nrm.z * t1.x, a2 * kinv);
      }
      const uint32_t ma = R::link_chain_mask[R::geom_link[ga]], mb = R::link_chain_mask[R::geom_link[gb]];
      const f3 rA = PA - O, rB = PB - O;
#pragma unroll 1
      for (int dir = 0; dir < 3; dir++) {
        const f3 nd = dir == 0 ? nrm : (dir == 1 ? t1 : t2);
        const f3 mA = cross3(rA, nd), mB = cross3(rB, nd);
        T y[NY];
#pragma unroll
        for (int i = N; i < NY; i++) y[i] = 0.f;
        T D2 = 0.f;
#pragma unroll
        for (int i = 0; i < N; i++) {
          const int di = D::dof_of(i);
          const bool inA = di < 0 || ((ma >> di) & 1u), inB = di < 0 || ((mb >> di) & 1u);
          T t = 0.f;
          if (inA) t += dot3(nd, sv[i]) + dot3(mA, sw[i]);
          if (inB) t -= dot3(nd, sv[i]) + dot3(mB, sw[i]);
#pragma unroll
          for (int kk = 0; kk < i; kk++)
            if (D::coupled(i, kk)) t -= L[D::lidx(i, kk)] * y[kk];
          y[i] = t * Ld[i];
          D2 += y[i] * y[i];
         
        }
        rw.put(first_normal + NRC * nc + dir, y, D2 > T(1e-12) ? fast_rcp(D2) : T(0),
               dir == 0 ? (pos_target(dist, P.k_contact, P.k_sep)) : T(0));
      }
      rw.mu(nc) = (T)R::pair_mu[pp];
      nc++;
    }
  }
  if constexpr (R::harder) nc = cube_contacts<R, LS>(s, k, sw, sv, O, L, Ld, rw, sub, csig, P, nc);

  STAMP(4)
  // --- PGS: 5 sweeps in u-space (gym_locomotion_envs -> scene_bases.py:65 numSolverIterations=5)
  for (int it = 0; it < P.iterations; it++) {
    // joint limits: lower then upper row of each limited dof, sharing y (compile-time)
    static_for<0, D::NLIM>([&](auto li_c) {
      constexpr int li = decltype(li_c)::value;
      constexpr int np = D::LIM.v[li][1], off = D::LIM.v[li][2];
      T yv[N];
      T acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < N; i++) {
        const int j = D::LIMPOS.v[li][i];
        if (j < 0) continue;
        yv[i] = rw.lim(off + j);
        acc[j & 3] += yv[i] * u[i];
      }
      const T meff = rw.lim(off + np), tlo = rw.lim(off + np + 1), thi = rw.lim(off + np + 2);
      const T llo = rw.lim(off + np + 3), lhi = rw.lim(off + np + 4);
      const T yu = (acc[0] + acc[1]) + (acc[2] + acc[3]);
      const T nlo = clampf(llo + meff * (tlo - yu), T(0), (T)PBG_LIMIT_MAX_IMPULSE);
      const T dlo = nlo - llo;
      // upper row sees u after the lower update: (-y).u' = -(yu + (y.y) dlo) = -(yu + dlo / meff)
      const T yu2 = meff > T(0) ? yu + dlo * fast_rcp(meff) : yu;
      const T nhi = clampf(lhi + meff * (thi + yu2), T(0), (T)PBG_LIMIT_MAX_IMPULSE);
      const T dhi = nhi - lhi;
      rw.lim(off + np + 3) = nlo;
      rw.lim(off + np + 4) = nhi;
      const T dl = dlo - dhi;
#pragma unroll
      for (int i = 0; i < N; i++)
        if (D::LIMPOS.v[li][i] >= 0) u[i] += yv[i] * dl;
    });
    for (int c = 0; c < nc; c++) rw.solve(first_normal + NRC * c, u, T(0), T(3.0e38f));   // contact normals
    if constexpr (NRC == 6) {  // spinning, rolling: +-mu_t lambda_n, before the lateral friction (oracle order)
      for (int c = 0; c < nc; c++) {
        const T ln = rw.lam(first_normal + NRC * c);
        if (!(ln > T(0))) continue;
        const T ls = (T)R::spin_mu * ln, lr = (T)R::roll_mu * ln;
        rw.solve(first_normal + NRC * c + 3, u, -ls, ls);
        rw.solve(first_normal + NRC * c + 4, u, -lr, lr);
        rw.solve(first_normal + NRC * c + 5, u, -lr, lr);
      }
    }
    for (int c = 0; c < nc; c++) {                                                  // frictions
      const T ln = rw.lam(first_normal + NRC * c);
      if (!(ln > T(0))) continue;  // [EXT] friction rows only under a positive normal impulse
      const T lim = rw.mu(c) * ln;
      rw.solve(first_normal + NRC * c + 1, u, -lim, lim);
      rw.solve(first_normal + NRC * c + 2, u, -lim, lim);
    }
  }

  STAMP(5)
  integrate<R>(s, L, Ld, u, nu, P);
  cube_integrate<R>(s, u + N, P);
  STAMP(6)
  return nc;
}

// ------------------------------------------------------------------ numpy-exact pack (float64)
#pragma clang fp contract(off)
PBG_DEV double np_sum_f64(const double* a, int n) {
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; i++) res += a[i];
    return 0.0 + res;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; j++) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; i++) res += a[i];
  return 0.0 + res;
}
// The same sums for a compile-time length (register-resident operands, no scratch).
template <int N, class F>
PBG_DEV F np_sum_n(const F* a) {
  if constexpr (N < 8) {
    F res = F(0);
#pragma unroll
    for (int i = 0; i < N; i++) res += a[i];
    return F(0) + res;
  } else {
    F r[8];
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] = a[j];
#pragma unroll
    for (int i = 8; i < N - (N % 8); i += 8)
#pragma unroll
      for (int j = 0; j < 8; j++) r[j] += a[i + j];
    F res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (int i = N - (N % 8); i < N; i++) res += a[i];
    return F(0) + res;
  }
}
PBG_DEV float clip5(float v) { return v < -5.0f ? -5.0f : (v > 5.0f ? 5.0f : v); }

// Inputs of the walker pack -- what the reference reads back from pybullet after the step.
template <class R>
struct PackIn {
  double part_x[R::NP + 1], part_y[R::NP + 1];
  int n_parts;
  double quat[4], pos[3], vel[3];
  double jq[R::NO > 0 ? R::NO : 1], jqd[R::NO > 0 ? R::NO : 1];
  float feet_prev[R::NF > 0 ? R::NF : 1];
  uint32_t feet_new;  // bitmask
  double potential_old, initial_z;  // initial_z NaN: take from this calc_state
  double target_x = PBG_WALK_TARGET_X, target_y = PBG_WALK_TARGET_Y;  // robot.walk_target_x/y
  double avel[3] = {0.0, 0.0, 0.0};  // base angular velocity (MuJoCo-observation walkers)
  double head_z = 0.0;               // Atlas: the head part's height (alive_bonus)
  double env_dt = R::dt_sub * R::substeps;  // Scene.dt (SimP::env_dt; the pack kernel: defaults)
};
struct PackOut {
  double reward, potential, initial_z, dist;  // dist: walk_target_dist
  double terms[5];  // the reference's self.rewards list (the terms `reward` sums), zero-padded
  double pitch;                               // body_rpy[1]
  int at_limit;                               // joints_at_limit
  uint32_t feet_out;  // bitmask
  bool done;
  double body_xyz[3];                         // robot.body_xyz (HumanoidFlagrunHarder)
};

// robot_locomotors.py:31-64 calc_state + gym_locomotion_envs.py:59-114 reward/done.
// GEN: any part count (golden-vector pack_kernel); otherwise the step's NP or NP + 1 parts.
// Broadcast lane K of each DPP quad (a float64 as two dword moves).
template <int K>
PBG_DEV double quad_bcast_f64(double x) {
  constexpr int CTRL = K * 85;  // quad_perm [K, K, K, K]
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// Q = 4: the four lanes of each DPP quad hold the same env and identical inputs (quad and
// gang kernels); the float64 transcendentals are dealt over them -- lane 0 roll, 1 pitch,
// 2 yaw, 3 target angle (atan2 / asin), then lanes 0-1 sin/cos(-yaw) and 2-3 sin/cos(ang)
// -- and broadcast back: the same library calls on the same arguments, so the same bits as
// Q = 1, for two atan2 and one sin/cos pair less per pack.
template <class R, bool GEN = false, int Q = 1>
PBG_DEV void walker_pack(const PackIn<R>& in, const float* act, float* obs, PackOut& out, int lane = 0) {
  float j[2 * (R::NO > 0 ? R::NO : 1)];
#pragma unroll
  for (int i = 0; i < R::NO; i++) {
    const int d = R::obs_dof[i];
    double pos = in.jq[i], vel = in.jqd[i];
    if (R::dof_lower[d] < R::dof_upper[d]) {
      const double mid = 0.5 * (R::dof_lower[d] + R::dof_upper[d]);
      pos = 2 * (pos - mid) / (R::dof_upper[d] - R::dof_lower[d]);
    }
    vel *= R::obs_vel_scale[i];
    j[2 * i] = (float)pos;
    j[2 * i + 1] = (float)vel;
  }
  int at_limit = 0;
#pragma unroll
  for (int i = 0; i < R::NO; i++) at_limit += fabsf(j[2 * i]) > PBG_JOINT_AT_LIMIT;
  double bx, by;
  if constexpr (GEN) {
    bx = np_sum_f64(in.part_x, in.n_parts) / (double)in.n_parts;
    by = np_sum_f64(in.part_y, in.n_parts) / (double)in.n_parts;
  } else if (in.n_parts == R::NP + 1) {
    bx = np_sum_n<R::NP + 1>(in.part_x) / (double)(R::NP + 1);
    by = np_sum_n<R::NP + 1>(in.part_y) / (double)(R::NP + 1);
  } else {
    bx = np_sum_n<R::NP>(in.part_x) / (double)R::NP;
    by = np_sum_n<R::NP>(in.part_y) / (double)R::NP;
  }
  const double bz = in.pos[2];
  const double* q = in.quat;
  const double sqx = q[0] * q[0], sqy = q[1] * q[1], sqz = q[2] * q[2], squ = q[3] * q[3];
  const double ry = 2 * (q[1] * q[2] + q[3] * q[0]), rx = squ - sqx - sqy + sqz;
  const double sarg = -2 * (q[0] * q[2] - q[3] * q[1]);
  const double yy = 2 * (q[0] * q[1] + q[3] * q[2]), yx = squ + sqx - sqy - sqz;
  const double z0 = isnan(in.initial_z) ? bz : in.initial_z;
  const double dy = in.target_y - by, dx = in.target_x - bx;
  double roll, pitch, yaw, theta, cy, sy, sa, ca;
  if constexpr (Q == 4) {
    const int k = lane & 3;
    double r;
    if (k == 1) r = sarg <= -1.0 ? -0.5 * 3.141592538 : (sarg >= 1.0 ? 0.5 * 3.141592538 : asin(sarg));
    else r = atan2(k == 0 ? ry : (k == 2 ? yy : dy), k == 0 ? rx : (k == 2 ? yx : dx));
    roll = quad_bcast_f64<0>(r);
    pitch = quad_bcast_f64<1>(r);
    yaw = quad_bcast_f64<2>(r);
    theta = quad_bcast_f64<3>(r);
    const double arg = k < 2 ? -yaw : theta - yaw;
    const double sv = sin(arg), cv = cos(arg);
    sy = quad_bcast_f64<0>(sv);
    cy = quad_bcast_f64<0>(cv);
    sa = quad_bcast_f64<2>(sv);
    ca = quad_bcast_f64<2>(cv);
  } else {
    (void)lane;
    roll = atan2(ry, rx);
    pitch = sarg <= -1.0 ? -0.5 * 3.141592538 : (sarg >= 1.0 ? 0.5 * 3.141592538 : asin(sarg));
    yaw = atan2(yy, yx);
    theta = atan2(dy, dx);
    cy = cos(-yaw);
    sy = sin(-yaw);
    sa = sin(theta - yaw);
    ca = cos(theta - yaw);
  }
  const double dist = sqrt(dy * dy + dx * dx);
  const double vx = cy * in.vel[0] + -sy * in.vel[1] + 0.0 * in.vel[2];
  const double vy = sy * in.vel[0] + cy * in.vel[1] + 0.0 * in.vel[2];
  const double vz = 0.0 * in.vel[0] + 0.0 * in.vel[1] + 1.0 * in.vel[2];
  const float more[8] = {(float)(bz - z0), (float)sa, (float)ca, (float)(0.3 * vx),
                         (float)(0.3 * vy), (float)(0.3 * vz), (float)roll, (float)pitch};
  bool has_nan = false;
  int o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) { obs[o] = clip5(more[i]); has_nan |= isnan(obs[o]); o++; }
#pragma unroll
  for (int i = 0; i < 2 * R::NO; i++) { obs[o] = clip5(j[i]); has_nan |= isnan(obs[o]); o++; }
#pragma unroll
  for (int i = 0; i < R::NF; i++) { obs[o] = clip5(in.feet_prev[i]); o++; }
  out.initial_z = z0;
  out.dist = dist;
  out.pitch = pitch;
  out.at_limit = at_limit;
  out.body_xyz[0] = bx; out.body_xyz[1] = by; out.body_xyz[2] = bz;
  out.potential = -dist / in.env_dt;  // robot_locomotors.py:79; scene_bases.py:17
  uint32_t fb = 0;
#pragma unroll
  for (int i = 0; i < R::NF; i++) fb |= (in.feet_prev[i] != 0.f ? 1u : 0u) << i;
  out.feet_out = fb;
#pragma unroll
  for (int i = 0; i < 5; i++) out.terms[i] = 0.0;
  if (!act) { out.reward = 0.0; out.done = false; return; }
  const float s0 = obs[0];
  double alive;
  if constexpr (R::alive == 0) {  // Hopper robot_locomotors.py:89-90
    const double z = (double)s0 + z0;
    alive = (z > 0.8 && fabs(pitch) < 1.0) ? 1.0 : -1.0;
  } else if constexpr (R::alive == 1) {  // HalfCheetah :116-118 (previous-step feet_contact)
    alive = (fabs(pitch) < 1.0 && !(in.feet_prev[1] != 0) && !(in.feet_prev[2] != 0) &&
             !(in.feet_prev[4] != 0) && !(in.feet_prev[5] != 0)) ? 1.0 : -1.0;
  } else if constexpr (R::alive == 2) {  // Ant :137-138
    const double z = (double)s0 + z0;
    alive = z > 0.26 ? 1.0 : -1.0;
  } else if constexpr (R::alive == 13) {  // Atlas :313-324: +4 - knees at limit if head z > 1.3
    int knees = 0;
#pragma unroll
    for (int k = 0; k < 2; k++) knees += fabsf(j[2 * R::knee_obs[k]]) > PBG_JOINT_AT_LIMIT;
    alive = in.head_z > 1.3 ? (double)(4 - knees) : -1.0;
  } else {  // Humanoid :191-192; np.float32 + 0.8 stays float32 (NEP 50)
    const float z = s0 + (float)z0;
    alive = z > 0.78f ? 2.0 : -1.0;
  }
  out.done = alive < 0 || has_nan;
  const double progress = out.potential - in.potential_old;
  out.feet_out = in.feet_new;
  float tmp[R::NA];
#pragma unroll
  for (int i = 0; i < R::NA; i++) tmp[i] = fabsf(act[i] * j[2 * i + 1]);
  const float mean_e = np_sum_n<R::NA>(tmp) / (float)R::NA;
#pragma unroll
  for (int i = 0; i < R::NA; i++) tmp[i] = act[i] * act[i];
  const float mean_s = np_sum_n<R::NA>(tmp) / (float)R::NA;
  double elec = R::electricity_cost * (double)mean_e;
  elec += R::stall_torque_cost * (double)mean_s;
  const double jal = R::joints_at_limit_cost * (double)at_limit;
  out.reward = ((((0.0 + alive) + progress) + elec) + jal) + 0.0;
  // gym_locomotion_envs.py:99-105 [alive, progress, electricity, joints_at_limit, feet_collision]
  out.terms[0] = alive; out.terms[1] = progress; out.terms[2] = elec; out.terms[3] = jal;
}

// HumanoidFlagrun walk target (robot_locomotors.py:195-226).
struct Flag {
  double tx, ty;  // walk_target_x / _y (float64, as the reference's)
  int timeout;    // flag_timeout
  int count;      // draws so far: the Philox counter of the next draw (never reset)
};
// flag_reposition (:203-216): np_random.uniform(+-halflen), uniform(+-halfwidth), times
// more_compact; here Philox4x32-10 keyed by the seed, counter (global env, draw index).
PBG_DEV void flag_draw(const Buffers& B, int e, Flag& f) {
  u4 ctr = {(uint32_t)(B.env_offset + e), (uint32_t)f.count, 0xF1A6u, 0x5EEDu};
  const u4 r = philox4x32_10(ctr, (uint32_t)B.seed, (uint32_t)(B.seed >> 32));
  f.tx = (-PBG_STADIUM_HALFLEN + 2.0 * PBG_STADIUM_HALFLEN * (double)u01(r.x)) * PBG_FLAG_COMPACT;
  f.ty = (-PBG_STADIUM_HALFWIDTH + 2.0 * PBG_STADIUM_HALFWIDTH * (double)u01(r.y)) * PBG_FLAG_COMPACT;
  f.timeout = B.sp.flag_timeout;
  f.count++;
}
// calc_state with HumanoidFlagrun's bookkeeping (:219-226): count the timeout down, pack
// against the current flag, and if the target is within 1 m or the timeout ran out, re-draw
// (`redraw(f)`) and pack again against the new flag.  Other robots: plain walker_pack.
// HumanoidFlagrunHarder bookkeeping (robot_locomotors.py:230-302); crawl_start NaN = None.
struct HarderBk {
  int frame, onground, launches;
  double crawl_start, crawl_ignored;
};
// potential_leak (:275-278): clip(body z, 0, 0.8) / 0.8 + 1 (NaN passes np.clip)
PBG_DEV double potential_leak(double z) {
  const double c = z < 0.0 ? 0.0 : (z > PBG_HARDER_GROUND_Z ? PBG_HARDER_GROUND_Z : z);
  return c / 0.8 + 1.0;
}
// calc_potential (:280-302) from Humanoid.calc_potential's fp and body_xyz[2]; every call
// updates the crawl bookkeeping (env reset, _step, and the flag re-draw's robot.potential)
PBG_DEV double harder_potential(HarderBk& h, double fp, double bz) {
  if (bz < PBG_HARDER_GROUND_Z) {
    if (isnan(h.crawl_start)) h.crawl_start = fp - h.crawl_ignored;
    h.crawl_ignored = fp - h.crawl_start;
    fp = h.crawl_start;
  } else {
    fp -= h.crawl_ignored;
    h.crawl_start = __builtin_nan("");
  }
  return fp + potential_leak(bz) * 100;
}

template <class R, int Q = 1, class Redraw>
PBG_DEV void flag_pack(PackIn<R>& in, const float* act, float* obs, PackOut& po, Flag& f, Redraw&& redraw, int lane = 0,
                       HarderBk* hb = nullptr) {
  if constexpr (R::flagrun) {
    f.timeout -= 1;
    in.target_x = f.tx; in.target_y = f.ty;
    walker_pack<R, false, Q>(in, act, obs, po, lane);
    if (po.dist < 1.0 || f.timeout <= 0) {  // env-uniform: a quad takes it together
      redraw(f);
      in.target_x = f.tx; in.target_y = f.ty;
      walker_pack<R, false, Q>(in, act, obs, po, lane);
      if constexpr (R::harder)  // self.potential = self.calc_potential() (:225) on the robot
        if (hb) (void)harder_potential(*hb, po.potential, po.body_xyz[2]);
    }
  } else {
    (void)hb;
    (void)f; (void)redraw;
    walker_pack<R, false, Q>(in, act, obs, po, lane);
  }
}
template <class R>
PBG_DEV Flag load_flag(const Buffers& B, int e) {
  Flag f = {0.0, 0.0, 0, 0};
  if constexpr (R::flagrun) { f.tx = B.tgt[e]; f.ty = B.tgt[B.n + e]; f.timeout = B.ftm[e]; f.count = B.ftm[B.n + e]; }
  return f;
}
template <class R>
PBG_DEV void store_flag(const Buffers& B, int e, const Flag& f) {
  if constexpr (R::flagrun) { B.tgt[e] = f.tx; B.tgt[B.n + e] = f.ty; B.ftm[e] = f.timeout; B.ftm[B.n + e] = f.count; }
}
template <class R>
PBG_DEV HarderBk load_harder(const Buffers& B, int e) {
  HarderBk h = {0, 0, 0, 0.0, 0.0};
  if constexpr (R::harder) {
    h.frame = B.hki[e]; h.onground = B.hki[B.n + e]; h.launches = B.hki[2 * B.n + e];
    h.crawl_start = B.hkd[e]; h.crawl_ignored = B.hkd[B.n + e];
  }
  return h;
}
template <class R>
PBG_DEV void store_harder(const Buffers& B, int e, const HarderBk& h) {
  if constexpr (R::harder) {
    B.hki[e] = h.frame; B.hki[B.n + e] = h.onground; B.hki[2 * B.n + e] = h.launches;
    B.hkd[e] = h.crawl_start; B.hkd[B.n + e] = h.crawl_ignored;
  }
}
// The cube launch of alive_bonus (:251-265) in float64: angle U(-3.14, 3.14), speed U(20, 30),
// jitter U(-1, 1)^3 (np_random there; Philox4x32-10 here, keyed by the seed, counter (global
// env, launch index, 0xC0BE / 0xC0BF, 0x5EED)); d (nullable) = recorded draws (golden tests).
// Writes the cube's position and velocity (orientation kept, angular velocity 0).
PBG_DEV void harder_launch(const Buffers& B, int e, HarderBk& h, const double* body_xyz, const double* speed,
                           double* pos, double* vel, const double* draws) {
  double d[5];
  if (draws) {
#pragma unroll
    for (int i = 0; i < 5; i++) d[i] = draws[i];
  } else {
    u4 c = {(uint32_t)(B.env_offset + e), (uint32_t)h.launches, 0xC0BEu, 0x5EEDu};
    u4 c2 = {(uint32_t)(B.env_offset + e), (uint32_t)h.launches, 0xC0BFu, 0x5EEDu};
    const u4 r = philox4x32_10(c, (uint32_t)B.seed, (uint32_t)(B.seed >> 32));
    const u4 r2 = philox4x32_10(c2, (uint32_t)B.seed, (uint32_t)(B.seed >> 32));
    d[0] = -3.14 + (3.14 - -3.14) * (double)u01(r.x);
    d[1] = 20.0 + (30.0 - 20.0) * (double)u01(r.y);
    d[2] = -1.0 + (1.0 - -1.0) * (double)u01(r.z);
    d[3] = -1.0 + (1.0 - -1.0) * (double)u01(r.w);
    d[4] = -1.0 + (1.0 - -1.0) * (double)u01(r2.x);
  }
  h.launches++;
  const double ttt = PBG_HARDER_FROM_DIST / d[1];
  double t[3], v[3];
#pragma unroll
  for (int i = 0; i < 3; i++) t[i] = body_xyz[i] + speed[i] * ttt;
  pos[0] = t[0] + PBG_HARDER_FROM_DIST * cos(d[0]);
  pos[1] = t[1] + PBG_HARDER_FROM_DIST * sin(d[0]);
  pos[2] = t[2] + 1.0;
#pragma unroll
  for (int i = 0; i < 3; i++) v[i] = t[i] - pos[i];
  const double sc = d[1] / sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
#pragma unroll
  for (int i = 0; i < 3; i++) {
    v[i] *= sc;
    vel[i] = v[i] + d[2 + i];
  }
}
// The Harder half of _step after calc_state (gym_locomotion_envs.py:59-70 with alive_bonus
// :250-273 and calc_potential :280-302): alive, done, potential, progress and the reward of po
// are redone.  Returns true when the cube was launched (pos / vel written).
template <class R>
PBG_DEV bool harder_step(const Buffers& B, int e, const PackIn<R>& in, const float* obs, PackOut& po, HarderBk& h,
                         double* pos, double* vel, const double* draws) {
  const float z = obs[0] + (float)R::initial_z_fixed;  // state[0] + initial_z (float32, NEP 50)
  bool launched = false;
  if (h.frame % PBG_HARDER_LAUNCH_EVERY == 0 && h.frame > PBG_HARDER_LAUNCH_AFTER && h.onground == 0) {
    harder_launch(B, e, h, po.body_xyz, in.vel, pos, vel, draws);
    launched = true;
  }
  if (z < (float)PBG_HARDER_GROUND_Z) h.onground += 1;
  else if (h.onground > 0) h.onground -= 1;
  h.frame += 1;
  const double alive = h.onground < PBG_HARDER_GROUND_FRAMES ? potential_leak(po.body_xyz[2]) : -1.0;
  bool done = alive < 0;
#pragma unroll
  for (int i = 0; i < R::OBS; i++) done |= isnan(obs[i]);
  po.potential = harder_potential(h, po.potential, po.body_xyz[2]);
  const double progress = po.potential - in.potential_old;
  po.terms[0] = alive; po.terms[1] = progress;
  po.reward = ((((0.0 + alive) + progress) + po.terms[2]) + po.terms[3]) + 0.0;
  po.done = done;
  return launched;
}

// MuJoCo-observation planar walkers (envs/mujoco, add_ignored_joints=True):
// calc_state = [qpos[1:], clip(qvel, -10, 10)] (HalfCheetah: qvel unclipped) over every
// ordered joint incl. the ignored root joints, float32 (mujoco robot_locomotors.py:93-102,
// 124-133, 172-181); calc_potential = (x_after - x_before) / dt of robot_body's x (:104-121);
// reward = sum([potential, alive 1.0, power_cost]) with power_cost = c * sum(a^2) in float32
// (HalfCheetah: no alive term), done per robot (mujoco gym_locomotion_envs.py:121-252).
// out.potential carries x_after (the next step's x_before).
template <class R>
PBG_DEV void mujoco_planar_pack(const double* jq, const double* jqd, double x_after, double x_before, const float* act,
                                float* obs, PackOut& out, double env_dt = R::dt_sub * R::substeps) {
  constexpr int NO = R::NO;
  constexpr float c = (float)R::qvel_clip;
  int o = 0;
#pragma unroll
  for (int i = 1; i < NO; i++) obs[o++] = (float)jq[i];
#pragma unroll
  for (int i = 0; i < NO; i++) {
    const float v = (float)jqd[i];
    obs[o++] = c > 0.f ? (v < -c ? -c : (v > c ? c : v)) : v;  // np.clip keeps NaN
  }
  out.potential = x_after; out.initial_z = 0.0; out.dist = 0.0; out.feet_out = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) out.terms[i] = 0.0;
  if (!act) { out.reward = 0.0; out.done = false; return; }
  const double potential = (x_after - x_before) / env_dt;
  float sq[R::NA];
#pragma unroll
  for (int i = 0; i < R::NA; i++) sq[i] = act[i] * act[i];
  const float power_cost = (float)R::power_cost * np_sum_n<R::NA>(sq);
  bool finite = true, small = true;
#pragma unroll
  for (int i = 0; i < R::OBS; i++) {
    finite &= isfinite(obs[i]);
    if (i >= 2) small &= fabsf(obs[i]) < 100.f;
  }
  const float height = obs[0], ang = obs[1];
  if constexpr (R::alive == 12) {  // HalfCheetah: never done; rewards [potential, power_cost]
    out.reward = (0.0 + potential) + (double)power_cost;
    out.done = false;
    out.terms[0] = potential; out.terms[1] = (double)power_cost;
  } else {  // rewards [potential, alive_bonus, power_cost] (mujoco gym_locomotion_envs.py:150-154)
    out.reward = ((0.0 + potential) + 1.0) + (double)power_cost;
    out.terms[0] = potential; out.terms[1] = 1.0; out.terms[2] = (double)power_cost;
    if constexpr (R::alive == 10)  // Hopper
      out.done = !(finite && small && height > -0.3f && fabsf(ang) < 0.2f);
    else  // Walker2D
      out.done = !(finite && small && (1.0f > height && height > -0.2f) && (-1.0f < ang && ang < 1.0f));
  }
}
template <class R>
PBG_DEV void mujoco_planar_pack_state(const State<R>& s, double x_before, const float* act, float* obs, PackOut& po,
                                      double env_dt) {
  double jq[R::NO], jqd[R::NO];
#pragma unroll
  for (int i = 0; i < R::NO; i++) { jq[i] = s.q[R::obs_dof[i]]; jqd[i] = s.qd[R::obs_dof[i]]; }
  Kin<R> k;
  fk_pos<R>(s, k);
  mujoco_planar_pack<R>(jq, jqd, (double)k.c[R::robot_body + 1].x, x_before, act, obs, po, env_dt);
}

// MuJoCo-observation Ant / Humanoid (mujoco robot_locomotors.py:210-319): WalkerBase.calc_state
// runs for its side effects (joints_at_limit, body_xyz / rpy, initial_z, walk_target_dist),
// then obs = [qpos[2:] = (z, quat x y z w, joint q), qvel = (v, w, joint qd), zeros] (float64
// in the reference, float32 through the C-ABI).  _step (mujoco gym_locomotion_envs.py:53-114):
// alive = alive_bonus(state[0] + initial_z), done = alive < 0 or a non-finite state,
// reward = sum([alive, progress, -0.1 joints_at_limit, 0]) -- no electricity term.
template <class R, bool GEN = false>
PBG_DEV void mujoco3d_pack(const PackIn<R>& in, const float* act, float* obs, PackOut& out) {
  walker_pack<R, GEN>(in, nullptr, obs, out);  // calc_state side effects (obs overwritten below)
  double st[5 + 2 * R::NO + 6];
  int o = 0;
  st[o++] = in.pos[2];
#pragma unroll
  for (int i = 0; i < 4; i++) st[o++] = in.quat[i];
#pragma unroll
  for (int i = 0; i < R::NO; i++) st[o++] = in.jq[i];
#pragma unroll
  for (int i = 0; i < 3; i++) st[o++] = in.vel[i];
#pragma unroll
  for (int i = 0; i < 3; i++) st[o++] = in.avel[i];
#pragma unroll
  for (int i = 0; i < R::NO; i++) st[o++] = in.jqd[i];
  bool finite = true;
#pragma unroll
  for (int i = 0; i < o; i++) { obs[i] = (float)st[i]; finite &= isfinite(st[i]); }
#pragma unroll
  for (int i = o; i < R::OBS; i++) obs[i] = 0.f;  // cfrc_ext / cinert / cvel / qfrc_actuator: zeros
  if (!act) { out.reward = 0.0; out.done = false; return; }  // reset: feet_contact stays as packed
  out.feet_out = in.feet_new;
  const double z = st[0] + out.initial_z;
  double alive;
  if constexpr (R::alive == 2) alive = z > 0.26 ? 1.0 : -1.0;  // Ant :307-308
  else alive = z > 0.78 ? 2.0 : -1.0;                         // Humanoid :318-319
  out.done = alive < 0 || !finite;
  const double progress = out.potential - in.potential_old;
  const double jal = -0.1 * (double)out.at_limit;
  out.reward = (((0.0 + alive) + progress) + jal) + 0.0;
  // mujoco gym_locomotion_envs.py:98-103 [alive, progress, joints_at_limit, feet_collision]
  out.terms[0] = alive; out.terms[1] = progress; out.terms[2] = jal; out.terms[3] = 0.0; out.terms[4] = 0.0;
}

// Pendulum packs (obs float64 in the reference, float32 through the C-ABI).
//  InvertedPendulum / Swingup: robot_pendula.py:27-51 + gym_pendulum_envs.py:26-39 --
//  non-finite vx / theta / theta_dot replaced by 0; balance: reward 1, done |theta| > .2;
//  swingup: reward cos(theta), never done.
template <class R>
PBG_DEV void pendulum_obs(const double* jq, const double* jqd, const double* tip, float* obs, PackOut& out) {
  out.potential = 0.0; out.initial_z = 0.0; out.feet_out = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) out.terms[i] = 0.0;
  if constexpr (R::alive == 7) {
    // InvertedDoublePendulumMuJoCo: mujoco/robot_pendula.py:75-89 obs [x, sin th, sin g, cos th,
    // cos g, clip(vx, th', g', +-10), qfrc_constraint zeros (3)]; mujoco/gym_pendulum_envs.py:60-72
    // reward sum([10, -dist_penalty, -(1e-3 th'^2 + 5e-3 g'^2)]), done y2 + 0.3 <= 1
    const double th = jq[0], thd = jqd[0], g = jq[1], gd = jqd[1], x = jq[2], vx = jqd[2];
    const double px = tip[0], py = tip[2];
    auto clip10 = [](double v) { return v < -10.0 ? -10.0 : (v > 10.0 ? 10.0 : v); };
    const double o[11] = {x, sin(th), sin(g), cos(th), cos(g), clip10(vx), clip10(thd), clip10(gd), 0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 0; i < 11; i++) obs[i] = (float)o[i];
    const double dist_penalty = 0.01 * (px * px) + ((py + 0.3) - 2) * ((py + 0.3) - 2);
    const double vel_penalty = 1e-3 * (thd * thd) + 5e-3 * (gd * gd);
    out.reward = ((0.0 + 10.0) + -dist_penalty) + -vel_penalty;
    out.terms[0] = 10.0; out.terms[1] = -dist_penalty; out.terms[2] = -vel_penalty;
    out.done = py + 0.3 <= 1;
  } else if constexpr (R::alive == 6) {
    // InvertedDoublePendulum: robot_pendula.py:76-88, gym_pendulum_envs.py:69-80
    const double th = jq[0], thd = jqd[0], g = jq[1], gd = jqd[1], x = jq[2], vx = jqd[2];
    const double px = tip[0], py = tip[2];  // pos_x, _, pos_y = pole2.pose().xyz()
    const double o[9] = {x, vx, px, cos(th), sin(th), thd, cos(g), sin(g), gd};
#pragma unroll
    for (int i = 0; i < 9; i++) obs[i] = (float)o[i];
    const double dist_penalty = 0.01 * (px * px) + ((py + 0.3) - 2) * ((py + 0.3) - 2);
    out.reward = ((0.0 + 10.0) + -dist_penalty) + 0.0;  // sum([alive 10, -dist, -vel 0])
    out.terms[0] = 10.0; out.terms[1] = -dist_penalty; out.terms[2] = -0.0;
    out.done = py + 0.3 <= 1;
  } else {
    double theta = jq[0], theta_dot = jqd[0], x = jq[1], vx = jqd[1];
    if (!isfinite(vx)) vx = 0.0;
    if (!isfinite(theta)) theta = 0.0;
    if (!isfinite(theta_dot)) theta_dot = 0.0;
    obs[0] = (float)x; obs[1] = (float)vx; obs[2] = (float)cos(theta); obs[3] = (float)sin(theta);
    obs[4] = (float)theta_dot;
    out.reward = R::alive == 5 ? cos(theta) : 1.0;
    out.terms[0] = out.reward;  // rewards [float(reward)]
    out.done = R::alive == 5 ? false : fabs(theta) > 0.2;
  }
}
#pragma clang fp contract(on)


// M3 -> quaternion (x,y,z,w): the float32 rotation matrix converted in float32 (one IEEE
// reciprocal per branch) and widened.  The matrix carries float32 rounding already, so the float64
// conversion (round 2: float64, four branches) bought no accuracy; the float64 sqrt and four float64 divisions per
// branch were 8-34 % of the gang walkers' step (r03 stamps).
PBG_DEV void m3_to_quat_f(const m3& mf, double* q) {
  const float* m = mf.m;
  const float t = m[0] + m[4] + m[8];
  float x, y, z, w;
  if (t > 0.f) {
    const float s = sqrtf(t + 1.f) * 2.f, r = 1.f / s;
    w = 0.25f * s; x = (m[7] - m[5]) * r; y = (m[2] - m[6]) * r; z = (m[3] - m[1]) * r;
  } else if (m[0] > m[4] && m[0] > m[8]) {
    const float s = sqrtf(1.f + m[0] - m[4] - m[8]) * 2.f, r = 1.f / s;
    w = (m[7] - m[5]) * r; x = 0.25f * s; y = (m[1] + m[3]) * r; z = (m[2] + m[6]) * r;
  } else if (m[4] > m[8]) {
    const float s = sqrtf(1.f + m[4] - m[0] - m[8]) * 2.f, r = 1.f / s;
    w = (m[2] - m[6]) * r; x = (m[1] + m[3]) * r; y = 0.25f * s; z = (m[5] + m[7]) * r;
  } else {
    const float s = sqrtf(1.f + m[8] - m[0] - m[4]) * 2.f, r = 1.f / s;
    w = (m[3] - m[1]) * r; x = (m[2] + m[6]) * r; y = (m[5] + m[7]) * r; z = 0.25f * s;
  }
  q[0] = x; q[1] = y; q[2] = z; q[3] = w;
}
// the float64 state's link rotation -> quaternion in float64 (the oracle's m3_to_quat, what
// pybullet's getLinkState computes from its double frame)
PBG_DEV void m3_to_quat_f(const M3<double>& md, double* q) {
  const double* m = md.m;
  const double t = m[0] + m[4] + m[8];
  if (t > 0) {
    const double s = sqrt(t + 1.0) * 2;
    q[3] = 0.25 * s; q[0] = (m[7] - m[5]) / s; q[1] = (m[2] - m[6]) / s; q[2] = (m[3] - m[1]) / s;
  } else if (m[0] > m[4] && m[0] > m[8]) {
    const double s = sqrt(1.0 + m[0] - m[4] - m[8]) * 2;
    q[3] = (m[7] - m[5]) / s; q[0] = 0.25 * s; q[1] = (m[1] + m[3]) / s; q[2] = (m[2] + m[6]) / s;
  } else if (m[4] > m[8]) {
    const double s = sqrt(1.0 + m[4] - m[0] - m[8]) * 2;
    q[3] = (m[2] - m[6]) / s; q[0] = (m[1] + m[3]) / s; q[1] = 0.25 * s; q[2] = (m[5] + m[7]) / s;
  } else {
    const double s = sqrt(1.0 + m[8] - m[0] - m[4]) * 2;
    q[3] = (m[3] - m[1]) / s; q[0] = (m[2] + m[6]) / s; q[1] = (m[5] + m[7]) / s; q[2] = 0.25 * s;
  }
}

// Gather pack inputs from the physical state (what pybullet's queries would return).
// st(integral_constant<int, i>): diagnostic phase stamps between the parts (no-op by default)
struct NoStamp {
  template <class C>
  PBG_DEV void operator()(C) const {}
};
template <class R, class St = NoStamp>
PBG_DEV void gather(const State<R>& s, bool has_floor, PackIn<R>& in, St st = St()) {
  using T = real_t<R>;
  using f3 = V3<T>;
  using m3 = M3<T>;
  Kin<R> k;
  fk_pos<R>(s, k);
  st(std::integral_constant<int, 14>{});
  int np = 0;
#pragma unroll
  for (int p = 0; p < R::NP; p++) {
    const f3 c = k.c[R::part_link[p] + 1];
    in.part_x[np] = c.x;
    in.part_y[np] = c.y;
    np++;
  }
  if (R::floor && has_floor) { in.part_x[np] = 0.0; in.part_y[np] = 0.0; np++; }
  in.n_parts = np;
  constexpr int b = R::robot_body + 1;
  if constexpr (b == 0) {  // getBasePositionAndOrientation: the state's own quaternion
#pragma unroll
    for (int i = 0; i < 4; i++) in.quat[i] = s.bq[i];
  } else {
    m3_to_quat_f(k.Rm[b], in.quat);
  }
  st(std::integral_constant<int, 15>{});
  in.pos[0] = k.c[b].x; in.pos[1] = k.c[b].y; in.pos[2] = k.c[b].z;
  if constexpr (R::head_link >= 0) in.head_z = k.c[R::head_link + 1].z;
  // robot_body COM velocity
  f3 vel;
  if constexpr (b == 0) {
    vel = mk3<T>(s.bv[0], s.bv[1], s.bv[2]);
  } else {
    // velocity of link b's COM: rigid/joint chain from the base (recomputed here)
    f3 w[R::NL + 1], v[R::NL + 1];
    w[0] = R::floating ? mk3<T>(s.bw[0], s.bw[1], s.bw[2]) : mk3<T>(0, 0, 0);
    v[0] = R::floating ? mk3<T>(s.bv[0], s.bv[1], s.bv[2]) : mk3<T>(0, 0, 0);
#pragma unroll
    for (int l = 0; l < R::NL; l++) {
      const int p = R::link_parent[l] + 1, jt = R::link_jtype[l], d = R::link_dof[l];
      const f3 cp = k.c[p], c = k.c[l + 1];
      if (jt == 0 || jt == 1) {
        const m3 Ro = quat_to_m3c<T>(R::link_offset_quat[l][0], R::link_offset_quat[l][1], R::link_offset_quat[l][2], R::link_offset_quat[l][3]);
        const m3 R0 = mulc(k.Rm[p], Ro);
        const f3 a = mulc(R0, (T)R::link_axis[l][0], (T)R::link_axis[l][1], (T)R::link_axis[l][2]);
        const f3 x0 = k.x[p] + mulc(k.Rm[p], (T)R::link_offset_pos[l][0], (T)R::link_offset_pos[l][1], (T)R::link_offset_pos[l][2]);
        if (jt == 0) {
          const f3 o = x0 + mulc(R0, (T)R::link_anchor[l][0], (T)R::link_anchor[l][1], (T)R::link_anchor[l][2]);
          const f3 vo = v[p] + cross3(w[p], o - cp);
          w[l + 1] = w[p] + s.qd[d] * a;
          v[l + 1] = vo + cross3(w[l + 1], c - o);
        } else {
          w[l + 1] = w[p];
          v[l + 1] = v[p] + cross3(w[p], c - cp) + s.qd[d] * a;
        }
      } else {
        w[l + 1] = w[p];
        v[l + 1] = v[p] + cross3(w[p], c - cp);
      }
    }
    vel = v[b];
  }
  in.vel[0] = vel.x; in.vel[1] = vel.y; in.vel[2] = vel.z;
  if constexpr (R::floating) { in.avel[0] = s.bw[0]; in.avel[1] = s.bw[1]; in.avel[2] = s.bw[2]; }
#pragma unroll
  for (int i = 0; i < R::NO; i++) { in.jq[i] = s.q[R::obs_dof[i]]; in.jqd[i] = s.qd[R::obs_dof[i]]; }
}

// Pendulum pack from the physical state: obs joints (hinge[, hinge2], slider) and, for the
// double pendulum, pole2's COM (getLinkState[0]).
template <class R>
PBG_DEV void pendulum_pack(const State<R>& s, float* obs, PackOut& po) {
  double jq[R::NO], jqd[R::NO], tip[3] = {0.0, 0.0, 0.0};
#pragma unroll
  for (int i = 0; i < R::NO; i++) { jq[i] = s.q[R::obs_dof[i]]; jqd[i] = s.qd[R::obs_dof[i]]; }
  if constexpr (R::tip_link >= 0) {
    Kin<R> k;
    fk_pos<R>(s, k);
    const V3<real_t<R>> c = k.c[R::tip_link + 1];
    tip[0] = c.x; tip[1] = c.y; tip[2] = c.z;
  }
  pendulum_obs<R>(jq, jqd, tip, obs, po);
}

// epi: resets of env e so far (the Philox counter); the caller bumps B.episode[e].
// Q = 4: the pack's transcendentals dealt over a DPP quad (quad / gang kernels, `lane`).
template <class R, int Q = 1>
PBG_DEV void reset_env_epi(const Buffers& B, int e, State<R>& s, const float* init_q, float* obs, bool& has_floor,
                           double& pot, real_t<R>& z0, uint32_t epi, Flag& fl, HarderBk* hb = nullptr, int lane = 0) {
  using T = real_t<R>;
  snapshot_state<R>(s);
  if (init_q) {
#pragma unroll
    for (int r = 0; r < R::NR; r++) s.q[R::reset_dof[r]] = (T)R::reset_offset[r] + (T)init_q[(size_t)e * R::NR + r];
  } else {
    // np_random.uniform(-0.1, 0.1) per ordered joint (robot_locomotors.py:18-19) -> Philox
    const uint32_t gid = (uint32_t)(B.env_offset + e);
#pragma unroll
    for (int blk = 0; blk < (R::NR + 3) / 4; blk++) {
      u4 ctr = {gid, epi, (uint32_t)blk, 0x5EEDu};
      const u4 rnd = philox4x32_10(ctr, (uint32_t)B.seed, (uint32_t)(B.seed >> 32));
      const uint32_t rr[4] = {rnd.x, rnd.y, rnd.z, rnd.w};
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const int r = 4 * blk + t;
        if (r < R::NR) s.q[R::reset_dof[r]] = (T)R::reset_offset[r] + (T)fmaf(0.2f, u01(rr[t]), -0.1f);
      }
    }
  }
  PackOut po;
  if constexpr (R::kind == 1) {
    pendulum_pack<R>(s, obs, po);
    has_floor = true; pot = 0.0; z0 = 0.f;
    return;
  } else if constexpr (R::kind == 2) {
    // reset: calc_state, then env.potential = calc_potential() stores x_after (env_bases.py:69-70)
    mujoco_planar_pack_state<R>(s, 0.0, nullptr, obs, po, B.sp.env_dt);
    has_floor = true; pot = po.potential; z0 = 0.f;
    return;
  } else {
  PackIn<R> in;
  in.env_dt = B.sp.env_dt;
  gather<R>(s, has_floor, in);
#pragma unroll
  for (int f = 0; f < R::NF; f++) in.feet_prev[f] = 0.f;
  in.feet_new = 0;
  in.potential_old = 0.0;
  in.initial_z = R::initial_z_fixed;
  auto draw = [&](Flag& f) { flag_draw(B, e, f); };
  if constexpr (R::flagrun) draw(fl);  // robot_specific_reset -> flag_reposition (:199-201)
  if constexpr (R::harder) {  // HumanoidFlagrunHarder.robot_specific_reset (:237-248)
    hb->frame = 0; hb->onground = 0; hb->crawl_start = __builtin_nan(""); hb->crawl_ignored = 0.0;
  }
  if constexpr (R::kind == 3) mujoco3d_pack<R>(in, nullptr, obs, po);
  else flag_pack<R, Q>(in, nullptr, obs, po, fl, draw, lane, hb);
  if constexpr (R::harder) po.potential = harder_potential(*hb, po.potential, po.body_xyz[2]);  // env_bases.py:70
  pot = po.potential;
  z0 = (T)po.initial_z;
  has_floor = true;  // gym_locomotion_envs.py:30-31: the floor joins robot.parts
  }
}

template <class R>
PBG_DEV void reset_env(const Buffers& B, int e, State<R>& s, const float* init_q, float* obs, bool& has_floor,
                       double& pot, real_t<R>& z0) {
  const uint32_t epi = B.episode[e];
  B.episode[e] = epi + 1;
  Flag fl = load_flag<R>(B, e);
  HarderBk hb = load_harder<R>(B, e);
  reset_env_epi<R>(B, e, s, init_q, obs, has_floor, pot, z0, epi, fl, &hb);
  store_flag<R>(B, e, fl);
  store_harder<R>(B, e, hb);
}

template <class R>
__global__ __launch_bounds__(64) void reset_kernel(Buffers B, ResetIO io) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B.n) return;
  if (io.mask && !io.mask[e]) return;
  State<R> s;
  bool has_floor = B.flags[e] & 1u;
  double pot;
  real_t<R> z0;
  float obs[R::OBS];
  reset_env<R>(B, e, s, io.init_q, obs, has_floor, pot, z0);
  store_state<R>(s, st_of<R>(B), B.n, e);
  B.pot[e] = pot;
  z0_of<R>(B)[e] = z0;
  B.elapsed[e] = 0;
  B.flags[e] = has_floor ? 1u : 0u;  // feet_contact cleared (robot_locomotors.py:22)
#pragma unroll
  for (int i = 0; i < R::OBS; i++) io.obs[(size_t)e * R::OBS + i] = obs[i];
}

template <class R, int LS>
__global__ __launch_bounds__(64) void step_kernel(Buffers B, StepIO io, float* __restrict__ scratch, int lds_rows) {
  extern __shared__ float lds_dyn[];
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B.n) return;
  STAMP_DECL
  using T = real_t<R>;
  State<R> s;
  load_state<R>(s, st_of<R>(B), B.n, e);
  float act[R::NA];
#pragma unroll
  for (int i = 0; i < R::NA; i++) act[i] = io.act[(size_t)e * R::NA + i];
  // apply_action: tau = power * power_coef * clip(a, -1, 1)   (robot_locomotors.py:26-29)
  T tau[R::NJ];
#pragma unroll
  for (int d = 0; d < R::NJ; d++) tau[d] = 0.f;
#pragma unroll
  for (int i = 0; i < R::NA; i++) {
    const float c = fminf(fmaxf(act[i], -1.f), 1.f);
    tau[R::act_dof[i]] += (T)(R::act_gain[i] * (double)c);
  }
  uint32_t slot_active[R::NS > 0 ? R::NS : 1];
  Rows<R, LS> rw;
  rw.lds = (lds_t<T>*)lds_dyn + threadIdx.x;
  rw.gbl = (T*)scratch + e;
  rw.n = B.n;
  rw.cap = lds_rows;
  int nc = 0;
  uint32_t csig = 0;
  STAMP(7)
  const SimPT<T>& P = sp_of<R>(B);
  for (int sub = 0; sub < P.substeps; sub++)
    nc = substep<R, LS>(s, tau, slot_active, rw, (uint32_t)sub, csig, P SUB_STAMP_PASS);
  if (io.ncontact) io.ncontact[e] = nc;
  if (io.csig) io.csig[e] = csig;
  const int el = B.elapsed[e] + 1;
  uint32_t flags = B.flags[e];
  float obs[R::OBS];
  PackOut po;
  double pot_new = 0.0;
  if constexpr (R::kind == 1) {
    pendulum_pack<R>(s, obs, po);
  } else if constexpr (R::kind == 2) {
    mujoco_planar_pack_state<R>(s, B.pot[e], act, obs, po, B.sp.env_dt);
    pot_new = po.potential;
  } else {
    PackIn<R> in;
    in.env_dt = B.sp.env_dt;
    gather<R>(s, flags & 1u, in);
    uint32_t fnew = 0;
#pragma unroll
    for (int f = 0; f < R::NF; f++) {
      bool c = false;
#pragma unroll
      for (int sl = 0; sl < R::NS; sl++)
        if (R::slot_link[sl] == R::foot_link[f]) c |= slot_active[sl] != 0;
      fnew |= (c ? 1u : 0u) << f;
      in.feet_prev[f] = ((flags >> (8 + f)) & 1u) ? 1.f : 0.f;
    }
    in.feet_new = fnew;
    in.potential_old = B.pot[e];
    in.initial_z = z0_of<R>(B)[e];
    Flag fl = load_flag<R>(B, e);
    HarderBk hb = load_harder<R>(B, e);
    if constexpr (R::kind == 3) mujoco3d_pack<R>(in, act, obs, po);
    else flag_pack<R>(in, act, obs, po, fl, [&](Flag& f) { flag_draw(B, e, f); }, 0, &hb);
    if constexpr (R::harder) {
      double pos[3], vel[3];
      if (harder_step<R>(B, e, in, obs, po, hb, pos, vel, nullptr)) {  // resetBasePosition / Velocity
#pragma unroll
        for (int i = 0; i < 3; i++) { s.cube.p[i] = (T)pos[i]; s.cube.v[i] = (T)vel[i]; s.cube.w[i] = 0.f; }
      }
      store_harder<R>(B, e, hb);
    }
    store_flag<R>(B, e, fl);
    pot_new = po.potential;
    flags = (flags & 0xFFu) | (po.feet_out << 8);
  }
  STAMP(8)
  const bool term = po.done;
  const bool trunc = el >= R::max_episode_steps;  // gym TimeLimit (envs/__init__.py max_episode_steps)
  io.rew[e] = (float)po.reward;
  if (io.rew64) io.rew64[e] = po.reward;
  if (io.rew_terms) {
#pragma unroll
    for (int i = 0; i < 5; i++) io.rew_terms[(size_t)e * 5 + i] = po.terms[i];
  }
  io.done[e] = term || trunc;
  if (io.trunc) io.trunc[e] = trunc && !term;
  if (io.autoreset && (term || trunc)) {
    if (io.term_obs) {
#pragma unroll
      for (int i = 0; i < R::OBS; i++) io.term_obs[(size_t)e * R::OBS + i] = obs[i];
    }
    bool has_floor = flags & 1u;
    double pot;
    T z0;
    reset_env<R>(B, e, s, nullptr, obs, has_floor, pot, z0);
    B.pot[e] = pot;
    z0_of<R>(B)[e] = z0;
    B.elapsed[e] = 0;
    B.flags[e] = has_floor ? 1u : 0u;
  } else {
    B.pot[e] = pot_new;
    B.elapsed[e] = el;
    B.flags[e] = flags;
  }
  store_state<R>(s, st_of<R>(B), B.n, e);
#pragma unroll
  for (int i = 0; i < R::OBS; i++) io.obs[(size_t)e * R::OBS + i] = obs[i];
  STAMP(9)
  STAMP_FLUSH
}

// Pack on explicit inputs (golden-vector parity of the device pack).  Per env the input
// record is float64: [part_xyz (NP+1)*3 | n_parts | quat 4 | pos 3 | vel 3 | jq NO | jqd NO |
// feet_prev NF | feet_new NF | act NA | potential_old | initial_z_in | is_step]; the output
// record: [obs OBS | reward | done | potential | initial_z | feet_out NF].
template <class R>
__global__ __launch_bounds__(64) void pack_kernel(int n, const double* __restrict__ inrec, double* __restrict__ outrec) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const double* r = inrec + (size_t)e * PackRec<R>::IN;
  double* w = outrec + (size_t)e * PackRec<R>::OUT;
  float obs[R::OBS];
  float act[R::NA];
  PackOut po;
  const int o_np = (R::NP + 1) * 3;
  const int o_q = o_np + 1, o_pos = o_q + 4, o_vel = o_pos + 3, o_jq = o_vel + 3, o_jqd = o_jq + R::NO;
  const int o_fp = o_jqd + R::NO, o_fn = o_fp + R::NF, o_act = o_fn + R::NF, o_pot = o_act + R::NA;
  const bool is_step = r[o_pot + 2] != 0.0;
#pragma unroll
  for (int i = 0; i < R::NA; i++) act[i] = (float)r[o_act + i];
  if constexpr (R::kind == 1) {
    pendulum_obs<R>(r + o_jq, r + o_jqd, r + o_pos, obs, po);  // pos: pole2 position (double pendulum)
  } else if constexpr (R::kind == 2) {
    // pos: robot_body position (x_after), potential_old: x_before
    mujoco_planar_pack<R>(r + o_jq, r + o_jqd, r[o_pos], r[o_pot], is_step ? act : nullptr, obs, po);
  } else {
    PackIn<R> in;
    in.n_parts = (int)r[o_np];
#pragma unroll
    for (int p = 0; p < R::NP + 1; p++) { in.part_x[p] = r[3 * p]; in.part_y[p] = r[3 * p + 1]; }
#pragma unroll
    for (int i = 0; i < 4; i++) in.quat[i] = r[o_q + i];
#pragma unroll
    for (int i = 0; i < 3; i++) { in.pos[i] = r[o_pos + i]; in.vel[i] = r[o_vel + i]; }
#pragma unroll
    for (int i = 0; i < R::NO; i++) { in.jq[i] = r[o_jq + i]; in.jqd[i] = r[o_jqd + i]; }
    uint32_t fn = 0;
#pragma unroll
    for (int f = 0; f < R::NF; f++) { in.feet_prev[f] = (float)r[o_fp + f]; fn |= (r[o_fn + f] != 0.0 ? 1u : 0u) << f; }
    in.feet_new = fn;
    in.potential_old = r[o_pot];
    in.initial_z = r[o_pot + 1];
    if constexpr (R::alive == 13) in.head_z = r[o_pot + 3];  // Atlas
    if constexpr (R::kind == 3) {
#pragma unroll
      for (int i = 0; i < 3; i++) in.avel[i] = r[o_pot + 3 + i];  // base angular velocity
      if (in.n_parts == R::NP || in.n_parts == R::NP + 1) mujoco3d_pack<R>(in, is_step ? act : nullptr, obs, po);
      else mujoco3d_pack<R, true>(in, is_step ? act : nullptr, obs, po);
    } else if constexpr (R::flagrun) {
      // [target x, y | flag_timeout | next target x, y]: the reposition takes the recorded draw
      const int o_f = o_pot + 3;
      Flag f = {r[o_f], r[o_f + 1], (int)r[o_f + 2], 0};
      // HumanoidFlagrunHarder: [frame | on_ground | crawl_start | crawl_ignored | launch draws 5]
      const int o_h = o_f + 5;
      HarderBk hb = {0, 0, 0, 0.0, 0.0};
      if constexpr (R::harder) hb = HarderBk{(int)r[o_h], (int)r[o_h + 1], 0, r[o_h + 2], r[o_h + 3]};
      flag_pack<R>(in, is_step ? act : nullptr, obs, po, f, [&](Flag& g) {
        g.tx = r[o_f + 3]; g.ty = r[o_f + 4]; g.timeout = PBG_FLAG_TIMEOUT; g.count++;
      }, 0, &hb);
      w[R::OBS + 4 + R::NF] = f.tx;
      w[R::OBS + 4 + R::NF + 1] = f.ty;
      w[R::OBS + 4 + R::NF + 2] = f.timeout;
      if constexpr (R::harder) {
        // out: [frame | on_ground | crawl_start | crawl_ignored | launched | cube position 3 | velocity 3]
        double pos[3] = {__builtin_nan(""), __builtin_nan(""), __builtin_nan("")}, vel[3] = {pos[0], pos[1], pos[2]};
        bool launched = false;
        if (is_step) {
          Buffers Bz{};
          launched = harder_step<R>(Bz, e, in, obs, po, hb, pos, vel, r + o_h + 4);
        } else {
          po.potential = harder_potential(hb, po.potential, po.body_xyz[2]);
        }
        double* ho = w + R::OBS + 4 + R::NF + 3;
        ho[0] = hb.frame; ho[1] = hb.onground; ho[2] = hb.crawl_start; ho[3] = hb.crawl_ignored; ho[4] = launched ? 1.0 : 0.0;
#pragma unroll
        for (int i = 0; i < 3; i++) { ho[5 + i] = pos[i]; ho[8 + i] = vel[i]; }
      }
    } else if (in.n_parts == R::NP || in.n_parts == R::NP + 1) {
      // the step's part counts take the kernels' compile-time path (what this test pins)
      walker_pack<R>(in, is_step ? act : nullptr, obs, po);
    } else {
      walker_pack<R, true>(in, is_step ? act : nullptr, obs, po);
    }
  }
  if (!is_step) { po.reward = 0.0; po.done = false; }
#pragma unroll
  for (int i = 0; i < R::OBS; i++) w[i] = (double)obs[i];
  w[R::OBS] = po.reward;
  w[R::OBS + 1] = po.done ? 1.0 : 0.0;
  w[R::OBS + 2] = po.potential;
  w[R::OBS + 3] = po.initial_z;
#pragma unroll
  for (int f = 0; f < R::NF; f++) w[R::OBS + 4 + f] = (po.feet_out >> f) & 1u;
}

// State record conversion: SoA float32 (+ bookkeeping) <-> AoS float64 records.
template <class R>
__global__ __launch_bounds__(64) void get_state_kernel(Buffers B, double* __restrict__ phys, double* __restrict__ aux) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B.n) return;
  constexpr int SD = Dims<R>::SD, AD = Records<R>::AD;
  const real_t<R>* st = st_of<R>(B);
  for (int i = 0; i < SD; i++) phys[(size_t)e * SD + i] = (double)st[(size_t)i * B.n + e];
  double* a = aux + (size_t)e * AD;
  a[0] = B.pot[e];
  a[1] = (double)z0_of<R>(B)[e];
  a[2] = (double)B.elapsed[e];
  a[3] = (double)(B.flags[e] & 1u);
  for (int f = 0; f < R::NF; f++) a[4 + f] = (double)((B.flags[e] >> (8 + f)) & 1u);
  if constexpr (R::flagrun) {
    const Flag fl = load_flag<R>(B, e);
    a[4 + R::NF] = fl.tx; a[5 + R::NF] = fl.ty; a[6 + R::NF] = fl.timeout; a[7 + R::NF] = fl.count;
  }
  if constexpr (R::harder) {
    const HarderBk h = load_harder<R>(B, e);
    a[8 + R::NF] = h.frame; a[9 + R::NF] = h.onground; a[10 + R::NF] = h.crawl_start;
    a[11 + R::NF] = h.crawl_ignored; a[12 + R::NF] = h.launches;
  }
  a[AD - 1] = (double)B.episode[e];  // the reset-noise Philox counter
}
template <class R>
__global__ __launch_bounds__(64) void set_state_kernel(Buffers B, const double* __restrict__ phys, const double* __restrict__ aux) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B.n) return;
  constexpr int SD = Dims<R>::SD, AD = Records<R>::AD;
  using T = real_t<R>;
  T* st = st_of<R>(B);
  for (int i = 0; i < SD; i++) st[(size_t)i * B.n + e] = (T)phys[(size_t)e * SD + i];
  if (aux) {
    const double* a = aux + (size_t)e * AD;
    B.pot[e] = a[0];
    z0_of<R>(B)[e] = (T)a[1];
    B.elapsed[e] = (int)a[2];
    uint32_t fl = a[3] != 0.0 ? 1u : 0u;
    for (int f = 0; f < R::NF; f++) fl |= (a[4 + f] != 0.0 ? 1u : 0u) << (8 + f);
    B.flags[e] = fl;
    if constexpr (R::flagrun)
      store_flag<R>(B, e, Flag{a[4 + R::NF], a[5 + R::NF], (int)a[6 + R::NF], (int)a[7 + R::NF]});
    if constexpr (R::harder)
      store_harder<R>(B, e, HarderBk{(int)a[8 + R::NF], (int)a[9 + R::NF], (int)a[12 + R::NF], a[10 + R::NF], a[11 + R::NF]});
    B.episode[e] = (uint32_t)a[AD - 1];
  }
}

}  // namespace pbg
