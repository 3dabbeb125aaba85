// pbg_team.hip -- quad-per-env step kernel for a floating base carrying 4 isomorphic
// branches (AntPyBulletEnv-v0: torso + 4 legs).  Included by pbg_robot.hip after
// pbg_step.hip; selected by plan_* when Team<R>::ok.
//
// Same physics, constraint-row order and numpy-exact pack as step_kernel (one lane per
// env, pbg_step.hip), which remains the kernel for the other robots.  Here an env's work
// is split over the 4 lanes of a quad: lane k owns branch k -- its links' kinematics and
// composite inertias, its block of the mass matrix and those Cholesky columns, its
// joint-limit rows and the contact rows of its slots.  Base quantities (pose, velocity,
// the 6x6 Schur complement and its factor, u_base) are replicated in all four lanes and
// stay bitwise identical: every cross-lane sum is a quad butterfly (DPP quad_perm) whose
// result is the same in each lane.  PGS stays sequential in Bullet's row order
// (scene_bases.py:65 numSolverIterations=5 -> limits, normals, frictions); per row the
// owner's branch dot product reaches the quad by DPP and the base part is replicated.
//
// Why: 16,384 Ant envs are 256 waves -- one per CU, one of its four SIMDs -- in the lane
// kernel; as quads they are 1,024 waves, one per SIMD, and each lane carries a quarter of
// the per-env register state (no scratch spills).
//
// Generalized order per lane: [branch dofs leaf-first (NDB) | base lin 0..2 | base ang 0..2],
// i.e. the lane kernel's order (pbg_step.hip Dims::gj) restricted to one branch + base.

namespace pbg {

// ------------------------------------------------------------------ quad (DPP) helpers
// bound_ctrl set: every permutation used here reads a valid lane, and with it the
// compiler folds `x + mov_dpp(x)` into one v_add_f32_dpp (no mov, no DPP hazard nop).
template <int CTRL>
PBG_DEV float qperm(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
PBG_DEV int qperm_i(int x) {
  return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, true);
}
// sum over the quad; identical bits in all four lanes ((x0+x1)+(x2+x3), addition commutes)
PBG_DEV float quad_sum(float x) {
  x = x + qperm<0xB1>(x);  // quad_perm [1,0,3,2]
  return x + qperm<0x4E>(x);  // quad_perm [2,3,0,1]
}
PBG_DEV int quad_sum_i(int x) {
  x = x + qperm_i<0xB1>(x);
  return x + qperm_i<0x4E>(x);
}
template <int K>
PBG_DEV float quad_bcast(float x) { return qperm<K | (K << 2) | (K << 4) | (K << 6)>(x); }
template <int K>
PBG_DEV int quad_bcast_i(int x) { return qperm_i<K | (K << 2) | (K << 4) | (K << 6)>(x); }
// float64 (F64<R>: the reference-precision path): a double moves as its two dwords
template <int CTRL>
PBG_DEV double qperm(double x) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
PBG_DEV double quad_sum(double x) {
  x = x + qperm<0xB1>(x);
  return x + qperm<0x4E>(x);
}
template <int K>
PBG_DEV double quad_bcast(double x) { return qperm<K | (K << 2) | (K << 4) | (K << 6)>(x); }
// LDS written by one lane and read by another lane of the same wave: a compiler fence
// (the wave's LDS operations execute in order).
#define PBG_QUAD_SYNC                                    \
  {                                                      \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); \
    __builtin_amdgcn_wave_barrier();                     \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); \
  }

// Diagnostic build only (-DPBG_TRACE64, tools/f64_quad_trace.py; never the product library): the float64
// quad kernel's per-lane values at its phase boundaries, in the last sub-step, as unconditional global
// stores at the existing scheduling fences (no branch: the trace splits no scheduling region).  Slot
// (block * 64 + lane) & 255: the diagnostic runs 64 envs (4 one-wave blocks).
#ifdef PBG_TRACE64
#define PBG_TRACE_PH 8
__device__ double g_trace64[256][PBG_TRACE_PH][8];
#define TRACE64(ph, i, v) \
  do { if constexpr (sizeof(Sc) == 8) g_trace64[(blockIdx.x * 64 + threadIdx.x) & 255][ph][i] = (double)(v); } while (0)
#else
#define TRACE64(ph, i, v) do {} while (0)
#endif

// ------------------------------------------------------------------ branch decomposition
template <int N, class S = float>
struct BTab {  // per-branch constant: v[entry][branch]
  S v[N > 0 ? N : 1][4];
};
template <int N>
struct BTabI {
  int v[N > 0 ? N : 1][4];
};

template <class R>
struct Team {
  using Sc = real_t<R>;
  static constexpr int NL = R::NL, NJ = R::NJ;
  static constexpr int roots() {
    int c = 0;
    for (int l = 0; l < NL; l++) c += R::link_parent[l] == -1;
    return c;
  }
  static constexpr int B = roots();
  static constexpr int NLB = B > 0 ? NL / B : 1;
  static constexpr int NDB = B > 0 ? NJ / B : 1;
  static constexpr int base_slots() {
    int c = 0;
    for (int s = 0; s < R::NS; s++) c += R::slot_link[s] == -1;
    return c;
  }
  static constexpr int NS0 = base_slots();
  static constexpr int NSB = B > 0 ? (R::NS - NS0) / B : 0;
  static constexpr int NC = R::NS;      // contact capacity
  static constexpr int W = 4 * NDB + 11;  // contact row: y_b (4 lane slots) | y_base (6 + 2 pad) | meff | target | lambda
  static constexpr int check() {
    if (!R::floating || (R::kind != 0 && R::kind != 3) || R::NPAIR != 0 || R::robot_body != -1 || B != 4) return false;
    if (NL % B || NJ % B || (R::NS - NS0) % B || NDB < 1 || NDB > 8) return false;
    for (int s = 0; s < NS0; s++)
      if (R::slot_link[s] != -1) return false;
    for (int k = 0; k < B; k++) {
      for (int i = 0; i < NLB; i++) {
        const int l = k * NLB + i, p = R::link_parent[l];
        if (i == 0 ? p != -1 : p != k * NLB + R::link_parent[i]) return false;
        if (R::link_jtype[l] != R::link_jtype[i]) return false;
        const int d0 = R::link_dof[i], d = R::link_dof[l];
        if (d0 < 0 ? d != -1 : d != k * NDB + d0) return false;
        if ((R::link_mass[l] > 0.0) != (R::link_mass[i] > 0.0)) return false;
      }
      for (int j = 0; j < NDB; j++)
        if (R::dof_limited[k * NDB + j] != R::dof_limited[j] || R::dof_jtype[k * NDB + j] != R::dof_jtype[j]) return false;
      for (int s = 0; s < NSB; s++)
        if (R::slot_link[NS0 + k * NSB + s] != k * NLB + R::slot_link[NS0 + s]) return false;
    }
    for (int f = 0; f < R::NF; f++)
      if (R::foot_link[f] < 0) return false;
    for (int i = 0; i < R::NA; i++)
      if (R::act_dof[i] < 0 || R::act_dof[i] >= NJ) return false;
    // no restitution or torsional friction rows (the gang and lane kernels model them)
    if (R::restitution != 0.0 || R::spin_mu != 0.0 || R::roll_mu != 0.0) return false;
    return true;
  }
  static constexpr bool ok = check();

  // local structure (branch 0 is the template); gen index a <-> local dof NDB-1-a
  static constexpr int dof_of(int a) { return NDB - 1 - a; }
  static constexpr int lg(int j) { return NDB - 1 - j; }
  static constexpr bool moves(int j, int i) { return i >= 0 && ((R::link_chain_mask[i] >> j) & 1u); }
  static constexpr bool coupled(int a, int b) {
    const int da = dof_of(a), db = dof_of(b);
    return moves(da, R::dof_link[db]) || moves(db, R::dof_link[da]);
  }
  static constexpr bool anc(int a, int i) { return a == i || ((R::link_anc_mask[i] >> a) & 1u); }
  static constexpr bool owner(int i) { return R::link_dof[i] >= 0; }
  static constexpr bool in_chain(int a, int i) { return moves(dof_of(a), i); }  // gen a moves link i
  // entry a of the branch part of limit row li (li-th limited dof of the branch) is
  // structurally nonzero: y = L^-1 e_gd vanishes above gd and off gd's coupled dofs
  static constexpr bool lim_nz(int li, int a) {
    int j = 0, c = 0;
    for (int jj = 0; jj < NDB; jj++)
      if (R::dof_limited[jj]) {
        if (c == li) j = jj;
        c++;
      }
    const int gd = lg(j);
    return !(a < gd || !coupled(a, gd));
  }

  // per-branch constants
  static constexpr BTab<NLB * 3, Sc> vec3(const double (*t)[3]) {
    BTab<NLB * 3, Sc> r{};
    for (int i = 0; i < NLB; i++)
      for (int c = 0; c < 3; c++)
        for (int k = 0; k < B; k++) r.v[i * 3 + c][k] = (Sc)t[k * NLB + i][c];
    return r;
  }
  static constexpr BTab<NLB * 9, Sc> make_rot() {
    BTab<NLB * 9, Sc> r{};
    for (int i = 0; i < NLB; i++)
      for (int k = 0; k < B; k++) {
        const double* q = R::link_offset_quat[k * NLB + i];
        const double x = q[0], y = q[1], z = q[2], w = q[3];
        const double m[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                             2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                             2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)};
        for (int c = 0; c < 9; c++) r.v[i * 9 + c][k] = (Sc)m[c];
      }
    return r;
  }
  static constexpr BTab<NLB, Sc> make_mass() {
    BTab<NLB, Sc> r{};
    for (int i = 0; i < NLB; i++)
      for (int k = 0; k < B; k++) r.v[i][k] = (Sc)R::link_mass[k * NLB + i];
    return r;
  }
  static constexpr BTab<NLB * 6, Sc> make_iner() {
    BTab<NLB * 6, Sc> r{};
    for (int i = 0; i < NLB; i++)
      for (int c = 0; c < 6; c++)
        for (int k = 0; k < B; k++) r.v[i * 6 + c][k] = (Sc)R::link_inertia[k * NLB + i][c];
    return r;
  }
  static constexpr BTab<NDB, Sc> dofs(const double* t) {
    BTab<NDB, Sc> r{};
    for (int j = 0; j < NDB; j++)
      for (int k = 0; k < B; k++) r.v[j][k] = (Sc)t[k * NDB + j];
    return r;
  }
  static constexpr BTab<NDB, Sc> make_gain() {  // tau = gain * clip(a) of the actuator driving the dof
    BTab<NDB, Sc> r{};
    for (int i = 0; i < R::NA; i++) r.v[R::act_dof[i] % NDB][R::act_dof[i] / NDB] = (Sc)R::act_gain[i];
    return r;
  }
  static constexpr BTabI<NDB> make_acti() {
    BTabI<NDB> r{};
    for (int j = 0; j < NDB; j++)
      for (int k = 0; k < B; k++) r.v[j][k] = -1;
    for (int i = 0; i < R::NA; i++) r.v[R::act_dof[i] % NDB][R::act_dof[i] / NDB] = i;
    return r;
  }
  static constexpr BTabI<NDB> make_rst() {
    BTabI<NDB> r{};
    for (int j = 0; j < NDB; j++)
      for (int k = 0; k < B; k++) r.v[j][k] = -1;
    for (int q = 0; q < R::NR; q++) r.v[R::reset_dof[q] % NDB][R::reset_dof[q] / NDB] = q;
    return r;
  }
  static constexpr BTabI<NLB> make_foot() {
    BTabI<NLB> r{};
    for (int i = 0; i < NLB; i++)
      for (int k = 0; k < B; k++) r.v[i][k] = -1;
    for (int f = 0; f < R::NF; f++) r.v[R::foot_link[f] % NLB][R::foot_link[f] / NLB] = f;
    return r;
  }
  static constexpr BTab<NSB * 3, Sc> make_spt() {
    BTab<NSB * 3, Sc> r{};
    for (int s = 0; s < NSB; s++)
      for (int c = 0; c < 3; c++)
        for (int k = 0; k < B; k++) r.v[s * 3 + c][k] = (Sc)R::slot_point[NS0 + k * NSB + s][c];
    return r;
  }
  static constexpr BTab<NSB, Sc> slots(const double* t) {
    BTab<NSB, Sc> r{};
    for (int s = 0; s < NSB; s++)
      for (int k = 0; k < B; k++) r.v[s][k] = (Sc)t[NS0 + k * NSB + s];
    return r;
  }
  static constexpr BTab<NLB * 3, Sc> OFFP = vec3(R::link_offset_pos);
  static constexpr BTab<NLB * 3, Sc> AXIS = vec3(R::link_axis);
  static constexpr BTab<NLB * 3, Sc> ANCH = vec3(R::link_anchor);
  static constexpr BTab<NLB * 3, Sc> COM = vec3(R::link_com);
  static constexpr BTab<NLB * 9, Sc> ROT = make_rot();
  static constexpr BTab<NLB, Sc> MASS = make_mass();
  static constexpr BTab<NLB * 6, Sc> INER = make_iner();
  static constexpr BTab<NDB, Sc> DLO = dofs(R::dof_lower);
  static constexpr BTab<NDB, Sc> DHI = dofs(R::dof_upper);
  static constexpr BTab<NDB, Sc> DAMP = dofs(R::dof_damping);
  static constexpr BTab<NDB, Sc> STIFF = dofs(R::dof_stiffness);
  static constexpr BTab<NDB, Sc> ARM = dofs(R::dof_armature);
  static constexpr BTab<NDB, Sc> GAIN = make_gain();
  static constexpr BTabI<NDB> ACTI = make_acti();
  static constexpr BTabI<NDB> RST = make_rst();
  static constexpr BTabI<NLB> FOOT = make_foot();
  static constexpr BTab<NSB * 3, Sc> SPT = make_spt();
  static constexpr BTab<NSB, Sc> SRAD = slots(R::slot_radius);
  static constexpr BTab<NSB, Sc> SMU = slots(R::slot_mu);
};

// The lane's branch and its one-hot weights, for picking per-branch constants.
struct Lane {
  int k;
  bool odd, hi, mid;
  float e0, e1, e2, e3;
};
PBG_DEV Lane make_lane(int k) {
  Lane L;
  L.k = k;
  L.odd = k & 1;
  L.hi = k >= 2;
  L.mid = k == 1 || k == 2;
  L.e0 = k == 0; L.e1 = k == 1; L.e2 = k == 2; L.e3 = k == 3;
  return L;
}
// per-branch constant of entry I of table T for this lane (a constant when all branches agree)
template <const auto& T, int I>
PBG_DEV auto pk(const Lane& L) {
  using S = std::remove_cv_t<std::remove_reference_t<decltype(T.v[0][0])>>;
  constexpr S a0 = T.v[I][0], a1 = T.v[I][1], a2 = T.v[I][2], a3 = T.v[I][3];
  if constexpr (a0 == a1 && a0 == a2 && a0 == a3) return a0;
  else if constexpr (a0 == a2 && a1 == a3) return L.odd ? a1 : a0;
  else if constexpr (a0 == a1 && a2 == a3) return L.hi ? a2 : a0;
  else if constexpr (a0 == a3 && a1 == a2) return L.mid ? a1 : a0;
  else return a0 * (S)L.e0 + a1 * (S)L.e1 + a2 * (S)L.e2 + a3 * (S)L.e3;
}
template <const auto& T, int I>
PBG_DEV int pki(const Lane& L) {
  constexpr int a0 = T.v[I][0], a1 = T.v[I][1], a2 = T.v[I][2], a3 = T.v[I][3];
  if constexpr (a1 - a0 == a2 - a1 && a2 - a1 == a3 - a2) return a0 + (a1 - a0) * L.k;
  else return L.k == 0 ? a0 : (L.k == 1 ? a1 : (L.k == 2 ? a2 : a3));
}
template <const auto& T, int I>
PBG_DEV auto pk3(const Lane& L) {
  return mk3<decltype(pk<T, 3 * I>(L))>(pk<T, 3 * I>(L), pk<T, 3 * I + 1>(L), pk<T, 3 * I + 2>(L));
}

// ------------------------------------------------------------------ per-lane state
template <class R>
struct TState {
  using Sc = real_t<R>;
  static constexpr int NDB = Team<R>::NDB;
  Sc bp[3], bq[4], bv[3], bw[3];  // replicated
  Sc q[NDB], qd[NDB];             // this lane's branch dofs (local order)
};

template <class R>
struct TKin {  // this lane's branch links
  using Sc = real_t<R>;
  using f3 = V3<Sc>;
  using m3 = M3<Sc>;
  static constexpr int NLB = Team<R>::NLB;
  m3 Rm[NLB];
  f3 x[NLB], c[NLB];
};

// branch forward kinematics (positions); joint axes / anchors of the branch dofs on request
template <class R, bool AXES = false>
PBG_DEV void team_fk(const TState<R>& s, const Lane& L, const M3<real_t<R>>& Rb, TKin<R>& k, V3<real_t<R>>* ja = nullptr,
                     V3<real_t<R>>* jo = nullptr) {
  using Sc = real_t<R>;
  using f3 = V3<Sc>;
  using m3 = M3<Sc>;
  using T = Team<R>;
  const f3 xb = mk3<Sc>(s.bp[0], s.bp[1], s.bp[2]);
  static_for<0, T::NLB>([&](auto i_c) {
    constexpr int i = decltype(i_c)::value;
    constexpr int p = R::link_parent[i], jt = R::link_jtype[i], d = R::link_dof[i];
    const m3& Rp = p < 0 ? Rb : k.Rm[p < 0 ? 0 : p];
    const f3 xp = p < 0 ? xb : k.x[p < 0 ? 0 : p];
    m3 Ro;
#pragma unroll
    for (int c = 0; c < 9; c++) Ro.m[c] = 0.f;
    static_for<0, 9>([&](auto c_c) { Ro.m[decltype(c_c)::value] = pk<T::ROT, 9 * i + decltype(c_c)::value>(L); });
    const m3 R0 = mulc(Rp, Ro);
    const f3 x0 = xp + mulc(Rp, pk3<T::OFFP, i>(L));
    if constexpr (jt == 0) {
      const f3 axl = pk3<T::AXIS, i>(L), anl = pk3<T::ANCH, i>(L);
      const m3 Rj = axis_angle_m3c(axl.x, axl.y, axl.z, s.q[d]);
      k.Rm[i] = mul(R0, Rj);
      k.x[i] = x0 + mul(R0, anl - mulc(Rj, anl));
      if constexpr (AXES) { ja[d] = mulc(R0, axl); jo[d] = x0 + mulc(R0, anl); }
    } else if constexpr (jt == 1) {
      const f3 axl = pk3<T::AXIS, i>(L);
      k.Rm[i] = R0;
      k.x[i] = x0 + s.q[d] * mulc(R0, axl);
      if constexpr (AXES) { ja[d] = mulc(R0, axl); jo[d] = x0; }
    } else {
      k.Rm[i] = R0;
      k.x[i] = x0;
    }
    k.c[i] = k.x[i] + mulc(k.Rm[i], pk3<T::COM, i>(L));
  });
}

// ------------------------------------------------------------------ contact rows
// Row r of the wave's 16 envs (LDS, one region per row of ES * W words):
//   P: 64 lanes x PW words, lane L = 4 e + k at PW * L: this lane's branch slot y_branch
//      (NDB words: the owner branch's y, zeros in the other three lanes) | base slice
//      (components k and k + 4 of y_base; lanes 2 and 3 hold a zero for k + 4)
//   S: 16 envs x 4 words at 64 PW + 4 e: m_eff | target | lambda | mu (the contact's friction)
// With PW = 4 (Ant: NDB = 2) a lane reads its whole P with one ds_read_b128 and its env's S
// with another (the quad's four lanes read the same S address: a broadcast); every 16-lane
// b128 group covers 16 distinct 16-B slots of the 256-B bank row, so a row load has no bank
// conflict (the round-2 [word][env] layout put the quad's four branch slots on one bank:
// 4-way conflicts, 47 % of LDS-active cycles).  Rows beyond the LDS capacity live in the
// device workspace, [word][env] with the same word order (P of lanes 0..3, then S).
// Row update: one quad reduction of the lane's slice dot, no owner test (the non-owner lanes'
// branch words are zero).
template <class R, int ES>
struct TRows {
  using T = Team<R>;
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  static constexpr int NDB = T::NDB, NC = T::NC, MR = 3 * T::NC, ES_ = ES;
  static constexpr int PW = NDB + 2;    // per-lane words of a row
  static constexpr int W = 4 * PW + 4;  // words per env per row (P of its 4 lanes + S)
  static constexpr int SOFF = 4 * ES * PW;  // S block within a row region
  // float64 (PL): a lane's P record (4 doubles, 32 B) as two 16-B planes -- branch words, then the
  // base slice -- and the S record as (m_eff, target) and (lambda, mu) planes, so every b128 access
  // of 64 lanes strides 16 B (with 32-B records every access was a 2-way LDS bank conflict, 48 % of
  // the float64 kernel's LDS-active cycles)
  static constexpr bool PL = sizeof(Sc) == 8 && PW == 4;
  static constexpr int P1OFF = 2 * 4 * ES;           // PL: the base-slice plane (words)
  static constexpr int LAMO = PL ? 2 * ES : 2;       // lambda's word offset from the (m_eff, target) pair
  static constexpr int HEAD = 0;        // per-env words before the rows (pack staging overlaps the rows)
  static_assert(NC <= 32, "contact_sweep keeps one bit per contact in a 32-bit mask");
  static constexpr int WORDS = MR * W;  // device workspace words per env
  typedef Sc v4f __attribute__((ext_vector_type(4)));
  typedef Sc v2f __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) v4f LW4;
  typedef __attribute__((address_space(3))) v2f LW2;
  LW* lds;   // LDS base + env slot (pack staging, [word][env])
  LW* rows;  // LDS base of the wave's row regions
  Sc* gbl;       // workspace base + env
  int n;
  int cap;          // rows resident in LDS
  int lane;         // lane in the wave (4 e + k)
  PBG_DEV LW& stage(int w) const { return lds[(size_t)w * ES]; }
  // row offsets by a 24-bit multiply (rows < 2^24): the 32-bit v_mul_lo_u32 the compiler chose for
  // an unbounded row index is a quarter-rate instruction, two of them per normal row of the sweep
  PBG_DEV int roff(int r) const { return (int)__umul24((unsigned)r, (unsigned)(ES * W)); }
  PBG_DEV LW* P(int r) const { return rows + roff(r) + (PL ? 2 : PW) * lane; }
  PBG_DEV LW* S(int r) const { return rows + roff(r) + SOFF + (PL ? 2 : 4) * (lane >> 2); }
  // row words of lane k in the workspace ([word][env], stride n)
  PBG_DEV Sc* gP(int r, int k) const { return gbl + ((size_t)r * W + (size_t)k * PW) * n; }
  PBG_DEV Sc* gS(int r) const { return gbl + ((size_t)r * W + 4 * PW) * n; }
  // slot: the writing lane's branch for a branch contact (the owner writes all four lanes'
  // P), -1 for a base contact (every lane of the quad writes, each its own P)
  PBG_DEV void put(int r, int slot, const Sc* yb, const Sc* yB, Sc meff, Sc target, Sc mu) const {
    const int k0 = lane & 3;
    auto pw = [&](int k, int i) -> Sc {  // word i of lane k's P
      if (i < NDB) return k == slot ? yb[i] : 0.f;
      if (i == NDB) return yB[k];
      return k < 2 ? yB[k + 4] : 0.f;
    };
    if (r < cap && PL) {
      LW* p0 = rows + roff(r) + 2 * (lane & ~3);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (slot < 0 && k != k0) continue;
        *(LW2*)(p0 + 2 * k) = v2f{pw(k, 0), pw(k, 1)};
        *(LW2*)(p0 + P1OFF + 2 * k) = v2f{pw(k, 2), pw(k, 3)};
      }
      *(LW2*)S(r) = v2f{meff, target};
      *(LW2*)(S(r) + LAMO) = v2f{0.f, mu};
    } else if (r < cap) {
      LW* p0 = rows + roff(r) + PW * (lane & ~3);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (slot < 0 && k != k0) continue;
        Sc v[PW];
#pragma unroll
        for (int i = 0; i < PW; i++) v[i] = pw(k, i);
        if constexpr (PW == 4) {
          *(LW4*)(p0 + PW * k) = v4f{v[0], v[1], v[2], v[3]};
        } else {
#pragma unroll
          for (int i = 0; i < PW; i++) p0[PW * k + i] = v[i];
        }
      }
      *(LW4*)S(r) = v4f{meff, target, 0.f, mu};
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (slot < 0 && k != k0) continue;
        Sc* q = gP(r, k);
#pragma unroll
        for (int i = 0; i < PW; i++) q[(size_t)i * n] = pw(k, i);
      }
      Sc* q = gS(r);
      q[0] = meff; q[n] = target; q[2 * (size_t)n] = 0.f; q[3 * (size_t)n] = mu;
    }
  }
  // One row in registers (loaded ahead of its update: PGS software pipelining): this
  // lane's branch slot and base slice.
  struct Row {
    Sc yb[NDB], yB[2], meff, tgt, lam;
  };
  // LDS: every row of the wave is resident (the common case, no workspace branches)
  template <bool LDS>
  PBG_DEV void load(int r, int kb, Row& row) const {
    if (LDS || r < cap) {
      if constexpr (PL) {
        const v2f a = *(const LW2*)P(r), c = *(const LW2*)(P(r) + P1OFF);
        row.yb[0] = a.x; row.yb[1] = a.y; row.yB[0] = c.x; row.yB[1] = c.y;
      } else if constexpr (PW == 4) {
        const v4f a = *(const LW4*)P(r);
        row.yb[0] = a.x; row.yb[1] = a.y; row.yB[0] = a.z; row.yB[1] = a.w;
      } else {
        const LW* p = P(r);
#pragma unroll
        for (int i = 0; i < NDB; i++) row.yb[i] = p[i];
        row.yB[0] = p[NDB]; row.yB[1] = p[NDB + 1];
      }
      // m_eff and target as one b64, lambda as a b32: a b128 whose fourth register (mu) is
      // dead lets the allocator reuse it at once, and the write-after-write on the pending
      // load forces an lgkmcnt(0) wait right behind the look-ahead load (no pipelining)
      const v2f b = *(const LW2*)S(r);
      row.meff = b.x; row.tgt = b.y; row.lam = S(r)[LAMO];
    } else {
      const Sc* p = gP(r, kb);
#pragma unroll
      for (int i = 0; i < NDB; i++) row.yb[i] = p[(size_t)i * n];
      row.yB[0] = p[(size_t)NDB * n]; row.yB[1] = p[(size_t)(NDB + 1) * n];
      const Sc* q = gS(r);
      row.meff = q[0]; row.tgt = q[n]; row.lam = q[2 * (size_t)n];
    }
  }
  // LDS-resident row at word offset o of the wave's row regions (P(r) = rows + o, o = roff(r) +
  // PW * lane; its S record at o + sdelta()): the normal sweep steps o by a compile-time stride
  // instead of recomputing the row address from the row index
  PBG_DEV int poff(int r) const { return roff(r) + (PL ? 2 : PW) * lane; }
  PBG_DEV int sdelta() const { return SOFF + (PL ? 2 : 4) * (lane >> 2) - (PL ? 2 : PW) * lane; }
  static PBG_DEV void load_at(const LW* p, const LW* q, Row& row) {
    if constexpr (PL) {
      const v2f a = *(const LW2*)p, c = *(const LW2*)(p + P1OFF);
      row.yb[0] = a.x; row.yb[1] = a.y; row.yB[0] = c.x; row.yB[1] = c.y;
    } else {
      const v4f a = *(const LW4*)p;
      row.yb[0] = a.x; row.yb[1] = a.y; row.yB[0] = a.z; row.yB[1] = a.w;
    }
    const v2f b = *(const LW2*)q;
    row.meff = b.x; row.tgt = b.y; row.lam = q[LAMO];
  }
  template <bool LDS>
  PBG_DEV void set_lam(int r, Sc v) const {
    if (LDS || r < cap) S(r)[LAMO] = v;
    else gS(r)[2 * (size_t)n] = v;
  }
  // friction bound of contact c: mu * lambda of its normal row (one ds_read_b64)
  template <bool LDS>
  PBG_DEV Sc fric_limit(int c) const {
    if (LDS || 3 * c < cap) {
      const v2f v = *(const LW2*)(S(3 * c) + LAMO);
      return v.y * v.x;
    }
    const Sc* q = gS(3 * c);
    return q[3 * (size_t)n] * q[2 * (size_t)n];
  }
  // projected Gauss-Seidel update of a loaded row (u: the branch part ub, the base slice
  // uBs); returns the new impulse, bitwise identical in the four lanes
  static PBG_DEV Sc update(const Row& r, Sc* ub, Sc* uBs, Sc lo, Sc hi) {
    Sc part = r.yB[0] * uBs[0] + r.yB[1] * uBs[1];
#pragma unroll
    for (int i = 0; i < NDB; i++) part += r.yb[i] * ub[i];
    const Sc yu = quad_sum(part);
    const Sc nl = clampf(r.lam + r.meff * (r.tgt - yu), lo, hi);
    const Sc dl = nl - r.lam;
    uBs[0] += r.yB[0] * dl;
    uBs[1] += r.yB[1] * dl;
#pragma unroll
    for (int i = 0; i < NDB; i++) ub[i] += r.yb[i] * dl;
    return nl;
  }
};

// y_base = Lbb^-1 t (6x6 lower, reciprocal diagonal)
template <class Sc>
PBG_DEV void fwd6(const Sc (&Lbb)[6][6], const Sc* Ldb, Sc* t) {
  static_for<0, 6>([&](auto g_c) {
    constexpr int g = decltype(g_c)::value;
    Sc v = t[g];
    static_for<0, g>([&](auto h_c) { v -= Lbb[g][decltype(h_c)::value] * t[decltype(h_c)::value]; });
    t[g] = v * Ldb[g];
  });
}

// One PGS sweep over the contact rows in Bullet's order: all normals, then the two
// friction rows of each contact whose normal impulse is positive, box-clamped at mu*lambda_n.
// Rows are loaded one step ahead of their update (two register buffers alternate, so LDS
// latency overlaps the previous update); the normal pass records which impulses came out
// positive, so the friction pass walks those contacts without a load-then-test round trip.
template <bool LDS, class RW>
PBG_DEV void contact_sweep(const RW& rw, int nc, int kb, typename RW::Sc* ub, typename RW::Sc* uB SUB_STAMP_ARGS) {
  using Sc = typename RW::Sc;
  using LW = typename RW::LW;
  using Row = typename RW::Row;
  if (nc <= 0) return;
  // The look-ahead loads are unconditional (the last row re-reads itself): a prefetch under a
  // branch makes the compiler's LDS wait at the join conservative (lgkmcnt(0)), which
  // serialises every row behind the next row's loads.
  uint32_t pos = 0;
  if constexpr (LDS && RW::PW == 4) {
    // normal rows 0, 3, 6, ...: word offsets stepped by the compile-time row stride, the look-ahead
    // clamped at the last normal row (an add and a min per row instead of the index arithmetic)
    constexpr int NS = 3 * RW::ES_ * RW::W;
    const int sd = rw.sdelta();
    const LW* plast = rw.rows + rw.poff(3 * (nc - 1));
    const LW *pA = rw.rows + rw.poff(0), *pB;
    LW *qA = (LW*)pA + sd, *qB;
    Row A, B;
    RW::load_at(pA, qA, A);
    int c = 0;
    while (true) {
      pB = pA + NS < plast ? pA + NS : plast;
      qB = (LW*)pB + sd;
      RW::load_at(pB, qB, B);
      Sc nl = RW::update(A, ub, uB, 0.f, 3.0e38f);
      qA[RW::LAMO] = nl;
      pos |= (nl > 0.f ? 1u : 0u) << c;
      if (++c >= nc) break;
      pA = pB + NS < plast ? pB + NS : plast;
      qA = (LW*)pA + sd;
      RW::load_at(pA, qA, A);
      nl = RW::update(B, ub, uB, 0.f, 3.0e38f);
      qB[RW::LAMO] = nl;
      pos |= (nl > 0.f ? 1u : 0u) << c;
      if (++c >= nc) break;
    }
  } else {
    Row A, B;
    rw.template load<LDS>(0, kb, A);
    int c = 0;
    while (true) {
      rw.template load<LDS>(3 * min(c + 1, nc - 1), kb, B);
      Sc nl = RW::update(A, ub, uB, 0.f, 3.0e38f);
      rw.template set_lam<LDS>(3 * c, nl);
      pos |= (nl > 0.f ? 1u : 0u) << c;
      if (++c >= nc) break;
      rw.template load<LDS>(3 * min(c + 1, nc - 1), kb, A);
      nl = RW::update(B, ub, uB, 0.f, 3.0e38f);
      rw.template set_lam<LDS>(3 * c, nl);
      pos |= (nl > 0.f ? 1u : 0u) << c;
      if (++c >= nc) break;
    }
  }
  STAMP(12)
  // [EXT] friction rows only under a positive normal impulse
  if (pos == 0u) return;
  // two register sets alternate (no copies between iterations)
  int c = __builtin_ctz(pos);
  pos &= pos - 1u;
  Row A1, A2, B1, B2;
  rw.template load<LDS>(3 * c + 1, kb, A1);
  rw.template load<LDS>(3 * c + 2, kb, A2);
  Sc limA = rw.template fric_limit<LDS>(c), limB;
  while (true) {
    bool more = pos != 0u;
    int c2 = more ? __builtin_ctz(pos) : c;
    pos &= pos - 1u;
    rw.template load<LDS>(3 * c2 + 1, kb, B1);
    rw.template load<LDS>(3 * c2 + 2, kb, B2);
    limB = rw.template fric_limit<LDS>(c2);
    rw.template set_lam<LDS>(3 * c + 1, RW::update(A1, ub, uB, -limA, limA));
    rw.template set_lam<LDS>(3 * c + 2, RW::update(A2, ub, uB, -limA, limA));
    if (!more) break;
    c = c2;
    more = pos != 0u;
    c2 = more ? __builtin_ctz(pos) : c;
    pos &= pos - 1u;
    rw.template load<LDS>(3 * c2 + 1, kb, A1);
    rw.template load<LDS>(3 * c2 + 2, kb, A2);
    limA = rw.template fric_limit<LDS>(c2);
    rw.template set_lam<LDS>(3 * c + 1, RW::update(B1, ub, uB, -limB, limB));
    rw.template set_lam<LDS>(3 * c + 2, RW::update(B2, ub, uB, -limB, limB));
    if (!more) break;
    c = c2;
  }
}

// ------------------------------------------------------------------ one physics sub-step
template <class R, int ES>
PBG_DEV int team_substep(TState<R>& s, const Lane& L, const real_t<R>* tau, uint32_t& slot_bits, uint32_t& base_bits,
                         const TRows<R, ES>& rw, const SimPT<real_t<R>>& P SUB_STAMP_ARGS) {
  using Sc = real_t<R>;
  using f3 = V3<Sc>;
  using m3 = M3<Sc>;
  using s6 = S6<Sc>;
  using T = Team<R>;
  constexpr int NDB = T::NDB, NLB = T::NLB;
  const Sc dt = P.dt;
  const Sc g = P.gravity;
  const int kb = L.k;
  // contact detection (float32: where the rows are built; float64: right after phase A, so the
  // branch's kinematic records die before the mass matrix is built)
  int n0 = 0, ci = 0, nc = 0;
  uint32_t act = 0;
  Sc sdist[T::NSB > 0 ? T::NSB : 1];
  f3 sP[T::NSB > 0 ? T::NSB : 1];
  constexpr bool OWN = sizeof(Sc) == 8;  // the float64 ordering and limit-row layout (below)

  // --- phase A: branch kinematics, velocities, bias accelerations; composites of the
  // branch's dof-owning links and the branch total (all about O = base COM)
  const m3 Rb = quat_to_m3(s.bq[0], s.bq[1], s.bq[2], s.bq[3]);
  const f3 O = mk3<Sc>(s.bp[0], s.bp[1], s.bp[2]);
  const f3 w0 = mk3<Sc>(s.bw[0], s.bw[1], s.bw[2]), v0 = mk3<Sc>(s.bv[0], s.bv[1], s.bv[2]);
  TKin<R> k;
  f3 ja[NDB], jo[NDB];
  Sc cmass[NLB];
  f3 cp1[NLB], cF[NLB], cN[NLB];
  s6 cJ[NLB];
  Sc tm = 0.f;
  f3 tp1 = mk3<Sc>(0, 0, 0), tF = mk3<Sc>(0, 0, 0), tN = mk3<Sc>(0, 0, 0);
  s6 tJ;
#pragma unroll
  for (int i = 0; i < 6; i++) tJ.a[i] = 0.f;
  static_for<0, NLB>([&](auto i_c) {
    constexpr int i = decltype(i_c)::value;
    if constexpr (T::owner(i)) {
      cmass[i] = 0.f; cp1[i] = mk3<Sc>(0, 0, 0); cF[i] = mk3<Sc>(0, 0, 0); cN[i] = mk3<Sc>(0, 0, 0);
#pragma unroll
      for (int c = 0; c < 6; c++) cJ[i].a[c] = 0.f;
    }
  });
  {
    f3 w[NLB], v[NLB], al[NLB], ac[NLB];
    static_for<0, NLB>([&](auto i_c) {
      constexpr int i = decltype(i_c)::value;
      constexpr int p = R::link_parent[i], jt = R::link_jtype[i], d = R::link_dof[i];
      const m3& Rp = p < 0 ? Rb : k.Rm[p < 0 ? 0 : p];
      const f3 xp = p < 0 ? O : k.x[p < 0 ? 0 : p];
      const f3 cp = p < 0 ? O : k.c[p < 0 ? 0 : p];
      const f3 wp = p < 0 ? w0 : w[p < 0 ? 0 : p], vp = p < 0 ? v0 : v[p < 0 ? 0 : p];
      const f3 alp = p < 0 ? mk3<Sc>(0, 0, 0) : al[p < 0 ? 0 : p], acp = p < 0 ? mk3<Sc>(0, 0, 0) : ac[p < 0 ? 0 : p];
      m3 Ro;
      static_for<0, 9>([&](auto c_c) { Ro.m[decltype(c_c)::value] = pk<T::ROT, 9 * i + decltype(c_c)::value>(L); });
      const m3 R0 = mulc(Rp, Ro);
      const f3 x0 = xp + mulc(Rp, pk3<T::OFFP, i>(L));
      if constexpr (jt == 0) {
        const f3 axl = pk3<T::AXIS, i>(L), anl = pk3<T::ANCH, i>(L);
        const m3 Rj = axis_angle_m3c(axl.x, axl.y, axl.z, s.q[d]);
        k.Rm[i] = mul(R0, Rj);
        k.x[i] = x0 + mul(R0, anl - mulc(Rj, anl));
        k.c[i] = k.x[i] + mulc(k.Rm[i], pk3<T::COM, i>(L));
        const f3 a = mulc(R0, axl);
        const f3 o = x0 + mulc(R0, anl);
        ja[d] = a;
        jo[d] = o;
        const f3 ro = o - cp;
        const f3 vo = vp + cross3(wp, ro);
        const f3 ao = acp + cross3(alp, ro) + cross3(wp, cross3(wp, ro));
        const f3 wl = wp + s.qd[d] * a;
        const f3 all = alp + s.qd[d] * cross3(wp, a);
        const f3 rc = k.c[i] - o;
        w[i] = wl;
        al[i] = all;
        v[i] = vo + cross3(wl, rc);
        ac[i] = ao + cross3(all, rc) + cross3(wl, cross3(wl, rc));
      } else if constexpr (jt == 1) {
        const f3 axl = pk3<T::AXIS, i>(L);
        k.Rm[i] = R0;
        const f3 a = mulc(R0, axl);
        k.x[i] = x0 + s.q[d] * a;
        k.c[i] = k.x[i] + mulc(k.Rm[i], pk3<T::COM, i>(L));
        ja[d] = a;
        jo[d] = x0;
        const f3 r = k.c[i] - cp;
        w[i] = wp;
        al[i] = alp;
        v[i] = vp + cross3(wp, r) + s.qd[d] * a;
        ac[i] = acp + cross3(alp, r) + cross3(wp, cross3(wp, r)) + (2.f * s.qd[d]) * cross3(wp, a);
      } else {
        k.Rm[i] = R0;
        k.x[i] = x0;
        k.c[i] = k.x[i] + mulc(k.Rm[i], pk3<T::COM, i>(L));
        const f3 r = k.c[i] - cp;
        w[i] = wp;
        al[i] = alp;
        v[i] = vp + cross3(wp, r);
        ac[i] = acp + cross3(alp, r) + cross3(wp, cross3(wp, r));
      }
      if constexpr (R::link_mass[i] > 0.0) {
        const Sc m = pk<T::MASS, i>(L);
        Sc I6[6];
        static_for<0, 6>([&](auto c_c) { I6[decltype(c_c)::value] = pk<T::INER, 6 * i + decltype(c_c)::value>(L); });
        const s6 Iw = rotate_inertia(k.Rm[i], I6);
        const f3 r = k.c[i] - O;
        const Sc rr = dot3(r, r);
        s6 J;
        J.a[0] = Iw.a[0] + m * (rr - r.x * r.x);
        J.a[1] = Iw.a[1] + m * (rr - r.y * r.y);
        J.a[2] = Iw.a[2] + m * (rr - r.z * r.z);
        J.a[3] = Iw.a[3] - m * r.x * r.y;
        J.a[4] = Iw.a[4] - m * r.x * r.z;
        J.a[5] = Iw.a[5] - m * r.y * r.z;
        const f3 Iww = mul(Iw, w[i]);
        const f3 f = m * (ac[i] - mk3<Sc>(0, 0, -g)) +
                     (m * ((Sc)PBG_LINEAR_DAMPING + (Sc)PBG_LINEAR_DAMPING * norm3(v[i]))) * v[i];
        const f3 n = mul(Iw, al[i]) + cross3(w[i], Iww) +
                     ((Sc)PBG_ANGULAR_DAMPING + (Sc)PBG_ANGULAR_DAMPING * norm3(w[i])) * Iww;
        const f3 pr = m * r, Nn = n + cross3(r, f);
        static_for<0, NLB>([&](auto a_c) {
          constexpr int a = decltype(a_c)::value;
          if constexpr (T::owner(a) && T::anc(a, i)) {
            cmass[a] += m; cp1[a] += pr; cF[a] += f; cN[a] += Nn;
#pragma unroll
            for (int c = 0; c < 6; c++) cJ[a].a[c] += J.a[c];
          }
        });
        tm += m; tp1 += pr; tF += f; tN += Nn;
#pragma unroll
        for (int c = 0; c < 6; c++) tJ.a[c] += J.a[c];
      }
      PBG_PHASE_BARRIER
    });
  }
  // whole-robot composite = sum of the branch totals + the base body (at O: r = 0)
  {
    tm = quad_sum(tm);
    tp1 = mk3<Sc>(quad_sum(tp1.x), quad_sum(tp1.y), quad_sum(tp1.z));
    tF = mk3<Sc>(quad_sum(tF.x), quad_sum(tF.y), quad_sum(tF.z));
    tN = mk3<Sc>(quad_sum(tN.x), quad_sum(tN.y), quad_sum(tN.z));
#pragma unroll
    for (int c = 0; c < 6; c++) tJ.a[c] = quad_sum(tJ.a[c]);
    const Sc m = (Sc)R::base_mass;
    const s6 Iw = rotate_inertia(Rb, R::base_inertia);
    const f3 Iww = mul(Iw, w0);
    const f3 f = m * (mk3<Sc>(0, 0, g)) + (m * ((Sc)PBG_LINEAR_DAMPING + (Sc)PBG_LINEAR_DAMPING * norm3(v0))) * v0;
    const f3 n = cross3(w0, Iww) + ((Sc)PBG_ANGULAR_DAMPING + (Sc)PBG_ANGULAR_DAMPING * norm3(w0)) * Iww;
    tm += m; tF += f; tN += n;
#pragma unroll
    for (int c = 0; c < 6; c++) tJ.a[c] += Iw.a[c];
  }
  TRACE64(0, 0, tm); TRACE64(0, 1, tp1.x); TRACE64(0, 2, tF.x); TRACE64(0, 3, tF.z); TRACE64(0, 4, tN.y);
  TRACE64(0, 5, tJ.a[0]); TRACE64(0, 6, tJ.a[5]); TRACE64(0, 7, kb);

  // this branch's active slots, then their contact indices (exclusive quad prefix)
  auto detect_branch = [&]() {
    act = 0;
    static_for<0, T::NSB>([&](auto sl_c) {
      constexpr int sl = decltype(sl_c)::value;
      constexpr int li = R::slot_link[T::NS0 + sl];
      const f3 cc = k.x[li] + mulc(k.Rm[li], pk3<T::SPT, sl>(L));
      const Sc rad = pk<T::SRAD, sl>(L);
      sdist[sl] = cc.z - rad;
      sP[sl] = mk3<Sc>(cc.x, cc.y, cc.z - rad);
      act |= (sdist[sl] < (Sc)PBG_CONTACT_THRESHOLD ? 1u : 0u) << sl;
    });
    const int cnt = __builtin_popcount(act);
    const int c0 = quad_bcast_i<0>(cnt), c1 = quad_bcast_i<1>(cnt), c2 = quad_bcast_i<2>(cnt), c3 = quad_bcast_i<3>(cnt);
    ci = n0 + (kb > 0 ? c0 : 0) + (kb > 1 ? c1 : 0) + (kb > 2 ? c2 : 0);
    nc = n0 + c0 + c1 + c2 + c3;
    slot_bits = act;
  };
  if constexpr (OWN) {
    n0 = 0;
    base_bits = 0;
    static_for<0, T::NS0>([&](auto sl_c) {
      constexpr int sl = decltype(sl_c)::value;
      const f3 cc = O + mulc(Rb, (Sc)R::slot_point[sl][0], (Sc)R::slot_point[sl][1], (Sc)R::slot_point[sl][2]);
      if (cc.z - (Sc)R::slot_radius[sl] < (Sc)PBG_CONTACT_THRESHOLD) {
        base_bits |= 1u << sl;
        n0++;
      }
    });
    detect_branch();
  }
  TRACE64(1, 0, n0); TRACE64(1, 1, nc); TRACE64(1, 2, ci); TRACE64(1, 3, act); TRACE64(1, 4, base_bits);
  TRACE64(1, 5, sdist[0]); TRACE64(1, 6, sP[0].x); TRACE64(1, 7, sP[0].z);

  STAMP(0)
  // --- mass matrix: branch block Lbr, base-branch block Lgb, base block Mbb; bias -------
  Sc Lbr[NDB][NDB], Lgb[6][NDB], Mbb[6][6];
  Sc rb[NDB], rB[6];
  f3 sw[NDB], sv[NDB];
  static_for<0, NDB>([&](auto a_c) {
    constexpr int a = decltype(a_c)::value;
    constexpr int d = T::dof_of(a);
    if constexpr (R::dof_jtype[d] == 0) { sw[a] = ja[d]; sv[a] = cross3(jo[d] - O, ja[d]); }
    else { sw[a] = mk3<Sc>(0, 0, 0); sv[a] = ja[d]; }
  });
  static_for<0, NDB>([&](auto a_c) {
    constexpr int a = decltype(a_c)::value;
    constexpr int ia = R::dof_link[T::dof_of(a)];
    rb[a] = -(dot3(sw[a], cN[ia]) + dot3(sv[a], cF[ia]));
    static_for<0, a + 1>([&](auto b_c) {
      constexpr int b = decltype(b_c)::value;
      if constexpr (T::coupled(a, b)) {
        constexpr int ibk = R::dof_link[T::dof_of(b)];
        const f3 Jw_ = mul(cJ[ibk], sw[b]) + cross3(cp1[ibk], sv[b]);
        const f3 Fv = cmass[ibk] * sv[b] - cross3(cp1[ibk], sw[b]);
        Lbr[a][b] = dot3(sw[a], Jw_) + dot3(sv[a], Fv);
      }
    });
    // base rows g against this dof (the dof's composite): lin g -> Fv_g, ang g -> Jw_g
    const f3 Jw_ = mul(cJ[ia], sw[a]) + cross3(cp1[ia], sv[a]);
    const f3 Fv = cmass[ia] * sv[a] - cross3(cp1[ia], sw[a]);
    Lgb[0][a] = Fv.x; Lgb[1][a] = Fv.y; Lgb[2][a] = Fv.z;
    Lgb[3][a] = Jw_.x; Lgb[4][a] = Jw_.y; Lgb[5][a] = Jw_.z;
  });
  // base block (lower): lin-lin m I; ang-lin p1 x e_h; ang-ang J
  Mbb[0][0] = tm; Mbb[1][1] = tm; Mbb[2][2] = tm;
  Mbb[1][0] = 0.f; Mbb[2][0] = 0.f; Mbb[2][1] = 0.f;
  Mbb[3][0] = 0.f;      Mbb[4][0] = tp1.z;  Mbb[5][0] = -tp1.y;  // p1 x e_x = (0, p1z, -p1y)
  Mbb[3][1] = -tp1.z;   Mbb[4][1] = 0.f;    Mbb[5][1] = tp1.x;   // p1 x e_y = (-p1z, 0, p1x)
  Mbb[3][2] = tp1.y;    Mbb[4][2] = -tp1.x; Mbb[5][2] = 0.f;     // p1 x e_z = (p1y, -p1x, 0)
  Mbb[3][3] = tJ.a[0]; Mbb[4][4] = tJ.a[1]; Mbb[5][5] = tJ.a[2];
  Mbb[4][3] = tJ.a[3]; Mbb[5][3] = tJ.a[4]; Mbb[5][4] = tJ.a[5];
  rB[0] = -tF.x; rB[1] = -tF.y; rB[2] = -tF.z;
  rB[3] = -tN.x; rB[4] = -tN.y; rB[5] = -tN.z;
  static_for<0, NDB>([&](auto j_c) {
    constexpr int j = decltype(j_c)::value;
    constexpr int a = T::lg(j);
    Lbr[a][a] += pk<T::ARM, j>(L);
    rb[a] += tau[j] - pk<T::DAMP, j>(L) * s.qd[j];
    if constexpr (has_springs<R>()) rb[a] -= pk<T::STIFF, j>(L) * s.q[j];  // mjcf.py B7
  });
  TRACE64(2, 0, Lbr[0][0]); TRACE64(2, 1, Lbr[NDB - 1][0]); TRACE64(2, 2, Lbr[NDB - 1][NDB - 1]);
  TRACE64(2, 3, Lgb[0][0]); TRACE64(2, 4, Lgb[5][NDB - 1]); TRACE64(2, 5, Mbb[3][3]); TRACE64(2, 6, rb[0]);
  TRACE64(2, 7, rB[2]);

  STAMP(1)
  // --- Cholesky: branch columns (lane), Schur complement of the base (quad sum), 6x6 ----
  Sc Ld[NDB];
  static_for<0, NDB>([&](auto b_c) {
    constexpr int b = decltype(b_c)::value;
    Sc sbb = Lbr[b][b];
    static_for<0, b>([&](auto k_c) {
      constexpr int kk = decltype(k_c)::value;
      if constexpr (T::coupled(b, kk)) sbb -= Lbr[b][kk] * Lbr[b][kk];
    });
    const Sc lbb = fast_sqrt(sbb);
    const Sc inv = fast_rcp(lbb);
    Ld[b] = inv;
    Lbr[b][b] = lbb;
    static_for<b + 1, NDB>([&](auto a_c) {
      constexpr int a = decltype(a_c)::value;
      if constexpr (T::coupled(a, b)) {
        Sc t = Lbr[a][b];
        static_for<0, b>([&](auto k_c) {
          constexpr int kk = decltype(k_c)::value;
          if constexpr (T::coupled(a, kk) && T::coupled(b, kk)) t -= Lbr[a][kk] * Lbr[b][kk];
        });
        Lbr[a][b] = t * inv;
      }
    });
#pragma unroll
    for (int gg = 0; gg < 6; gg++) {
      Sc t = Lgb[gg][b];
      static_for<0, b>([&](auto k_c) {
        constexpr int kk = decltype(k_c)::value;
        if constexpr (T::coupled(b, kk)) t -= Lgb[gg][kk] * Lbr[b][kk];
      });
      Lgb[gg][b] = t * inv;
    }
  });
  Sc Lbb[6][6], Ldb[6];
  static_for<0, 6>([&](auto g_c) {
    constexpr int gg = decltype(g_c)::value;
    static_for<0, gg + 1>([&](auto h_c) {
      constexpr int h = decltype(h_c)::value;
      Sc c = 0.f;
#pragma unroll
      for (int b = 0; b < NDB; b++) c += Lgb[gg][b] * Lgb[h][b];
      Lbb[gg][h] = Mbb[gg][h] - quad_sum(c);
    });
  });
  static_for<0, 6>([&](auto j_c) {
    constexpr int j = decltype(j_c)::value;
    Sc sjj = Lbb[j][j];
    static_for<0, j>([&](auto k_c) { sjj -= Lbb[j][decltype(k_c)::value] * Lbb[j][decltype(k_c)::value]; });
    const Sc ljj = fast_sqrt(sjj);
    const Sc inv = fast_rcp(ljj);
    Ldb[j] = inv;
    Lbb[j][j] = ljj;
    static_for<j + 1, 6>([&](auto i_c) {
      constexpr int i = decltype(i_c)::value;
      Sc t = Lbb[i][j];
      static_for<0, j>([&](auto k_c) { t -= Lbb[i][decltype(k_c)::value] * Lbb[j][decltype(k_c)::value]; });
      Lbb[i][j] = t * inv;
    });
  });

  TRACE64(3, 0, Ld[0]); TRACE64(3, 1, Ld[NDB - 1]); TRACE64(3, 2, Lbb[0][0]); TRACE64(3, 3, Lbb[5][5]);
  TRACE64(3, 4, Ldb[5]); TRACE64(3, 5, Lbb[5][3]); TRACE64(3, 6, Lgb[2][0]); TRACE64(3, 7, Lbr[NDB - 1][0]);
  // --- unconstrained velocity nu_pred = nu + dt M^-1 (tau - C); u = L^T nu_pred --------
  Sc yb[NDB], yB[6];
  static_for<0, NDB>([&](auto a_c) {
    constexpr int a = decltype(a_c)::value;
    Sc t = rb[a];
    static_for<0, a>([&](auto k_c) {
      constexpr int kk = decltype(k_c)::value;
      if constexpr (T::coupled(a, kk)) t -= Lbr[a][kk] * yb[kk];
    });
    yb[a] = t * Ld[a];
  });
#pragma unroll
  for (int gg = 0; gg < 6; gg++) {
    Sc c = 0.f;
#pragma unroll
    for (int b = 0; b < NDB; b++) c += Lgb[gg][b] * yb[b];
    yB[gg] = rB[gg] - quad_sum(c);
  }
  fwd6(Lbb, Ldb, yB);
  Sc xB[6], xb[NDB];
  static_for<0, 6>([&](auto r_c) {
    constexpr int gg = 5 - decltype(r_c)::value;
    Sc t = yB[gg];
    static_for<gg + 1, 6>([&](auto h_c) { t -= Lbb[decltype(h_c)::value][gg] * xB[decltype(h_c)::value]; });
    xB[gg] = t * Ldb[gg];
  });
  static_for<0, NDB>([&](auto r_c) {
    constexpr int a = NDB - 1 - decltype(r_c)::value;
    Sc t = yb[a];
    static_for<a + 1, NDB>([&](auto k_c) {
      constexpr int kk = decltype(k_c)::value;
      if constexpr (T::coupled(kk, a)) t -= Lbr[kk][a] * xb[kk];
    });
#pragma unroll
    for (int gg = 0; gg < 6; gg++) t -= Lgb[gg][a] * xB[gg];
    xb[a] = t * Ld[a];
  });
  Sc nb[NDB], nB[6];
  static_for<0, NDB>([&](auto j_c) {
    constexpr int j = decltype(j_c)::value;
    constexpr int a = T::lg(j);
    nb[a] = clampf(s.qd[j] + dt * xb[a], -(Sc)PBG_MAX_COORD_VELOCITY, (Sc)PBG_MAX_COORD_VELOCITY);
  });
#pragma unroll
  for (int i = 0; i < 3; i++) {
    nB[i] = clampf(s.bv[i] + dt * xB[i], -(Sc)PBG_MAX_COORD_VELOCITY, (Sc)PBG_MAX_COORD_VELOCITY);
    nB[3 + i] = clampf(s.bw[i] + dt * xB[3 + i], -(Sc)PBG_MAX_COORD_VELOCITY, (Sc)PBG_MAX_COORD_VELOCITY);
  }
  Sc ub[NDB], uB[6];
  static_for<0, NDB>([&](auto a_c) {
    constexpr int a = decltype(a_c)::value;
    Sc t = 0.f;
    static_for<a, NDB>([&](auto k_c) {
      constexpr int kk = decltype(k_c)::value;
      if constexpr (T::coupled(kk, a)) t += Lbr[kk][a] * nb[kk];
    });
#pragma unroll
    for (int gg = 0; gg < 6; gg++) t += Lgb[gg][a] * nB[gg];
    ub[a] = t;
  });
  static_for<0, 6>([&](auto g_c) {
    constexpr int gg = decltype(g_c)::value;
    Sc t = 0.f;
    static_for<gg, 6>([&](auto h_c) { t += Lbb[decltype(h_c)::value][gg] * nB[decltype(h_c)::value]; });
    uB[gg] = t;
  });
  TRACE64(4, 0, yb[0]); TRACE64(4, 1, yB[0]); TRACE64(4, 2, xB[2]); TRACE64(4, 3, xb[0]); TRACE64(4, 4, nB[2]);
  TRACE64(4, 5, nb[0]); TRACE64(4, 6, ub[0]); TRACE64(4, 7, uB[5]);

  STAMP(2)
  // --- joint-limit rows (lane: its branch dofs), in registers; base part broadcast ------
  constexpr int NLIMB = [] {
    int c = 0;
    for (int j = 0; j < NDB; j++) c += R::dof_limited[j];
    return c;
  }();
  constexpr int NLB_ = NLIMB > 0 ? NLIMB : 1;
  // every lane needs each branch's m_eff and targets, and its own slice (components kb,
  // kb + 4) of each branch's base part (the sweeps' base dot products are sliced)
  // (and its own branch part, zero in the lanes of the other branches: no owner test in
  // the sweeps)
  // Float64 (OWN): 48 replicated doubles (96 registers) would live through the sweeps; there each
  // lane keeps only its own branch's m_eff / targets / impulses and the owner's impulse change
  // reaches the quad by a DPP broadcast (the same arithmetic on the same values: same results)
  Sc BY[4][NLB_][2], Bm[4][NLB_], Brm[4][NLB_], Btl[4][NLB_], Bth[4][NLB_], Blo[4][NLB_], Bhi[4][NLB_];
  Sc Byb[4][NLB_][NDB];
  Sc Om[NLB_], Orm[NLB_], Otl[NLB_], Oth[NLB_], Olo[NLB_], Ohi[NLB_];
  // the limit rows (float64: built after the contact rows -- see below)
  auto lim_setup = [&]() {
    Sc Lyb[NLB_][NDB], Lm[NLB_], Ltl[NLB_], Lth[NLB_], LyB[NLB_][6];
    static_for<0, NDB>([&](auto j_c) {
      constexpr int j = decltype(j_c)::value;
      if constexpr (R::dof_limited[j]) {
        constexpr int li = [] {
          int c = 0;
          for (int jj = 0; jj < j; jj++) c += R::dof_limited[jj];
          return c;
        }();
        constexpr int gd = T::lg(j);
        Sc y[NDB];
        static_for<0, NDB>([&](auto a_c) {
          constexpr int a = decltype(a_c)::value;
          if constexpr (a < gd || !T::coupled(a, gd)) {
            y[a] = 0.f;
          } else {
            Sc t = a == gd ? 1.f : 0.f;
            static_for<gd, a>([&](auto k_c) {
              constexpr int kk = decltype(k_c)::value;
              if constexpr (T::coupled(a, kk) && T::coupled(kk, gd)) t -= Lbr[a][kk] * y[kk];
            });
            y[a] = t * Ld[a];
          }
        });
        Sc t6[6];
  #pragma unroll
        for (int gg = 0; gg < 6; gg++) {
          Sc c = 0.f;
  #pragma unroll
          for (int b = 0; b < NDB; b++) c += Lgb[gg][b] * y[b];
          t6[gg] = -c;
        }
        fwd6(Lbb, Ldb, t6);
        Sc D2 = 0.f;
  #pragma unroll
        for (int a = 0; a < NDB; a++) { D2 += y[a] * y[a]; }
  #pragma unroll
        for (int gg = 0; gg < 6; gg++) { D2 += t6[gg] * t6[gg]; }
        const Sc meff = D2 > Sc(1e-12) ? fast_rcp(D2) : 0.f;
        const Sc plo = s.q[j] - pk<T::DLO, j>(L), phi = pk<T::DHI, j>(L) - s.q[j];
        Ltl[li] = pos_target(plo, P.k_limit, P.k_sep);
        Lth[li] = pos_target(phi, P.k_limit, P.k_sep);
        Lm[li] = meff;
  #pragma unroll
        for (int a = 0; a < NDB; a++) Lyb[li][a] = y[a];
  #pragma unroll
        for (int gg = 0; gg < 6; gg++) LyB[li][gg] = t6[gg];
      }
    });
    if constexpr (OWN) {
      static_for<0, NLIMB>([&](auto l_c) {
        constexpr int li = decltype(l_c)::value;
        Om[li] = Lm[li];
        Orm[li] = Lm[li] > 0.f ? fast_rcp(Lm[li]) : 0.f;
        Otl[li] = Ltl[li];
        Oth[li] = Lth[li];
        Olo[li] = 0.f;
        Ohi[li] = 0.f;
      });
    }
    static_for<0, 4>([&](auto k_c) {
      constexpr int kk = decltype(k_c)::value;
      static_for<0, NLIMB>([&](auto l_c) {
        constexpr int li = decltype(l_c)::value;
  #pragma unroll
        for (int a = 0; a < NDB; a++) Byb[kk][li][a] = kb == kk ? Lyb[li][a] : 0.f;
        Sc b6[6];
  #pragma unroll
        for (int gg = 0; gg < 6; gg++) b6[gg] = quad_bcast<kk>(LyB[li][gg]);
        BY[kk][li][0] = kb == 0 ? b6[0] : (kb == 1 ? b6[1] : (kb == 2 ? b6[2] : b6[3]));
        BY[kk][li][1] = kb == 0 ? b6[4] : (kb == 1 ? b6[5] : 0.f);
        if constexpr (OWN) return;
        Bm[kk][li] = quad_bcast<kk>(Lm[li]);
        Brm[kk][li] = Bm[kk][li] > 0.f ? fast_rcp(Bm[kk][li]) : 0.f;  // off the sweeps' dependency chain
        Btl[kk][li] = quad_bcast<kk>(Ltl[li]);
        Bth[kk][li] = quad_bcast<kk>(Lth[li]);
        Blo[kk][li] = 0.f;
        Bhi[kk][li] = 0.f;
      });
    });
  };
  if constexpr (!OWN) lim_setup();

  STAMP(3)
  // --- contact rows: base slots (replicated), then each branch's slots (owner lane) ------
  if constexpr (!OWN) {
    n0 = 0;
    base_bits = 0;
    static_for<0, T::NS0>([&](auto sl_c) {
      constexpr int sl = decltype(sl_c)::value;
      const f3 cc = O + mulc(Rb, (Sc)R::slot_point[sl][0], (Sc)R::slot_point[sl][1], (Sc)R::slot_point[sl][2]);
      const Sc rad = (Sc)R::slot_radius[sl];
      const Sc dist = cc.z - rad;
      if (!(dist < (Sc)PBG_CONTACT_THRESHOLD)) return;
      base_bits |= 1u << sl;
      const f3 rP = mk3<Sc>(cc.x, cc.y, cc.z - rad) - O;
  #pragma unroll
      for (int dir = 0; dir < 3; dir++) {
        const f3 nd = dir == 0 ? mk3<Sc>(0, 0, 1) : (dir == 1 ? mk3<Sc>(0, -1, 0) : mk3<Sc>(1, 0, 0));
        const f3 mm = cross3(rP, nd);
        Sc y6[6] = {nd.x, nd.y, nd.z, mm.x, mm.y, mm.z};
        fwd6(Lbb, Ldb, y6);
        Sc D2 = 0.f;
  #pragma unroll
        for (int gg = 0; gg < 6; gg++) { D2 += y6[gg] * y6[gg]; }
        Sc z[NDB];
  #pragma unroll
        for (int a = 0; a < NDB; a++) z[a] = 0.f;
        rw.put(3 * n0 + dir, -1, z, y6, D2 > Sc(1e-12) ? fast_rcp(D2) : 0.f,
               dir == 0 ? (pos_target(dist, P.k_contact, P.k_sep)) : 0.f, (Sc)R::slot_mu[sl]);
      }
      n0++;
    });
    detect_branch();
  } else {  // float64: the detection ran after phase A; the base rows here
    static_for<0, T::NS0>([&](auto sl_c) {
      constexpr int sl = decltype(sl_c)::value;
      if (!((base_bits >> sl) & 1u)) return;
      const f3 cc = O + mulc(Rb, (Sc)R::slot_point[sl][0], (Sc)R::slot_point[sl][1], (Sc)R::slot_point[sl][2]);
      const Sc rad = (Sc)R::slot_radius[sl];
      const Sc dist = cc.z - rad;
      const f3 rP = mk3<Sc>(cc.x, cc.y, cc.z - rad) - O;
      const int r0 = __builtin_popcount(base_bits & ((1u << sl) - 1u));
#pragma unroll
      for (int dir = 0; dir < 3; dir++) {
        const f3 nd = dir == 0 ? mk3<Sc>(0, 0, 1) : (dir == 1 ? mk3<Sc>(0, -1, 0) : mk3<Sc>(1, 0, 0));
        const f3 mm = cross3(rP, nd);
        Sc y6[6] = {nd.x, nd.y, nd.z, mm.x, mm.y, mm.z};
        fwd6(Lbb, Ldb, y6);
        Sc D2 = 0.f;
#pragma unroll
        for (int gg = 0; gg < 6; gg++) { D2 += y6[gg] * y6[gg]; }
        Sc z[NDB];
#pragma unroll
        for (int a = 0; a < NDB; a++) z[a] = 0.f;
        rw.put(3 * r0 + dir, -1, z, y6, D2 > Sc(1e-12) ? fast_rcp(D2) : 0.f,
               dir == 0 ? (pos_target(dist, P.k_contact, P.k_sep)) : 0.f, (Sc)R::slot_mu[sl]);
      }
    });
  }
  static_for<0, T::NSB>([&](auto sl_c) {
    constexpr int sl = decltype(sl_c)::value;
    if (!((act >> sl) & 1u)) return;
    constexpr int li = R::slot_link[T::NS0 + sl];
    const Sc dist = sdist[sl];
    const f3 rP = sP[sl] - O;
#pragma unroll
    for (int dir = 0; dir < 3; dir++) {
      const f3 nd = dir == 0 ? mk3<Sc>(0, 0, 1) : (dir == 1 ? mk3<Sc>(0, -1, 0) : mk3<Sc>(1, 0, 0));
      const f3 mm = cross3(rP, nd);
      Sc y[NDB];
      static_for<0, NDB>([&](auto a_c) {
        constexpr int a = decltype(a_c)::value;
        if constexpr (!T::in_chain(a, li)) {
          y[a] = 0.f;
        } else {
          Sc t = dot3(nd, sv[a]) + dot3(mm, sw[a]);
          static_for<0, a>([&](auto k_c) {
            constexpr int kk = decltype(k_c)::value;
            if constexpr (T::coupled(a, kk) && T::in_chain(kk, li)) t -= Lbr[a][kk] * y[kk];
          });
          y[a] = t * Ld[a];
        }
      });
      Sc y6[6] = {nd.x, nd.y, nd.z, mm.x, mm.y, mm.z};
#pragma unroll
      for (int gg = 0; gg < 6; gg++) {
#pragma unroll
        for (int b = 0; b < NDB; b++) y6[gg] -= Lgb[gg][b] * y[b];
      }
      fwd6(Lbb, Ldb, y6);
      Sc D2 = 0.f;
#pragma unroll
      for (int a = 0; a < NDB; a++) { D2 += y[a] * y[a]; }
#pragma unroll
      for (int gg = 0; gg < 6; gg++) { D2 += y6[gg] * y6[gg]; }
      rw.put(3 * ci + dir, kb, y, y6, D2 > Sc(1e-12) ? fast_rcp(D2) : 0.f,
             dir == 0 ? (pos_target(dist, P.k_contact, P.k_sep)) : 0.f, pk<T::SMU, sl>(L));
    }
    ci++;
  });
  if constexpr (OWN) lim_setup();
  if (3 * nc > rw.cap) {  // rows in the device workspace: same-CU visibility
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  PBG_QUAD_SYNC
  if constexpr (OWN && NLIMB > 0) {
    TRACE64(5, 0, Om[0]); TRACE64(5, 1, Orm[0]); TRACE64(5, 2, Otl[0]); TRACE64(5, 3, Oth[0]);
    TRACE64(5, 4, BY[0][0][0]); TRACE64(5, 5, BY[1][0][1]); TRACE64(5, 6, Byb[0][0][0]); TRACE64(5, 7, Om[NLIMB - 1]);
  }
  // wave-uniform: do all rows of the wave's envs live in LDS?
  const bool all_lds = __builtin_amdgcn_ballot_w64(3 * nc > rw.cap) == 0;

  STAMP(4)
  // --- PGS, 5 sweeps, Bullet order: joint limits (dof order), normals, frictions ------
  // u's base part sliced over the quad: lane kb owns components kb and kb + 4 (kb < 2)
  Sc uBs[2] = {kb == 0 ? uB[0] : (kb == 1 ? uB[1] : (kb == 2 ? uB[2] : uB[3])),
                  kb == 0 ? uB[4] : (kb == 1 ? uB[5] : 0.f)};
  // the limit rows of one sweep (Bullet's order: limits, then the contact normals and frictions)
  auto limit_sweep = [&]() {
    static_for<0, 4>([&](auto k_c) {
      constexpr int kk = decltype(k_c)::value;
      static_for<0, NLIMB>([&](auto l_c) {
        constexpr int li = decltype(l_c)::value;
        Sc part = BY[kk][li][0] * uBs[0] + BY[kk][li][1] * uBs[1];
        static_for<0, NDB>([&](auto a_c) {  // structural zeros of the row skipped
          constexpr int a = decltype(a_c)::value;
          if constexpr (T::lim_nz(li, a)) part += Byb[kk][li][a] * ub[a];
        });
        const Sc yu = quad_sum(part);
        Sc dl;
        if constexpr (OWN) {  // every lane runs its own row li; lane kk's result is the one kept
          const Sc meff = Om[li], llo = Olo[li], lhi = Ohi[li];
          const Sc nlo = clampf(llo + meff * (Otl[li] - yu), 0.f, (Sc)PBG_LIMIT_MAX_IMPULSE);
          const Sc dlo = nlo - llo;
          const Sc yu2 = yu + dlo * Orm[li];
          const Sc nhi = clampf(lhi + meff * (Oth[li] + yu2), 0.f, (Sc)PBG_LIMIT_MAX_IMPULSE);
          const Sc dhi = nhi - lhi;
          if (kb == kk) { Olo[li] = nlo; Ohi[li] = nhi; }
          dl = quad_bcast<kk>(dlo - dhi);
        } else {
          const Sc meff = Bm[kk][li], llo = Blo[kk][li], lhi = Bhi[kk][li];
          const Sc nlo = clampf(llo + meff * (Btl[kk][li] - yu), 0.f, (Sc)PBG_LIMIT_MAX_IMPULSE);
          const Sc dlo = nlo - llo;
          // upper row sees u after the lower update: (-y).u' = -(yu + dlo / meff)
          const Sc yu2 = yu + dlo * Brm[kk][li];  // Brm = 0 when meff = 0
          const Sc nhi = clampf(lhi + meff * (Bth[kk][li] + yu2), 0.f, (Sc)PBG_LIMIT_MAX_IMPULSE);
          const Sc dhi = nhi - lhi;
          Blo[kk][li] = nlo;
          Bhi[kk][li] = nhi;
          dl = dlo - dhi;
        }
        uBs[0] += BY[kk][li][0] * dl;
        uBs[1] += BY[kk][li][1] * dl;
        static_for<0, NDB>([&](auto a_c) {
          constexpr int a = decltype(a_c)::value;
          if constexpr (T::lim_nz(li, a)) ub[a] += Byb[kk][li][a] * dl;
        });
      });
    });
  };
  // one loop per row source: a wave-uniform branch inside the sweep loop made its back edge merge
  // the LDS and workspace paths' register assignments (copies of every loop-carried value)
  if (all_lds) {
    for (int it = 0; it < P.iterations; it++) {
      limit_sweep();
      STAMP(11)
      contact_sweep<true>(rw, nc, kb, ub, uBs SUB_STAMP_PASS);
      STAMP(13)
    }
  } else {
    for (int it = 0; it < P.iterations; it++) {
      limit_sweep();
      STAMP(11)
      contact_sweep<false>(rw, nc, kb, ub, uBs SUB_STAMP_PASS);
      STAMP(13)
    }
  }
  // gather the base part back (replicated for the back-substitution)
  {
    const Sc s0 = uBs[0], s1 = uBs[1];
    uB[0] = quad_bcast<0>(s0); uB[1] = quad_bcast<1>(s0); uB[2] = quad_bcast<2>(s0); uB[3] = quad_bcast<3>(s0);
    uB[4] = quad_bcast<0>(s1); uB[5] = quad_bcast<1>(s1);
  }
  TRACE64(6, 0, uBs[0]); TRACE64(6, 1, uBs[1]); TRACE64(6, 2, ub[0]); TRACE64(6, 3, ub[NDB - 1]);
  TRACE64(6, 4, uB[0]); TRACE64(6, 5, uB[5]); TRACE64(6, 6, nc); TRACE64(6, 7, uB[2]);

  STAMP(5)
  // --- nu = L^-T u (base first, replicated; then the branch); clamp; integrate ---------
  static_for<0, 6>([&](auto r_c) {
    constexpr int gg = 5 - decltype(r_c)::value;
    Sc t = uB[gg];
    static_for<gg + 1, 6>([&](auto h_c) { t -= Lbb[decltype(h_c)::value][gg] * nB[decltype(h_c)::value]; });
    nB[gg] = clampf(t * Ldb[gg], -(Sc)PBG_MAX_COORD_VELOCITY, (Sc)PBG_MAX_COORD_VELOCITY);
  });
  static_for<0, NDB>([&](auto r_c) {
    constexpr int a = NDB - 1 - decltype(r_c)::value;
    Sc t = ub[a];
    static_for<a + 1, NDB>([&](auto k_c) {
      constexpr int kk = decltype(k_c)::value;
      if constexpr (T::coupled(kk, a)) t -= Lbr[kk][a] * nb[kk];
    });
#pragma unroll
    for (int gg = 0; gg < 6; gg++) t -= Lgb[gg][a] * nB[gg];
    nb[a] = t * Ld[a];
  });
  static_for<0, NDB>([&](auto j_c) {
    constexpr int j = decltype(j_c)::value;
    s.qd[j] = clampf(nb[T::lg(j)], -(Sc)PBG_MAX_COORD_VELOCITY, (Sc)PBG_MAX_COORD_VELOCITY);
    s.q[j] += dt * s.qd[j];
  });
#pragma unroll
  for (int i = 0; i < 3; i++) {
    s.bv[i] = nB[i];
    s.bw[i] = nB[3 + i];
    s.bp[i] += dt * s.bv[i];
  }
  {
    const f3 wv = mk3<Sc>(s.bw[0], s.bw[1], s.bw[2]);
    Sc ang = norm3(wv);
    if (ang * dt > (Sc)PBG_ANGULAR_MOTION_THRESHOLD) ang = P.ang_max;
    Sc sh, dw;
    sincos_fast(Sc(0.5f) * ang * dt, &sh, &dw);
    f3 ax;
    if (ang < Sc(0.001)) ax = (Sc(0.5f) * dt - P.dt3c * ang * ang) * wv;
    else ax = (sh / ang) * wv;
    const Sc x = s.bq[0], y = s.bq[1], z = s.bq[2], ww = s.bq[3];
    const Sc nx = dw * x + ax.x * ww + ax.y * z - ax.z * y;
    const Sc ny = dw * y - ax.x * z + ax.y * ww + ax.z * x;
    const Sc nz = dw * z + ax.x * y - ax.y * x + ax.z * ww;
    const Sc nw = dw * ww - ax.x * x - ax.y * y - ax.z * z;
    const Sc inv = fast_rsq(nx * nx + ny * ny + nz * nz + nw * nw);
    s.bq[0] = nx * inv; s.bq[1] = ny * inv; s.bq[2] = nz * inv; s.bq[3] = nw * inv;
  }
  TRACE64(7, 0, nB[0]); TRACE64(7, 1, nB[3]); TRACE64(7, 2, nb[0]); TRACE64(7, 3, nb[NDB - 1]);
  TRACE64(7, 4, s.qd[0]); TRACE64(7, 5, s.bv[2]); TRACE64(7, 6, s.bw[0]); TRACE64(7, 7, s.bq[3]);
  STAMP(6)
  return nc;
}

// ------------------------------------------------------------------ calc_state (pack)
// Part COMs and joint states of all branches meet in the env's LDS staging area; every
// lane of the quad then runs the (numpy-exact, float64) pack on identical inputs.
template <class R, int ES>
PBG_DEV void team_gather(const TState<R>& s, const Lane& L, const TRows<R, ES>& rw, bool has_floor, PackIn<R>& in) {
  using T = Team<R>;
  using Sc = real_t<R>;
  using f3 = V3<Sc>;
  using m3 = M3<Sc>;
  constexpr int NL = R::NL, NJ = R::NJ, NDB = T::NDB, NLB = T::NLB;
  const m3 Rb = quat_to_m3(s.bq[0], s.bq[1], s.bq[2], s.bq[3]);
  TKin<R> k;
  team_fk<R>(s, L, Rb, k);
  PBG_QUAD_SYNC  // staging may still be read by the previous pack
#pragma unroll
  for (int i = 0; i < NLB; i++) {
    rw.stage(L.k * NLB + i) = k.c[i].x;
    rw.stage(NL + L.k * NLB + i) = k.c[i].y;
  }
#pragma unroll
  for (int j = 0; j < NDB; j++) {
    rw.stage(2 * NL + L.k * NDB + j) = s.q[j];
    rw.stage(2 * NL + NJ + L.k * NDB + j) = s.qd[j];
  }
  PBG_QUAD_SYNC
  int np = 0;
#pragma unroll
  for (int p = 0; p < R::NP; p++) {
    const int l = R::part_link[p];
    in.part_x[np] = l < 0 ? (double)s.bp[0] : (double)rw.stage(l);
    in.part_y[np] = l < 0 ? (double)s.bp[1] : (double)rw.stage(NL + l);
    np++;
  }
  if (R::floor && has_floor) { in.part_x[np] = 0.0; in.part_y[np] = 0.0; np++; }
  in.n_parts = np;
#pragma unroll
  for (int i = 0; i < 4; i++) in.quat[i] = s.bq[i];
#pragma unroll
  for (int i = 0; i < 3; i++) { in.pos[i] = s.bp[i]; in.vel[i] = s.bv[i]; in.avel[i] = s.bw[i]; }
#pragma unroll
  for (int i = 0; i < R::NO; i++) {
    in.jq[i] = rw.stage(2 * NL + R::obs_dof[i]);
    in.jqd[i] = rw.stage(2 * NL + NJ + R::obs_dof[i]);
  }
}

// snapshot + Philox reset noise (pbg_step.hip reset_env); returns the reset pack
template <class R, int ES>
PBG_DEV void team_reset(const Buffers& B, int e, const Lane& L, TState<R>& s, const TRows<R, ES>& rw, float* obs,
                        bool& has_floor, double& pot, real_t<R>& z0) {
  using T = Team<R>;
  using Sc = real_t<R>;
#pragma unroll
  for (int i = 0; i < 3; i++) s.bp[i] = (Sc)R::base_pos[i];
#pragma unroll
  for (int i = 0; i < 4; i++) s.bq[i] = (Sc)R::base_quat[i];
#pragma unroll
  for (int i = 0; i < 3; i++) { s.bv[i] = 0.f; s.bw[i] = 0.f; }
  const uint32_t epi = B.episode[e];
  const uint32_t gid = (uint32_t)(B.env_offset + e);
  float noise[R::NR > 0 ? R::NR : 1];
#pragma unroll
  for (int blk = 0; blk < (R::NR + 3) / 4; blk++) {
    u4 ctr = {gid, epi, (uint32_t)blk, 0x5EEDu};
    const u4 rnd = philox4x32_10(ctr, (uint32_t)B.seed, (uint32_t)(B.seed >> 32));
    const uint32_t rr[4] = {rnd.x, rnd.y, rnd.z, rnd.w};
#pragma unroll
    for (int t = 0; t < 4; t++)
      if (4 * blk + t < R::NR) noise[4 * blk + t] = fmaf(0.2f, u01(rr[t]), -0.1f);
  }
  static_for<0, T::NDB>([&](auto j_c) {
    constexpr int j = decltype(j_c)::value;
    const int r = pki<T::RST, j>(L);
    Sc q = 0.f;
#pragma unroll
    for (int t = 0; t < R::NR; t++) q = r == t ? noise[t] : q;
    s.q[j] = q;
    s.qd[j] = 0.f;
  });
  PackIn<R> in;
  in.env_dt = sp_of<R>(B).env_dt;
  team_gather<R, ES>(s, L, rw, has_floor, in);
#pragma unroll
  for (int f = 0; f < R::NF; f++) in.feet_prev[f] = 0.f;
  in.feet_new = 0;
  in.potential_old = 0.0;
  in.initial_z = R::initial_z_fixed;
  PackOut po;
  if constexpr (R::kind == 3) mujoco3d_pack<R>(in, nullptr, obs, po);
  else walker_pack<R>(in, nullptr, obs, po);
  pot = po.potential;
  z0 = (Sc)po.initial_z;
  has_floor = true;
  if (L.k == 0) B.episode[e] = epi + 1;
}

template <class R, int ES>
__global__ __launch_bounds__(64) void team_step_kernel(Buffers B, StepIO io, float* __restrict__ scratch, int lds_rows) {
  using T = Team<R>;
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  constexpr int NDB = T::NDB, SB = PBG_BASE_WORDS;
  extern __shared__ float lds_dyn[];
  const int tid = xcd_block() * blockDim.x + threadIdx.x;
  const int e = tid >> 2;
  if (e >= B.n) return;
  const Lane L = make_lane(tid & 3);
  const int kb = L.k;
  STAMP_DECL
  TState<R> s;
#pragma unroll
  for (int i = 0; i < 3; i++) s.bp[i] = st_of<R>(B)[(size_t)i * B.n + e];
#pragma unroll
  for (int i = 0; i < 4; i++) s.bq[i] = st_of<R>(B)[(size_t)(3 + i) * B.n + e];
#pragma unroll
  for (int i = 0; i < 3; i++) s.bv[i] = st_of<R>(B)[(size_t)(7 + i) * B.n + e];
#pragma unroll
  for (int i = 0; i < 3; i++) s.bw[i] = st_of<R>(B)[(size_t)(10 + i) * B.n + e];
#pragma unroll
  for (int j = 0; j < NDB; j++) {
    s.q[j] = st_of<R>(B)[(size_t)(SB + kb * NDB + j) * B.n + e];
    s.qd[j] = st_of<R>(B)[(size_t)(SB + R::NJ + kb * NDB + j) * B.n + e];
  }
  // the pack's bookkeeping loads: float32 issues them here so their latency overlaps the physics;
  // float64 after the physics, and it re-reads the actions there too (the registers those values would
  // hold through the sub-steps are the ones its physics spills for)
  constexpr bool LATE = sizeof(Sc) == 8;
  int el = 0;
  uint32_t flags = 0;
  double pot_old = 0.0;
  Sc z0_old = 0.f;
  auto book = [&]() {
    el = B.elapsed[e] + 1;
    flags = B.flags[e];
    pot_old = B.pot[e];
    z0_old = z0_of<R>(B)[e];
  };
  if constexpr (!LATE) book();
  float act[R::NA];
#pragma unroll
  for (int i = 0; i < R::NA; i++) act[i] = io.act[(size_t)e * R::NA + i];
  // apply_action (robot_locomotors.py:26-29): this branch's motors
  Sc tau[NDB];
  static_for<0, NDB>([&](auto j_c) {
    constexpr int j = decltype(j_c)::value;
    const int ai = pki<T::ACTI, j>(L);
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < R::NA; i++) a = ai == i ? act[i] : a;
    tau[j] = ai < 0 ? 0.f : (Sc)((double)pk<T::GAIN, j>(L) * (double)fminf(fmaxf(a, -1.f), 1.f));
  });
  TRows<R, ES> rw;
  rw.lds = (LW*)lds_dyn + (threadIdx.x >> 2);
  rw.rows = (LW*)lds_dyn + TRows<R, ES>::HEAD * ES;
  rw.lane = threadIdx.x;
  rw.gbl = (Sc*)scratch + e;
  rw.n = B.n;
  rw.cap = lds_rows;
  uint32_t slot_bits = 0, base_bits = 0;
  int nc = 0;
  STAMP(7)
  uint32_t csig = 0;  // this lane's share of the contact-set signature
  for (int sub = 0; sub < sp_of<R>(B).substeps; sub++) {
    nc = team_substep<R, ES>(s, L, tau, slot_bits, base_bits, rw, sp_of<R>(B) SUB_STAMP_PASS);
    if (io.csig) {  // base slots counted by lane 0, branch k's slots (global NS0 + k NSB + sl) by lane k
      if (kb == 0)
        for (int sl = 0; sl < T::NS0; sl++)
          if ((base_bits >> sl) & 1u) csig += pbg_contact_hash((uint32_t)sub, (uint32_t)sl);
      for (int sl = 0; sl < T::NSB; sl++)
        if ((slot_bits >> sl) & 1u) csig += pbg_contact_hash((uint32_t)sub, (uint32_t)(T::NS0 + kb * T::NSB + sl));
    }
  }
  if (io.ncontact && kb == 0) io.ncontact[e] = nc;
  if (io.csig) {
    uint32_t sig = csig;  // quad sum mod 2^32
    sig += (uint32_t)qperm_i<0xB1>((int)sig);
    sig += (uint32_t)qperm_i<0x4E>((int)sig);
    if (kb == 0) io.csig[e] = sig;
  }
  if constexpr (LATE) {
    book();
    const float* ap = io.act;
    asm volatile("" : "+s"(ap));  // a fresh pointer: the loads are not merged with the ones above
#pragma unroll
    for (int i = 0; i < R::NA; i++) act[i] = ap[(size_t)e * R::NA + i];
  }
  // feet contact flags of the last sub-step: this branch's feet, OR-ed over the quad
  uint32_t fb = 0;
  static_for<0, T::NSB>([&](auto sl_c) {
    constexpr int sl = decltype(sl_c)::value;
    constexpr int li = R::slot_link[T::NS0 + sl];
    const int f = pki<T::FOOT, li>(L);
    if (f >= 0 && ((slot_bits >> sl) & 1u)) fb |= 1u << f;
  });
  const uint32_t fnew = (uint32_t)quad_sum_i((int)fb);  // disjoint bits: sum == or
  float obs[R::OBS];
  PackOut po;
  {
    PackIn<R> in;
    in.env_dt = sp_of<R>(B).env_dt;
    team_gather<R, ES>(s, L, rw, flags & 1u, in);
#pragma unroll
    for (int f = 0; f < R::NF; f++) in.feet_prev[f] = ((flags >> (8 + f)) & 1u) ? 1.f : 0.f;
    in.feet_new = fnew;
    in.potential_old = pot_old;
    in.initial_z = z0_old;
    if constexpr (R::kind == 3) mujoco3d_pack<R>(in, act, obs, po);
    else walker_pack<R, false, 4>(in, act, obs, po, kb);
    flags = (flags & 0xFFu) | (po.feet_out << 8);
  }
  STAMP(8)
  // float64: the env index through an empty asm, so the stores below form their addresses here
  // instead of reloading the 64-bit addresses the compiler formed at the kernel's start and spilled
  // (each such scratch reload waited, vmcnt(0), for every store issued before it: 29 % of the
  // float64 kernel's cycles went to this phase, 8 % in float32)
  int eo = e;
  if constexpr (sizeof(Sc) == 8) asm volatile("" : "+v"(eo));
  const bool term = po.done;
  const bool trunc = el >= R::max_episode_steps;
  if (kb == 0) {
    io.rew[eo] = (float)po.reward;
    if (io.rew64) io.rew64[eo] = po.reward;
    if (io.rew_terms) {
#pragma unroll
      for (int i = 0; i < 5; i++) io.rew_terms[(size_t)eo * 5 + i] = po.terms[i];
    }
    io.done[eo] = term || trunc;
    if (io.trunc) io.trunc[eo] = trunc && !term;
  }
  if (io.autoreset && (term || trunc)) {
    if (io.term_obs) lanes_store_row<R, 4>(obs, io.term_obs, eo, kb);
    bool has_floor = flags & 1u;
    double pot;
    Sc z0;
    team_reset<R, ES>(B, eo, L, s, rw, obs, has_floor, pot, z0);
    if (kb == 0) {
      B.pot[eo] = pot;
      z0_of<R>(B)[eo] = z0;
      B.elapsed[eo] = 0;
      B.flags[eo] = has_floor ? 1u : 0u;
    }
  } else if (kb == 0) {
    B.pot[eo] = po.potential;
    B.elapsed[eo] = el;
    B.flags[eo] = flags;
  }
  {
    // replicated base words and obs dealt over the quad (lane kb: elements kb, kb+4, ...)
    const Sc bw[PBG_BASE_WORDS] = {s.bp[0], s.bp[1], s.bp[2], s.bq[0], s.bq[1], s.bq[2], s.bq[3],
                                      s.bv[0], s.bv[1], s.bv[2], s.bw[0], s.bw[1], s.bw[2]};
    static_for<0, (PBG_BASE_WORDS + 3) / 4>([&](auto m_c) {
      constexpr int m = decltype(m_c)::value;
      const Sc v = lanes_pick<4, m, PBG_BASE_WORDS>(bw, kb);
      if (4 * m + kb < PBG_BASE_WORDS) st_of<R>(B)[(size_t)(4 * m + kb) * B.n + eo] = v;
    });
    lanes_store_row<R, 4>(obs, io.obs, eo, kb);
  }
#pragma unroll
  for (int j = 0; j < NDB; j++) {
    st_of<R>(B)[(size_t)(SB + kb * NDB + j) * B.n + eo] = s.q[j];
    st_of<R>(B)[(size_t)(SB + R::NJ + kb * NDB + j) * B.n + eo] = s.qd[j];
  }
  STAMP(9)
  STAMP_FLUSH
}

}  // namespace pbg
