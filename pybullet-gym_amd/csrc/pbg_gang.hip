// pbg_gang.hip -- gang-per-env step kernel: T = 16 lanes (one DPP row) per env, four
// envs per wave.  Included by pbg_robot.hip after pbg_step.hip / pbg_team.hip; selected
// by plan_* for the robots without a quad decomposition (Humanoid, Hopper, HalfCheetah,
// Walker2D) when the env count leaves SIMDs idle in the lane kernel.
//
// Same physics, Bullet row order and numpy-exact pack as step_kernel (pbg_step.hip).
// What changes is who does the work:
//  * replicated -- every lane of the gang runs the unconstrained dynamics (dynamics():
//    composites, mass matrix, Cholesky, u = L^T nu), integration and the pack on identical
//    inputs, so the results are bitwise identical across the gang;
//  * distributed -- collision candidates (floor slots, self-collision pairs), constraint
//    rows (joint limits + 3 rows per contact: y = L^-1 J^T, m_eff, target) and the PGS
//    vector work.  Candidates and rows are dealt round-robin to the lanes and run through
//    ONE generic code path (runtime link / slot / pair index, model constants from a
//    __constant__ table) instead of the lane kernel's fully unrolled per-slot code: the
//    whole contact phase is a few hundred instructions per lane instead of tens of
//    thousands, and the contact count per lane is nc / 16.
//  * PGS keeps Bullet's sequential row order; the generalized velocity in Cholesky space
//    u is sliced over the gang (lane t owns u[t], u[t+16], ...), each row is a slice dot
//    product + a 16-lane DPP all-reduce (quad_perm, row_half_mirror, row_mirror: the same
//    bits in every lane) + a replicated impulse update.
// Contacts are compacted in candidate order with a wave ballot (rank = popcount of the
// gang's lower lanes), which reproduces the lane kernel's contact order: floor slots in
// slot order, then pairs in pair order.
//
// Why: at the BASELINE env counts (Humanoid 4,096 / GPU, Hopper and Walker2D 4,096,
// HalfCheetah 8,192) the lane kernel runs 64-256 waves of 16-32 active lanes -- one SIMD
// in four busy, three lanes in four idle, every instruction's latency exposed.  The gang
// kernel runs n/4 full waves (1,024 at 4,096 envs: one per SIMD).
//
// Per-env LDS region (words), [gang-shared]:
//   L (NNZ) | Ld (N) | u (YS) | rhs (N) | s_w | s_v (6N, interleaved per index) | q | qd | tau (NJ
//   each) | joint axis | origin (6 NJ, interleaved) | base state (13, front path) | cube state (13,
//   FlagrunHarder) | body frames (12 NB) | limit pos (2 NLIM) | limit rows NLIM x (YS + 5) or the
//   composites (16 NB) | contacts 0..cap-1 x PERC (kinematic parts, 16 NB, at the contacts' start
//   until M is built).  Records start on 16-byte boundaries (Gang<R, T>::AL).
// contact c: descriptor (DW) | mu | 3 rows x (y (YS) | m_eff | target | lambda); a row's y is
// lane-major (lane t's NSL words y[t], y[t + T], ... contiguous: one ds_read_b64 for
// Humanoid's two); contacts at c >= cap live at the same offsets in the env's device
// workspace.  (Pairing m_eff | target and lambda | mu for b64 loads needs an even row length:
// one word more per contact, which costs HalfCheetah at 8,192 envs one LDS-resident contact.)
#ifdef PBG_DEV_CHECKS
#include <cassert>
#endif
#include "pbg_fronts.h"

namespace pbg {

#define PBG_GANG_BLOCK 256  // lanes per gang workgroup (4 waves)
// Atlas (886 floor-contact candidates, 36 dofs): a two-wave workgroup of 8 envs -- the model
// tables (32 KB) and 8 env regions (13.8 KB each) fill 142 KB of the CU's 160 KB; 16 envs would
// not fit, and one-wave workgroups (87 KB: one per CU) left three SIMDs of each CU idle
// (4.72 -> 3.05 ms per step at 4,096 envs, A/B)
template <class R, int T = 16>
constexpr int gang_block();  // (after the layout: the float64 regions decide it)

// bound_ctrl set: every permutation used here reads a valid lane, and with it the
// compiler folds `x + mov_dpp(x)` into one v_add_f32_dpp (no mov, no DPP hazard nop).
template <int CTRL>
PBG_DEV float dpp_f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
// float64: the two dwords moved by the same permutation
template <int CTRL>
PBG_DEV double dpp_f(double x) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// gfx950 v_permlane16_swap_b32 a, b: the odd rows of a trade places with the even rows of b.
// With a = b = x (x uniform within each row) a ends up holding the even row's value and b the odd
// row's, in both rows of each pair.  Inline asm because this ROCm's builtin
// (__builtin_amdgcn_permlane16_swap) returns the first register for both of its results.  The
// compiler's hazard recognizer cannot see inside the asm, so the s_nop 3 (4 wait states) covers
// both hazards a preceding VALU instruction can leave for a permlane: a VALU write of an operand
// register, and a VALU write of EXEC (v_cmpx) -- the latter needs 4 wait states on gfx950.
// gang_sum<32> is only called from the 32-lane kernel's row reductions, all reached with the
// gang's full EXEC mask (wave-uniform control flow).
PBG_DEV void row_pair_swap(float& a, float& b) {
  asm volatile("s_nop 3\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
PBG_DEV void row_pair_swap_u(uint32_t& a, uint32_t& b) {
  asm volatile("s_nop 3\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
PBG_DEV void row_pair_swap(double& a, double& b) {  // the two dwords of each
  uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
  uint32_t al = (uint32_t)ua, ah = (uint32_t)(ua >> 32), bl = (uint32_t)ub, bh = (uint32_t)(ub >> 32);
  row_pair_swap_u(al, bl);
  row_pair_swap_u(ah, bh);
  a = __builtin_bit_cast(double, ((uint64_t)ah << 32) | al);
  b = __builtin_bit_cast(double, ((uint64_t)bh << 32) | bl);
}
// all-reduce over the T (4, 8, 16 or 32) lanes of a DPP row segment (T = 32: a row pair);
// identical bits in every lane (each step adds a value and its mirror image: a + b == b + a;
// the row-pair step adds the even row's sum to the odd row's in that order in both rows)
template <int T, class V>
PBG_DEV V gang_sum(V x) {
  x = x + dpp_f<0xB1>(x);  // quad_perm [1,0,3,2]
  x = x + dpp_f<0x4E>(x);  // quad_perm [2,3,0,1]
  if constexpr (T >= 8) x = x + dpp_f<0x141>(x);   // row_half_mirror
  if constexpr (T >= 16) x = x + dpp_f<0x140>(x);  // row_mirror
  if constexpr (T >= 32) {
    V a = x, b = x;
    row_pair_swap(a, b);  // a: the even row's value, b: the odd row's, in both rows of the pair
    x = a + b;
  }
  return x;
}
PBG_DEV bool wave_any(bool p) { return __ballot(p) != 0ull; }
// a 32-bit chain mask stored in a word of the contact descriptor (its bits, not a number)
template <class S>
PBG_DEV S mask_word(uint32_t m) {
  if constexpr (sizeof(S) == 8) return __builtin_bit_cast(S, (uint64_t)m);
  else return __builtin_bit_cast(S, m);
}
PBG_DEV uint32_t word_mask(float w) { return __builtin_bit_cast(uint32_t, w); }
PBG_DEV uint32_t word_mask(double w) { return (uint32_t)__builtin_bit_cast(uint64_t, w); }
template <int CTRL>
PBG_DEV uint32_t dpp_u(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, true);
}
// integer sum over the T lanes of a DPP row segment (mod 2^32), same in every lane
template <int T>
PBG_DEV uint32_t gang_sum_u32(uint32_t x) {
  x += dpp_u<0xB1>(x);
  x += dpp_u<0x4E>(x);
  if constexpr (T >= 8) x += dpp_u<0x141>(x);
  if constexpr (T >= 16) x += dpp_u<0x140>(x);
  if constexpr (T >= 32) {
    uint32_t a = x, b = x;
    row_pair_swap_u(a, b);
    x = a + b;
  }
  return x;
}
// 32-lane gangs (two envs per wave): for the robots whose factorisation is front-parallel and
// whose per-lane registers then fit two waves per SIMD (Humanoid family).  The 16-lane kernel
// stays for the others, and for these under pbg_create_debug(gang_lanes = 16).
template <class R>
constexpr bool gang32_ok() { return FP<R>::NF > 0 && R::NDOF >= 20 && R::NS <= 128; }
// waves per SIMD the kernel's register budget is compiled for (__launch_bounds__): float32 32-lane
// gangs exist to put two waves on a SIMD; float64 ones (the Humanoid family) to put a wave on each
// of the four SIMDs of a CU whose LDS holds only 8 float64 envs
template <class R, int T>
constexpr int gang_waves_per_simd() { return T >= 32 && sizeof(real_t<R>) == 4 ? 2 : 1; }

// ------------------------------------------------------------------ constant tables
template <class R>
struct GangTab {
  using Sc = real_t<R>;
  static constexpr int NS1 = R::NS > 0 ? R::NS : 1, NP1 = R::NPAIR > 0 ? R::NPAIR : 1;
  static constexpr int NG1 = R::NG > 0 ? R::NG : 1, NB = R::NL + 1;
  static constexpr int NL1 = Dims<R>::NLIM > 0 ? Dims<R>::NLIM : 1;
  Sc gp0[NG1][4];   // capsule end 0 | radius
  Sc gp1[NG1][4];   // capsule end 1
  int geom_body[NG1];
  int pga[NP1], pgb[NP1];
  Sc pmu[NP1], pbound2[NP1];
  uint32_t chain[NB];  // joint dofs moving body b (0: the base)
  int lim_g[NL1];      // generalized index of limit row li
  // floor slots last: robots with many (Atlas) keep them out of the workgroup's LDS copy
  Sc slot[NS1][4];  // point (link frame) | radius
  Sc slot_mu[NS1];
  int slot_body[NS1];
};
// The gang kernel records floor contact for the first 64 slots only (the slot pass's 64-bit
// mask, the feet test of the pack): every foot slot must be among them (codegen.py puts the
// feet's slots first when a robot has more than 64)
template <class R>
constexpr bool feet_slots_below_64() {
  for (int sl = 64; sl < R::NS; sl++)
    for (int f = 0; f < R::NF; f++)
      if (R::slot_link[sl] == R::foot_link[f]) return false;
  return true;
}
// Atlas-sized models (more than 128 floor slots): the slot table is read from the __constant__
// table (L1 / L2-resident, 21 KB) and the joint-limit rows live in the device workspace, so that
// 16 envs' LDS regions fit a 4-wave workgroup
template <class R>
constexpr bool gang_big() { return R::NS > 128; }
template <class R>
constexpr GangTab<R> make_gang_tab() {
  using D = Dims<R>;
  GangTab<R> t{};
  for (int s = 0; s < R::NS; s++) {
    for (int c = 0; c < 3; c++) t.slot[s][c] = (real_t<R>)R::slot_point[s][c];
    t.slot[s][3] = (real_t<R>)R::slot_radius[s];
    t.slot_mu[s] = (real_t<R>)R::slot_mu[s];
    t.slot_body[s] = R::slot_link[s] + 1;
  }
  for (int g = 0; g < R::NG; g++) {
    for (int c = 0; c < 3; c++) { t.gp0[g][c] = (real_t<R>)R::geom_p0[g][c]; t.gp1[g][c] = (real_t<R>)R::geom_p1[g][c]; }
    t.gp0[g][3] = (real_t<R>)R::geom_r[g];
    t.geom_body[g] = R::geom_link[g] + 1;
  }
  for (int p = 0; p < R::NPAIR; p++) {
    t.pga[p] = R::pair_ga[p];
    t.pgb[p] = R::pair_gb[p];
    t.pmu[p] = (real_t<R>)R::pair_mu[p];
    t.pbound2[p] = D::PAIR_BOUND2.v[p][0];
  }
  t.chain[0] = 0;
  for (int l = 0; l < R::NL; l++) t.chain[l + 1] = R::link_chain_mask[l];
  for (int li = 0; li < D::NLIM; li++) t.lim_g[li] = D::gj(D::LIM.v[li][0]);
  return t;
}
template <class R>
__constant__ GangTab<R> g_gang_tab = make_gang_tab<R>();

// body tree for the distributed dynamics: body 0 = base, body l+1 = link l
template <class R>
struct GangDynTab {
  using Sc = real_t<R>;
  static constexpr int NB = R::NL + 1, N = R::NDOF, NNZ = Dims<R>::NNZ, NJ1 = R::NJ > 0 ? R::NJ : 1;
  int parent[NB], jt[NB], dof[NB];
  int lev_start[NB + 2], lev_body[NB];  // bodies grouped by depth
  int child_start[NB + 1], child[NB];
  Sc ro[NB][9], opos[NB][3], axis[NB][3], anchor[NB][3], com[NB][3], mass[NB], inertia[NB][6];
  int me_i[NNZ], me_k[NNZ], me_b[NNZ];  // packed lower-triangle entries of M: rows, cols, composite
  Sc me_arm[NNZ];                     // armature on joint diagonals
  int g_body[N], g_dof[N];               // composite owning generalized index i; its joint dof (-1: base)
  Sc damping[NJ1], stiffness[NJ1];
};
template <class R>
constexpr int body_depth(int b) {
  int d = 0;
  while (b > 0) { b = R::link_parent[b - 1] + 1; d++; }
  return d;
}
template <class R>
constexpr int gang_nlev() {
  int m = 0;
  for (int b = 0; b <= R::NL; b++) m = body_depth<R>(b) > m ? body_depth<R>(b) : m;
  return m + 1;
}
template <class R>
constexpr GangDynTab<R> make_gang_dyn_tab() {
  using D = Dims<R>;
  GangDynTab<R> t{};
  constexpr int NB = R::NL + 1;
  for (int b = 0; b < NB; b++) {
    t.parent[b] = b == 0 ? -1 : R::link_parent[b - 1] + 1;
    t.jt[b] = b == 0 ? 4 : R::link_jtype[b - 1];
    t.dof[b] = b == 0 ? -1 : R::link_dof[b - 1];
    t.mass[b] = (real_t<R>)D::body_mass(b);
    for (int i = 0; i < 6; i++) t.inertia[b][i] = (real_t<R>)(b == 0 ? R::base_inertia[i] : R::link_inertia[b - 1][i]);
    if (b > 0) {
      const int l = b - 1;
      const double x = R::link_offset_quat[l][0], y = R::link_offset_quat[l][1], z = R::link_offset_quat[l][2], w = R::link_offset_quat[l][3];
      const double m[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                           2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                           2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)};
      for (int i = 0; i < 9; i++) t.ro[b][i] = (real_t<R>)m[i];
      for (int c = 0; c < 3; c++) {
        t.opos[b][c] = (real_t<R>)R::link_offset_pos[l][c];
        t.axis[b][c] = (real_t<R>)R::link_axis[l][c];
        t.anchor[b][c] = (real_t<R>)R::link_anchor[l][c];
        t.com[b][c] = (real_t<R>)R::link_com[l][c];
      }
    }
  }
  constexpr int NLEV = gang_nlev<R>();
  int k = 0;
  for (int lv = 0; lv < NLEV; lv++) {
    t.lev_start[lv] = k;
    for (int b = 0; b < NB; b++)
      if (body_depth<R>(b) == lv) t.lev_body[k++] = b;
  }
  for (int lv = NLEV; lv < NB + 2; lv++) t.lev_start[lv] = k;
  k = 0;
  for (int b = 0; b < NB; b++) {
    t.child_start[b] = k;
    for (int c = 1; c < NB; c++)
      if (R::link_parent[c - 1] + 1 == b) t.child[k++] = c;
  }
  t.child_start[NB] = k;
  // packed entries of M in the factor's word order (pbg_fronts.h: front-major, or the plain
  // lower triangle for robots without a front decomposition)
  for (int a = 0; a < R::NDOF; a++)
    for (int b = 0; b <= a; b++)
      if (D::coupled(a, b)) {
        const int e = FP<R>::idx(a, b);
        const int dk = D::dof_of(b), da = D::dof_of(a);
        t.me_i[e] = a;
        t.me_k[e] = b;
        t.me_b[e] = dk >= 0 ? R::dof_link[dk] + 1 : 0;
        t.me_arm[e] = (a == b && da >= 0) ? (real_t<R>)R::dof_armature[da] : 0.f;
      }
  for (int i = 0; i < R::NDOF; i++) {
    const int di = D::dof_of(i);
    t.g_dof[i] = di;
    t.g_body[i] = di >= 0 ? R::dof_link[di] + 1 : 0;
  }
  for (int d = 0; d < R::NJ; d++) {
    t.damping[d] = (real_t<R>)R::dof_damping[d];
    t.stiffness[d] = (real_t<R>)R::dof_stiffness[d];
  }
  return t;
}
template <class R>
__constant__ GangDynTab<R> g_gang_dyn = make_gang_dyn_tab<R>();
// the same table as a compile-time value (level-round code indexes it with constant bodies)
template <class R>
struct GangDT {
  static constexpr GangDynTab<R> v = make_gang_dyn_tab<R>();
};

// Per-lane selection of compile-time constants.  In a round of a level the lanes t < KN own
// the compile-time bodies Src::at(t).  ksel(t, fn) is fn(body) for this lane's body -- a
// select chain over KN compile-time constants, or the constant itself when every body of the
// round agrees (then kmul / mulc fold it: an identity offset rotation, a zero anchor or a
// shared joint axis costs nothing).  fn gets the body as std::integral_constant.
template <class Src, int KN, class V, class F>
PBG_DEV V ksel(int t, F&& fn) {
  V v = (V)fn(std::integral_constant<int, Src::at(KN - 1)>{});
  static_for<0, KN - 1>([&](auto i_c) {
    constexpr int k = KN - 2 - decltype(i_c)::value;
    const V a = (V)fn(std::integral_constant<int, Src::at(k)>{});
    v = t == k ? a : v;
  });
  return v;
}
// bodies of the tree level starting at lev_body[K0]
template <class R, int K0>
struct LevSrc {
  static constexpr int at(int k) { return GangDT<R>::v.lev_body[K0 + k]; }
};
template <class R, int K0, int KN, class F>
PBG_DEV real_t<R> lvsel(int t, F&& fn) { return ksel<LevSrc<R, K0>, KN, real_t<R>>(t, fn); }
template <class R, int K0, int KN, class F>
PBG_DEV int lvsel_i(int t, F&& fn) { return ksel<LevSrc<R, K0>, KN, int>(t, fn); }
// opaque copy of the lane index: the lane compares of the selects stay where they are used
// (hoisted out of the sub-step loop, their masks pinned SGPRs for the whole kernel and spilled)
PBG_DEV int opaque_lane(int t) {
  asm volatile("" : "+v"(t));
  return t;
}

// composites pass: per level, the bodies that have children (a leaf's composite is its own)
template <class R>
struct GangComp {
  static constexpr int NB = R::NL + 1;
  struct Tab {
    int cnt[NB + 1];
    int body[NB + 1][NB];
    int nch[NB];
    int ch[NB][NB];
  };
  static constexpr Tab make() {
    Tab t{};
    for (int b = 0; b < NB; b++) {
      for (int c = 1; c < NB; c++)
        if (R::link_parent[c - 1] + 1 == b) t.ch[b][t.nch[b]++] = c;
      if (t.nch[b] > 0) {
        const int lv = body_depth<R>(b);
        t.body[lv][t.cnt[lv]++] = b;
      }
    }
    return t;
  }
  static constexpr Tab v = make();
  static constexpr int maxch(int lv, int k0, int kn) {
    int m = 0;
    for (int k = 0; k < kn; k++) m = v.nch[v.body[lv][k0 + k]] > m ? v.nch[v.body[lv][k0 + k]] : m;
    return m;
  }
};
template <class R, int LV, int K0>
struct CompSrc {
  static constexpr int at(int k) { return GangComp<R>::v.body[LV][K0 + k]; }
};

// joint type shared by the round's bodies, or -1 when they differ
template <class R>
constexpr int lv_jt(int k0, int kn) {
  const int j = GangDT<R>::v.jt[GangDT<R>::v.lev_body[k0]];
  for (int k = 1; k < kn; k++)
    if (GangDT<R>::v.jt[GangDT<R>::v.lev_body[k0 + k]] != j) return -1;
  return j;
}
// A * B where B's entries may be compile-time constants (its zeros fold away)
template <class S>
PBG_DEV M3<S> mul_kb(const M3<S>& A, const M3<S>& B) {
  M3<S> C;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
      C.m[3 * i + j] = kmul(B.m[j], A.m[3 * i]) + kmul(B.m[3 + j], A.m[3 * i + 1]) + kmul(B.m[6 + j], A.m[3 * i + 2]);
  return C;
}

// ------------------------------------------------------------------ layout
template <class R, int T>
struct Gang {
  using D = Dims<R>;
  static constexpr int N = R::NDOF, NNZ = D::NNZ, NB = D::NB, NLIM = D::NLIM;
  static constexpr int NY = D::NY;             // row length: the robot's dofs (+ the cube's 6)
  static constexpr int NSL = (NY + T - 1) / T;  // u entries per lane
  static constexpr int YS = NSL * T;           // padded row length
  static constexpr int MAXC = D::NC;  // floor slots, self pairs (+ the cube's corners and robot geoms)
  static constexpr int DW = 16;                // descriptor: rA 3 | rB 3 | n 3 | dist | fA | fB | mA | mB | floor | pad
  // rows of NSL = 2 robots (Humanoid) are laid out for one ds_read_b64 of a lane's y pair:
  // an even row length, the first row at an even LDS word (the env region, FIXED and the
  // record length are even)
  static constexpr bool Y64 = NSL == 2;
  static constexpr int CRW = YS + 3 + (Y64 ? 1 : 0);  // y (lane-major) | m_eff | target | lambda [| pad]
  static constexpr int LRW = YS + 5;           // y | m_eff | t_lo | t_hi | pad 2
  static constexpr int RW0 = DW + 1;  // first row of a contact record (after descriptor and mu)
  // word of generalized index i in a lane-major row: lane i % T, slice i / T
  static constexpr int yw(int i) { return (i % T) * NSL + i / T; }
  static constexpr int NJ1 = R::NJ > 0 ? R::NJ : 1;
  static constexpr int BW = 27;                // body record: Rm 9 | x 3 | c 3 | w 3 | v 3 | al 3 | ac 3
  static constexpr int FW = 12;                // its frame part (Rm | x) lives at O_FR, stride FW; the
  static constexpr int CW = 16;                // composite: J 6 | m r 3 | F 3 | N 3 | m
  // front path (pbg_fronts.h) of the distributed dynamics: state in LDS, front-parallel algebra
  static constexpr bool LST = FP<R>::NF > 0;
  // AL: the aligned layout -- 16-byte env regions whose records (frames, kinematic parts,
  // composites) start on 16-byte boundaries and whose 3-vectors pair up on 8-byte ones, so the
  // compiler, which can prove it from the kernel's address arithmetic, emits b64 / b128 accesses
  // with immediate offsets (round-4 A/B against 8-byte regions: Walker2D -7.6 %, HalfCheetah
  // -6.6 %, Hopper -2.5 %; Humanoid -8 % over the three steps).  The factor, 1 / diag and u start
  // on 16-byte boundaries on the front path (b128 factor loads).
  static constexpr bool AL = true;
  static constexpr int REGION_ALIGN = AL ? 4 : 2;
  // kinematic part (c | w | v | al | ac) at O_KV, stride KW (aligned layout: a 16-word record on a
  // 16-byte boundary, read and written as four b128; not for Atlas, whose 30 bodies' kinematic
  // area is the env region's floor and must stay within the LDS budget)
  static constexpr bool KAL = AL && !gang_big<R>();
  static constexpr int KW = KAL ? 16 : BW - FW;
  static constexpr int NNZ4 = LST ? (NNZ + 3) & ~3 : NNZ, N4 = LST ? (N + 3) & ~3 : N;
  // motion vectors s_w | s_v of generalized index i: the front path interleaves them per index
  // at an even word, stride SS = 6 (three b64 loads per index); the small trees keep two
  // stride-3 arrays (their round-3 layout)
  static constexpr int SS = AL ? 6 : 3;
  static constexpr int O_L = 0, O_LD = O_L + NNZ4, O_U = O_LD + N4, O_RHS = O_U + YS;
  static constexpr int O_SW = AL ? (O_RHS + N + 1) & ~1 : O_RHS + N, O_SV = AL ? O_SW + 3 : O_SW + 3 * N;
  static constexpr int O_Q = O_SW + 6 * N, O_QD = O_Q + NJ1, O_TAU = O_QD + NJ1;
  // joint axis | origin of dof d, interleaved like s_w | s_v on the front path
  static constexpr int O_JA = AL ? (O_TAU + NJ1 + 1) & ~1 : O_TAU + NJ1, O_JO = AL ? O_JA + 3 : O_JA + 3 * NJ1;
  // the base's state words [p 3 | quat 4 | v 3 | w 3] (front path: the env's state lives in LDS
  // through the sub-steps, q / qd at O_Q / O_QD)
  static constexpr int O_BS = O_JA + 6 * NJ1;
  static constexpr int O_CS = O_BS + (LST ? 13 : 0);  // HumanoidFlagrunHarder: the cube's state words (same layout)
  // front path: the body frames (FW = 12) and the composites / limit rows (CW = 16) on 16-byte
  // boundaries, so their records load as b128 with immediate offsets (ds_read2_b32 pairs past
  // the first KiB of the region needed a v_add_u32 per address)
  static constexpr int al4(int x) { return AL ? (x + 3) & ~3 : x; }
  static constexpr int O_FR = al4(O_CS + (R::harder ? 13 : 0)), O_LP = O_FR + FW * NB, O_LR = al4(O_LP + 2 * NLIM);
  static_assert(!R::harder || LST, "the cube robot runs the front path");
  // the composites (dead once M is built) share their words with the limit rows
  static constexpr int O_CP = O_LR;
  // limit rows in the device workspace (Atlas; HumanoidFlagrunHarder: its cube brings ~10 contacts
  // per env, and the 629 words of LDS limit rows -- dead once the PGS holds them in registers --
  // are 3 more LDS-resident contacts)
  static constexpr bool LIM_WS = gang_big<R>() || R::harder;
  static constexpr int LRSZ = (!LIM_WS && NLIM * LRW > NB * CW) ? NLIM * LRW : NB * CW;
  static constexpr int FIXED = O_LR + LRSZ + (Y64 ? ((O_LR + LRSZ + RW0) & 1) : 0);  // Y64: rows start even
  // rows per contact: normal, 2 lateral friction (+ spinning, 2 rolling: HalfCheetahMuJoCo's links)
  static constexpr int NRC = (R::spin_mu > 0.0 || R::roll_mu > 0.0) ? 6 : 3;
  static_assert(NRC == 3 || (!R::harder && R::NPAIR == 0), "torsional rows: robot-floor contacts only");
  static constexpr int PERC = RW0 + NRC * CRW + (Y64 ? ((RW0 + NRC * CRW) & 1) : 0);
  // the kinematic parts are dead once M and the bias are built, before any contact is
  // written: they share the start of the contact area (the env region holds >= KW*NB words)
  static constexpr int O_KV = KAL ? al4(FIXED) : FIXED;
  static constexpr int MIN_CONTACT_WORDS = (O_KV - FIXED) + KW * NB;
  static constexpr int GW_LR = (MAXC > 0 ? MAXC : 1) * PERC;    // LIM_WS: limit rows after the contacts
  static constexpr int GWORDS = GW_LR + (LIM_WS ? NLIM * LRW : 0);  // device workspace per env
  static constexpr int ROUNDS_S = (R::NS + T - 1) / T;
};

// per-lane view of the env's LDS region and device workspace
template <class S>
struct GangCtxT {
  lds_float* tabs;  // workgroup copy of GangTab<R> | GangDynTab<R> (4-byte words)
  lds_t<S>* l;   // env LDS region (words of the physics scalar S)
  S* g;          // env device workspace
  int cap;       // contacts resident in LDS
#ifdef PBG_DEV_CHECKS
  int env_words;  // the env region's words (contact_at's bound check)
#endif
  int t;         // lane in the gang
  int le;        // gang in the wave
  SimPT<S> P;    // scene parameters (kernel arguments)
};
template <class R>
using GangCtx = GangCtxT<real_t<R>>;
// n words (n % 4 == 0) from / to a 16-byte aligned LDS address as b128 accesses (front path:
// the composite records; the compiler split them into ds_read2_b32 pairs with an address add each)
template <int n, class S>
PBG_DEV void lds_ld4(const lds_t<S>* p, S* v) {
  typedef S v4f __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) const v4f lds_v4f;
#pragma unroll
  for (int k = 0; k < n / 4; k++) {
    const v4f a = ((lds_v4f*)p)[k];
    v[4 * k] = a.x; v[4 * k + 1] = a.y; v[4 * k + 2] = a.z; v[4 * k + 3] = a.w;
  }
}
template <int n, class S>
PBG_DEV void lds_st4(lds_t<S>* p, const S* v) {
  typedef S v4f __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) v4f lds_v4f;
#pragma unroll
  for (int k = 0; k < n / 4; k++) ((lds_v4f*)p)[k] = v4f{v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]};
}
// word w (0..26) of body b's record: frame part (w < 12) or kinematic part
template <class R, int T>
PBG_DEV lds_t<real_t<R>>* body_word(const lds_t<real_t<R>>* l, int b, int w) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
  return (LW*)l + (w < G::FW ? G::O_FR + G::FW * b + w : G::O_KV + G::KW * b + (w - G::FW));
}
// model tables, copied once per workgroup into LDS (vector-memory loads of a __constant__
// table indexed by lane cost hundreds of cycles each; the level loops chain several)
template <class R>
struct GangTabs {
  typedef __attribute__((address_space(3))) const GangTab<R> Tab;
  typedef __attribute__((address_space(3))) const GangDynTab<R> Dyn;
  static constexpr int TAB_COPY = (int)((gang_big<R>() ? offsetof(GangTab<R>, slot) : sizeof(GangTab<R>)) / 4);
  // 4-byte words; the tables end on a 16-byte (float32) or 32-byte (float64 regions: 4 words of 8
  // bytes) boundary, the alignment the env regions after them need
  static constexpr int AW = sizeof(real_t<R>) == 8 ? 8 : 4;
  static constexpr int TAB_WORDS = (TAB_COPY + AW - 1) / AW * AW;
  static constexpr int DYN_WORDS = (int)((sizeof(GangDynTab<R>) + 4 * AW - 1) / (4 * AW)) * AW;
  static constexpr int WORDS = TAB_WORDS + DYN_WORDS;
  static PBG_DEV Tab& tab(const lds_float* p) { return *(Tab*)p; }
  static PBG_DEV Dyn& dyn(const lds_float* p) { return *(Dyn*)(p + TAB_WORDS); }
};
// Lanes per workgroup: 4 waves of T-lane gangs; the float64 path (F64<R>: every region word 8
// bytes) takes 2 waves of 16-lane gangs when 16 envs' fixed words and four contacts each would not
// fit one CU's LDS (its 32-lane gangs keep 4 waves: 8 envs)
template <class R, int T>
constexpr int gang_block() {
  using G = Gang<R, T>;
  constexpr long need =
      4L * GangTabs<R>::WORDS + (long)(PBG_GANG_BLOCK / T) * (long)sizeof(real_t<R>) * (G::FIXED + 4L * G::PERC);
  // float64 Atlas: not even 8 envs' regions fit -- one-wave workgroups of 4 envs
  constexpr long need8 = 4L * GangTabs<R>::WORDS + 8L * (long)sizeof(real_t<R>) * (G::FIXED + G::MIN_CONTACT_WORDS);
  if constexpr (sizeof(real_t<R>) == 8 && T == 16 && need8 > 163840L) return PBG_GANG_BLOCK / 4;
  return sizeof(real_t<R>) == 8 && T == 16 && need > 163840L ? PBG_GANG_BLOCK / 2 : PBG_GANG_BLOCK;
}
#define PBG_GANG_SYNC                                    \
  {                                                      \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); \
    __builtin_amdgcn_wave_barrier();                     \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); \
  }

// word offset of contact c's record (24-bit multiply: the 64-bit v_mad_u64_u32 the compiler chose
// for the row addresses is a multi-pass instruction, two per normal row of the sweep)
template <class R, int T>
PBG_DEV int coff(int c) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  return (int)__umul24((unsigned)c, (unsigned)Gang<R, T>::PERC);
}
// f(p) with p the first word of contact c: its LDS record if resident, else its device
// workspace record -- one branch for a whole record's loads or stores (a per-word
// accessor left one divergent branch per word in the code: 442 branches in the detection
// pass, 186 in the rows pass)
template <class R, int T, class F>
PBG_DEV void contact_at(const GangCtx<R>& X, int c, F&& f) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
#ifdef PBG_DEV_CHECKS  // diagnostic build: a contact record inside its LDS region / workspace slice
  assert(c >= 0 && c < G::MAXC && (c >= X.cap || G::FIXED + (c + 1) * G::PERC <= X.env_words));
#endif
  if (c < X.cap) f(X.l + G::FIXED + coff<R, T>(c));
  else f(X.g + coff<R, T>(c));
}

// f(p) with p the first word of joint-limit row li (LDS, or the workspace for LIM_WS models)
template <class R, int T, class F>
PBG_DEV void limit_at(const GangCtx<R>& X, int li, F&& f) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
  if constexpr (G::LIM_WS) f(X.g + G::GW_LR + li * G::LRW);
  else f(X.l + G::O_LR + li * G::LRW);
}

// A contact row in registers (loaded one step ahead of its update: PGS software
// pipelining): this lane's slice of y, m_eff, target, lambda.
template <class R, int T>
struct GRow {
  using Sc = real_t<R>;
  Sc y[Gang<R, T>::NSL], meff, tgt, lam;
};
// row (c, dir); LDS: the caller knows every row of the wave is LDS-resident (no branch, so
// the compiler's LDS wait before the next update counts only this row's loads)
template <class R, int T, bool LDS>
PBG_DEV void gang_load_row(const GangCtx<R>& X, int c, int dir, GRow<R, T>& r) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
  typedef Sc v2f __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) const v2f lds_v2f;
  const int w0 = G::RW0 + dir * G::CRW;
  if (LDS || c < X.cap) {
    const LW* p = X.l + G::FIXED + coff<R, T>(c) + w0;
    if constexpr (G::Y64) {
      static_assert((G::FIXED + G::RW0) % 2 == 0 && G::PERC % 2 == 0 && G::CRW % 2 == 0, "b64 rows");
      const v2f a = *(lds_v2f*)(p + 2 * X.t);
      r.y[0] = a.x; r.y[1] = a.y;
    } else {
#pragma unroll
      for (int m = 0; m < G::NSL; m++) r.y[m] = p[X.t * G::NSL + m];
    }
    r.meff = p[G::YS]; r.tgt = p[G::YS + 1]; r.lam = p[G::YS + 2];
  } else {
    const Sc* p = X.g + coff<R, T>(c) + w0;
#pragma unroll
    for (int m = 0; m < G::NSL; m++) r.y[m] = p[X.t * G::NSL + m];
    r.meff = p[G::YS]; r.tgt = p[G::YS + 1]; r.lam = p[G::YS + 2];
  }
}
// friction bound of contact c: mu * lambda of its normal row
template <class R, int T, bool LDS>
PBG_DEV real_t<R> gang_fric_limit(const GangCtx<R>& X, int c) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
  typedef Sc v2f __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) const v2f lds_v2f;
  constexpr int w = G::RW0 + G::YS + 2;
  if (LDS || c < X.cap) {
    const LW* p = X.l + G::FIXED + coff<R, T>(c);
    return p[G::DW] * p[w];
  }
  const Sc* p = X.g + coff<R, T>(c);
  return p[G::DW] * p[w];
}
// lambda of contact c's normal row
template <class R, int T, bool LDS>
PBG_DEV real_t<R> gang_normal_lam(const GangCtx<R>& X, int c) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
  constexpr int w = G::RW0 + G::YS + 2;
  if (LDS || c < X.cap) return X.l[G::FIXED + coff<R, T>(c) + w];
  return X.g[coff<R, T>(c) + w];
}
template <class R, int T, bool LDS>
PBG_DEV void gang_set_lam(const GangCtx<R>& X, int c, int dir, real_t<R> v) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
  const int w = G::RW0 + dir * G::CRW + G::YS + 2;
  if (X.t == 0) {
    if (LDS || c < X.cap) X.l[G::FIXED + coff<R, T>(c) + w] = v;
    else X.g[coff<R, T>(c) + w] = v;
  }
}
// PGS update of a loaded row with u sliced over the gang; the new impulse has the same bits
// in every lane
template <class R, int T>
PBG_DEV real_t<R> gang_update(const GRow<R, T>& r, real_t<R>* us, real_t<R> lo, real_t<R> hi) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  Sc part = 0.f;
#pragma unroll
  for (int m = 0; m < Gang<R, T>::NSL; m++) part += r.y[m] * us[m];
  const Sc yu = gang_sum<T>(part);
  const Sc nl = clampf(r.lam + r.meff * (r.tgt - yu), lo, hi);
  const Sc dl = nl - r.lam;
#pragma unroll
  for (int m = 0; m < Gang<R, T>::NSL; m++) us[m] += r.y[m] * dl;
  return nl;
}
// One PGS sweep over the contact rows in Bullet's order: all normals, then the two friction
// rows of each contact whose normal impulse came out positive [EXT], box-clamped at
// mu * lambda_n.  Rows are loaded one step ahead of their update (two register sets
// alternate); the look-ahead loads are unconditional (the last row re-reads itself), and the
// normal pass records the positive impulses in a bitmask, so the friction pass walks those
// contacts without a load-then-test round trip.  Each gang leaves the loops on its own
// (the DPP reductions stay inside the gang's row of 16 lanes): with a wave-uniform loop and a
// masked update, a finished gang's look-ahead registers stayed pending on the skipped path
// and the compiler's wait at the loop head drained every LDS load (lgkmcnt(0)), so no row's
// loads overlapped the previous update.
// NW: 32-bit words of the positive-impulse mask (the caller takes NW = 1 when no env of the wave
// has more than 32 contacts, the model's full width otherwise)
template <class R, int T, bool LDS, int NW>
PBG_DEV void gang_contact_sweep(const GangCtx<R>& X, int nc, real_t<R>* us) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
  using Row = GRow<R, T>;
  if (nc <= 0) return;
  // positive normal impulses, one bit per contact in NW 32-bit words, set and walked
  // branch-free (selects over the words) -- the 64-bit mask with a branch per word cost 6-8 %
  // of the step; the three-word selects of the Humanoid's 95 candidates were 12 of a normal
  // row's ~50 instructions, hence the one-word instantiation for the common case
  if constexpr (NW > 4 || G::NRC == 6) {
    // more than 128 contact candidates (Atlas), or torsional rows (HalfCheetahMuJoCo): the plain
    // order -- every normal, [the spinning and rolling rows,] then the two friction rows of each
    // contact whose normal impulse came out positive, a load-then-test
    for (int c = 0; c < nc; c++) {
      Row A;
      gang_load_row<R, T, LDS>(X, c, 0, A);
      gang_set_lam<R, T, LDS>(X, c, 0, gang_update<R, T>(A, us, 0.f, 3.0e38f));
    }
    if constexpr (G::NRC == 6) {  // +-mu_t lambda_n, before the lateral friction (the oracle's order)
      for (int c = 0; c < nc; c++) {
        const Sc ln = gang_normal_lam<R, T, LDS>(X, c);
        if (!(ln > 0.f)) continue;
#pragma unroll
        for (int dir = 3; dir < 6; dir++) {
          const Sc lim = (Sc)(dir == 3 ? R::spin_mu : R::roll_mu) * ln;
          Row A;
          gang_load_row<R, T, LDS>(X, c, dir, A);
          gang_set_lam<R, T, LDS>(X, c, dir, gang_update<R, T>(A, us, -lim, lim));
        }
      }
    }
    for (int c = 0; c < nc; c++) {
      const Sc lim = gang_fric_limit<R, T, LDS>(X, c);
      if (!(lim > 0.f)) continue;  // mu * lambda_n: lambda_n > 0 (mu > 0)
      Row A1, A2;
      gang_load_row<R, T, LDS>(X, c, 1, A1);
      gang_set_lam<R, T, LDS>(X, c, 1, gang_update<R, T>(A1, us, -lim, lim));
      gang_load_row<R, T, LDS>(X, c, 2, A2);
      gang_set_lam<R, T, LDS>(X, c, 2, gang_update<R, T>(A2, us, -lim, lim));
    }
    return;
  }
  uint32_t pw0 = 0u, pw1 = 0u, pw2 = 0u, pw3 = 0u;
  auto pwr = [&](auto w_c) -> uint32_t& {
    constexpr int w = decltype(w_c)::value;
    if constexpr (w == 0) return pw0;
    else if constexpr (w == 1) return pw1;
    else if constexpr (w == 2) return pw2;
    else return pw3;
  };
  auto mark = [&](int c, Sc nl) {
    const uint32_t bit = nl > 0.f ? 1u << (c & 31) : 0u;
    if constexpr (NW == 1) {
      pw0 |= bit;
    } else {
      static_for<0, NW>([&](auto w_c) {
        constexpr int w = decltype(w_c)::value;
        pwr(w_c) |= (c >> 5) == w ? bit : 0u;  // selects (a branch per word became an indexed scratch store)
      });
    }
  };
  {
    if constexpr (LDS || G::NSL > 2) {  // (Atlas, NSL = 3: a third register set spilled)
      Row A, B;
      gang_load_row<R, T, LDS>(X, 0, 0, A);
      int c = 0;
      while (true) {
        gang_load_row<R, T, LDS>(X, min(c + 1, nc - 1), 0, B);
        Sc nl = gang_update<R, T>(A, us, 0.f, 3.0e38f);
        gang_set_lam<R, T, LDS>(X, c, 0, nl);
        mark(c, nl);
        if (++c >= nc) break;
        gang_load_row<R, T, LDS>(X, min(c + 1, nc - 1), 0, A);
        nl = gang_update<R, T>(B, us, 0.f, 3.0e38f);
        gang_set_lam<R, T, LDS>(X, c, 0, nl);
        mark(c, nl);
        if (++c >= nc) break;
      }
    } else {
      // rows past the LDS capacity come from the device workspace (L2): loaded two rows ahead,
      // three register sets in rotation (a row's impulse is written only by its own update, and a
      // clamped look-ahead that re-reads the last row is never used)
      Row A, B, C;
      gang_load_row<R, T, LDS>(X, 0, 0, A);
      gang_load_row<R, T, LDS>(X, min(1, nc - 1), 0, B);
      int c = 0;
      while (true) {
        gang_load_row<R, T, LDS>(X, min(c + 2, nc - 1), 0, C);
        Sc nl = gang_update<R, T>(A, us, 0.f, 3.0e38f);
        gang_set_lam<R, T, LDS>(X, c, 0, nl);
        mark(c, nl);
        if (++c >= nc) break;
        gang_load_row<R, T, LDS>(X, min(c + 2, nc - 1), 0, A);
        nl = gang_update<R, T>(B, us, 0.f, 3.0e38f);
        gang_set_lam<R, T, LDS>(X, c, 0, nl);
        mark(c, nl);
        if (++c >= nc) break;
        gang_load_row<R, T, LDS>(X, min(c + 2, nc - 1), 0, B);
        nl = gang_update<R, T>(C, us, 0.f, 3.0e38f);
        gang_set_lam<R, T, LDS>(X, c, 0, nl);
        mark(c, nl);
        if (++c >= nc) break;
      }
    }
  }
  // next contact with a positive normal impulse (-1: none left)
  auto next = [&]() -> int {
    int c = -1;
    static_for<0, NW>([&](auto k_c) {  // lowest non-empty word wins
      constexpr int w = NW - 1 - decltype(k_c)::value;
      const uint32_t m = pwr(std::integral_constant<int, w>{});
      c = m ? 32 * w + __builtin_ctz(m) : c;
    });
    // clear that bit: the lowest set bit of the first non-empty word
    bool done = false;
    static_for<0, NW>([&](auto w_c) {
      const uint32_t m = pwr(w_c);
      const bool take = !done && m != 0u;
      pwr(w_c) = take ? (m & (m - 1u)) : m;
      done = done || take;
    });
    return c;
  };
  int c = next();
  if (c < 0) return;
  Row A1, A2, B1, B2;
  gang_load_row<R, T, LDS>(X, c, 1, A1);
  gang_load_row<R, T, LDS>(X, c, 2, A2);
  Sc limA = gang_fric_limit<R, T, LDS>(X, c), limB;
  while (true) {
    int c2 = next();
    const bool more = c2 >= 0;
    c2 = more ? c2 : c;  // the last look-ahead re-reads the current contact
    gang_load_row<R, T, LDS>(X, c2, 1, B1);
    gang_load_row<R, T, LDS>(X, c2, 2, B2);
    limB = gang_fric_limit<R, T, LDS>(X, c2);
    gang_set_lam<R, T, LDS>(X, c, 1, gang_update<R, T>(A1, us, -limA, limA));
    gang_set_lam<R, T, LDS>(X, c, 2, gang_update<R, T>(A2, us, -limA, limA));
    if (!more) break;
    c = c2;
    c2 = next();
    const bool more2 = c2 >= 0;
    c2 = more2 ? c2 : c;
    gang_load_row<R, T, LDS>(X, c2, 1, A1);
    gang_load_row<R, T, LDS>(X, c2, 2, A2);
    limA = gang_fric_limit<R, T, LDS>(X, c2);
    gang_set_lam<R, T, LDS>(X, c, 1, gang_update<R, T>(B1, us, -limB, limB));
    gang_set_lam<R, T, LDS>(X, c, 2, gang_update<R, T>(B2, us, -limB, limB));
    if (!more2) break;
    c = c2;
  }
}

// Distributed unconstrained dynamics of one sub-step (the gang counterpart of dyn_mass):
// level-synchronous forward kinematics / velocities / bias accelerations (one body per
// lane per tree level), per-body inertia + wrench about the reference point O, composites
// by a leaf-to-root pass over the levels, then the packed lower triangle of M and the bias
// dealt round-robin over the lanes.  Everything lands in the gang's LDS: body records
// (frames for the collision pass), motion vectors sw / sv, M at O_L, the right-hand side
// at O_RHS.  Same formulas as dyn_mass with run-time model constants.
template <class R, int T>
PBG_DEV V3<real_t<R>> gang_O(const GangCtx<R>& X) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
  constexpr int rb = Dims<R>::REF_BODY;
  const LW* p = body_word<R, T>(X.l, rb, 12);
  return mk3<Sc>(p[0], p[1], p[2]);
}
// Forward kinematics / velocities / bias accelerations of one round of a tree level: lane
// t < KN owns body lev_body[K0 + t] (compile-time), reads its parent's record from LDS and
// writes its own.  Model constants are selected per lane (lvsel), so constants shared by the
// round's bodies fold (the lane kernel's kmul rules).
#define PBG_LV(expr) lvsel<R, K0, KN>(t, [&](auto bc_) { constexpr int b = decltype(bc_)::value; return (expr); })
#define PBG_LVI(expr) lvsel_i<R, K0, KN>(t, [&](auto bc_) { constexpr int b = decltype(bc_)::value; return (expr); })
template <class R, int T, int K0, int KN>
PBG_DEV void gang_fk_round(const GangCtx<R>& X) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
  using DTh = GangDT<R>;
  constexpr int JT = lv_jt<R>(K0, KN);
  const int t = opaque_lane(X.t);
  if (t >= KN) return;
  const int body = PBG_LVI(b), p = PBG_LVI(DTh::v.parent[b]), d = PBG_LVI(DTh::v.dof[b]);
  const LW* P = body_word<R, T>(X.l, p, 0);
  const LW* PK = body_word<R, T>(X.l, p, G::FW) - G::FW;  // PK[12..26]
  M3<Sc> Rp, Ro;
  Sc pr[G::FW + G::KW];  // the parent's record: frame | kinematic part
  if constexpr (G::KAL) {
    lds_ld4<G::FW>(P, pr);
    lds_ld4<G::KW>(PK + G::FW, pr + G::FW);
  } else {
#pragma unroll
    for (int i = 0; i < G::FW; i++) pr[i] = P[i];
#pragma unroll
    for (int i = G::FW; i < G::BW; i++) pr[i] = PK[i];
  }
#pragma unroll
  for (int i = 0; i < 9; i++) Rp.m[i] = pr[i];
  static_for<0, 9>([&](auto i_c) {
    constexpr int i = decltype(i_c)::value;
    Ro.m[i] = PBG_LV(DTh::v.ro[b][i]);
  });
  const V3<Sc> xp = mk3<Sc>(pr[9], pr[10], pr[11]), cp = mk3<Sc>(pr[12], pr[13], pr[14]), wp = mk3<Sc>(pr[15], pr[16], pr[17]);
  const V3<Sc> vp = mk3<Sc>(pr[18], pr[19], pr[20]), alp = mk3<Sc>(pr[21], pr[22], pr[23]), acp = mk3<Sc>(pr[24], pr[25], pr[26]);
  const M3<Sc> R0 = mul_kb(Rp, Ro);
  const V3<Sc> x0 = xp + mulc(Rp, PBG_LV(DTh::v.opos[b][0]), PBG_LV(DTh::v.opos[b][1]), PBG_LV(DTh::v.opos[b][2]));
  const V3<Sc> axl = mk3<Sc>(PBG_LV(DTh::v.axis[b][0]), PBG_LV(DTh::v.axis[b][1]), PBG_LV(DTh::v.axis[b][2]));
  const V3<Sc> anl = mk3<Sc>(PBG_LV(DTh::v.anchor[b][0]), PBG_LV(DTh::v.anchor[b][1]), PBG_LV(DTh::v.anchor[b][2]));
  const V3<Sc> com = mk3<Sc>(PBG_LV(DTh::v.com[b][0]), PBG_LV(DTh::v.com[b][1]), PBG_LV(DTh::v.com[b][2]));
  auto kin = [&](auto jt_c) {
    constexpr int jt = decltype(jt_c)::value;
    const Sc q = jt != 4 ? X.l[G::O_Q + d] : 0.f, qd = jt != 4 ? X.l[G::O_QD + d] : 0.f;
    M3<Sc> Rm = R0;
    V3<Sc> x = x0, w, v, al, ac, c;
    if constexpr (jt == 0) {
      Sc sn, cs;
      sincos_fast(q, &sn, &cs);
      const Sc t1 = 1.f - cs;
      M3<Sc> Rj;
      const Sc axx = PBG_LV(DTh::v.axis[b][0] * DTh::v.axis[b][0]), ayy = PBG_LV(DTh::v.axis[b][1] * DTh::v.axis[b][1]);
      const Sc azz = PBG_LV(DTh::v.axis[b][2] * DTh::v.axis[b][2]), axy = PBG_LV(DTh::v.axis[b][0] * DTh::v.axis[b][1]);
      const Sc axz = PBG_LV(DTh::v.axis[b][0] * DTh::v.axis[b][2]), ayz = PBG_LV(DTh::v.axis[b][1] * DTh::v.axis[b][2]);
      Rj.m[0] = kmul(axx, t1) + cs;                 Rj.m[1] = kmul(axy, t1) - kmul(axl.z, sn); Rj.m[2] = kmul(axz, t1) + kmul(axl.y, sn);
      Rj.m[3] = kmul(axy, t1) + kmul(axl.z, sn);    Rj.m[4] = kmul(ayy, t1) + cs;              Rj.m[5] = kmul(ayz, t1) - kmul(axl.x, sn);
      Rj.m[6] = kmul(axz, t1) - kmul(axl.y, sn);    Rj.m[7] = kmul(ayz, t1) + kmul(axl.x, sn); Rj.m[8] = kmul(azz, t1) + cs;
      Rm = mul_kb(R0, Rj);
      const V3<Sc> rja = mulc(Rj, anl);
      x = x0 + mulc(R0, anl - rja);
      c = x + mulc(Rm, com);
      const V3<Sc> a = mulc(R0, axl);
      const V3<Sc> o = x0 + mulc(R0, anl);
      const V3<Sc> ro = o - cp;
      const V3<Sc> vo = vp + cross3(wp, ro);
      const V3<Sc> ao = acp + cross3(alp, ro) + cross3(wp, cross3(wp, ro));
      w = wp + qd * a;
      al = alp + qd * cross3(wp, a);
      const V3<Sc> rc = c - o;
      v = vo + cross3(w, rc);
      ac = ao + cross3(al, rc) + cross3(w, cross3(w, rc));
      X.l[G::O_JA + G::SS * d] = a.x; X.l[G::O_JA + G::SS * d + 1] = a.y; X.l[G::O_JA + G::SS * d + 2] = a.z;
      X.l[G::O_JO + G::SS * d] = o.x; X.l[G::O_JO + G::SS * d + 1] = o.y; X.l[G::O_JO + G::SS * d + 2] = o.z;
    } else if constexpr (jt == 1) {
      const V3<Sc> a = mulc(R0, axl);
      x = x0 + q * a;
      c = x + mulc(Rm, com);
      const V3<Sc> r = c - cp;
      w = wp;
      al = alp;
      v = vp + cross3(wp, r) + qd * a;
      ac = acp + cross3(alp, r) + cross3(wp, cross3(wp, r)) + (2.f * qd) * cross3(wp, a);
      X.l[G::O_JA + G::SS * d] = a.x; X.l[G::O_JA + G::SS * d + 1] = a.y; X.l[G::O_JA + G::SS * d + 2] = a.z;
      X.l[G::O_JO + G::SS * d] = x0.x; X.l[G::O_JO + G::SS * d + 1] = x0.y; X.l[G::O_JO + G::SS * d + 2] = x0.z;
    } else {
      c = x + mulc(Rm, com);
      const V3<Sc> r = c - cp;
      w = wp;
      al = alp;
      v = vp + cross3(wp, r);
      ac = acp + cross3(alp, r) + cross3(wp, cross3(wp, r));
    }
    const Sc rec[G::BW + 1] = {Rm.m[0], Rm.m[1], Rm.m[2], Rm.m[3], Rm.m[4], Rm.m[5], Rm.m[6], Rm.m[7], Rm.m[8],
                                  x.x, x.y, x.z, c.x, c.y, c.z, w.x, w.y, w.z, v.x, v.y, v.z, al.x, al.y, al.z, ac.x, ac.y, ac.z, 0.f};
    if constexpr (G::KAL) {
      lds_st4<G::FW>(body_word<R, T>(X.l, body, 0), rec);
      lds_st4<G::KW>(body_word<R, T>(X.l, body, G::FW), rec + G::FW);
    } else {
#pragma unroll
      for (int i = 0; i < G::BW; i++) *body_word<R, T>(X.l, body, i) = rec[i];
    }
  };
  if constexpr (JT >= 0) {
    kin(std::integral_constant<int, JT>{});
  } else {
    const int jt = PBG_LVI(DTh::v.jt[b]);
    if (jt == 0) kin(std::integral_constant<int, 0>{});
    else if (jt == 1) kin(std::integral_constant<int, 1>{});
    else kin(std::integral_constant<int, 4>{});
  }
}

template <class R, int T>
PBG_DEV void gang_dyn_mass(const State<R>& s, const GangCtx<R>& X SUB_STAMP_ARGS) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using D = Dims<R>;
  using G = Gang<R, T>;
  auto& TD = GangTabs<R>::dyn(X.tabs);
  constexpr int NB = D::NB, N = R::NDOF, NLEV = gang_nlev<R>();
  const Sc g = X.P.gravity;
  const bool w0 = X.t == 0;
  // base record and joint state (replicated registers -> LDS; the front path keeps the state in
  // LDS: q / qd are there, the base words at O_BS)
  if (w0) {
    Sc bp[3], bq[4], bv[3], bw[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
      bp[i] = G::LST ? X.l[G::O_BS + i] : s.bp[i];
      bv[i] = G::LST ? X.l[G::O_BS + 7 + i] : s.bv[i];
      bw[i] = G::LST ? X.l[G::O_BS + 10 + i] : s.bw[i];
    }
#pragma unroll
    for (int i = 0; i < 4; i++) bq[i] = G::LST ? X.l[G::O_BS + 3 + i] : s.bq[i];
    const M3<Sc> Rb = quat_to_m3(bq[0], bq[1], bq[2], bq[3]);
    const Sc rec[G::BW] = {Rb.m[0], Rb.m[1], Rb.m[2], Rb.m[3], Rb.m[4], Rb.m[5], Rb.m[6], Rb.m[7], Rb.m[8],
                              bp[0], bp[1], bp[2], bp[0], bp[1], bp[2],
                              R::floating ? bw[0] : 0.f, R::floating ? bw[1] : 0.f, R::floating ? bw[2] : 0.f,
                              R::floating ? bv[0] : 0.f, R::floating ? bv[1] : 0.f, R::floating ? bv[2] : 0.f,
                              0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < G::BW; i++) *body_word<R, T>(X.l, 0, i) = rec[i];
    if constexpr (!G::LST) {
#pragma unroll
      for (int d = 0; d < R::NJ; d++) { X.l[G::O_Q + d] = s.q[d]; X.l[G::O_QD + d] = s.qd[d]; }
    }
  }
  PBG_GANG_SYNC
  // forward pass, one level at a time (a body's parent is one level up)
  static_for<1, NLEV>([&](auto lv_c) {
    constexpr int lv = decltype(lv_c)::value;
    constexpr int K0 = GangDT<R>::v.lev_start[lv], NBL = GangDT<R>::v.lev_start[lv + 1] - K0;
    static_for<0, (NBL + T - 1) / T>([&](auto r_c) {
      constexpr int r = decltype(r_c)::value;
      gang_fk_round<R, T, K0 + r * T, (NBL - r * T < T ? NBL - r * T : T)>(X);
    });
    PBG_GANG_SYNC
  });
  STAMP(0)
  const V3<Sc> O = gang_O<R, T>(X);
  // per-body inertia and wrench about O; motion vectors about O
#pragma unroll
  for (int r_ = 0; r_ < (NB + T - 1) / T; r_++) {  // rounds unrolled: table loads of all rounds overlap
    const int b = r_ * T + X.t;
    if (b >= NB) continue;
    const LW* P = body_word<R, T>(X.l, b, 0);
    const LW* PK = body_word<R, T>(X.l, b, G::FW) - G::FW;
    M3<Sc> Rm;
#pragma unroll
    for (int i = 0; i < 9; i++) Rm.m[i] = P[i];
    const V3<Sc> c = mk3<Sc>(PK[12], PK[13], PK[14]), w = mk3<Sc>(PK[15], PK[16], PK[17]), v = mk3<Sc>(PK[18], PK[19], PK[20]);
    const V3<Sc> al = mk3<Sc>(PK[21], PK[22], PK[23]), ac = mk3<Sc>(PK[24], PK[25], PK[26]);
    const Sc m = TD.mass[b];
    Sc I6[6];
#pragma unroll
    for (int i = 0; i < 6; i++) I6[i] = TD.inertia[b][i];
    const S6<Sc> Iw = rotate_inertia(Rm, I6);
    const V3<Sc> r = c - O;
    const Sc rr = dot3(r, r);
    const V3<Sc> Iww = mul(Iw, w);
    const V3<Sc> f = m * (ac - mk3<Sc>(0, 0, -g)) + (m * ((Sc)PBG_LINEAR_DAMPING + (Sc)PBG_LINEAR_DAMPING * norm3(v))) * v;
    const V3<Sc> n = mul(Iw, al) + cross3(w, Iww) + ((Sc)PBG_ANGULAR_DAMPING + (Sc)PBG_ANGULAR_DAMPING * norm3(w)) * Iww;
    const V3<Sc> pr = m * r, Nn = n + cross3(r, f);
    const Sc cmp[G::CW] = {Iw.a[0] + m * (rr - r.x * r.x), Iw.a[1] + m * (rr - r.y * r.y), Iw.a[2] + m * (rr - r.z * r.z),
                              Iw.a[3] - m * r.x * r.y, Iw.a[4] - m * r.x * r.z, Iw.a[5] - m * r.y * r.z,
                              pr.x, pr.y, pr.z, f.x, f.y, f.z, Nn.x, Nn.y, Nn.z, m};
    LW* C = X.l + G::O_CP + G::CW * b;
    const bool massive = m > 0.f;
    Sc cv[G::CW];
#pragma unroll
    for (int i = 0; i < G::CW; i++) cv[i] = massive ? cmp[i] : 0.f;
    if constexpr (G::AL) lds_st4<G::CW>(C, cv);
    else {
#pragma unroll
      for (int i = 0; i < G::CW; i++) C[i] = cv[i];
    }
  }
#pragma unroll
  for (int r_ = 0; r_ < (N + T - 1) / T; r_++) {
    const int i = r_ * T + X.t;
    if (i >= N) continue;
    const int d = TD.g_dof[i];
    V3<Sc> sw, sv;
    if (d >= 0) {
      const V3<Sc> a = mk3<Sc>(X.l[G::O_JA + G::SS * d], X.l[G::O_JA + G::SS * d + 1], X.l[G::O_JA + G::SS * d + 2]);
      const V3<Sc> o = mk3<Sc>(X.l[G::O_JO + G::SS * d], X.l[G::O_JO + G::SS * d + 1], X.l[G::O_JO + G::SS * d + 2]);
      const bool rev = TD.jt[TD.g_body[i]] == 0;
      sw = rev ? a : mk3<Sc>(0, 0, 0);
      sv = rev ? cross3(o - O, a) : a;
    } else {
      const int kk = i - R::NJ;  // 0..2 linear, 3..5 angular
      const V3<Sc> e = mk3<Sc>(kk % 3 == 0, kk % 3 == 1, kk % 3 == 2);
      sw = kk < 3 ? mk3<Sc>(0, 0, 0) : e;
      sv = kk < 3 ? e : mk3<Sc>(0, 0, 0);
    }
    X.l[G::O_SW + G::SS * i] = sw.x; X.l[G::O_SW + G::SS * i + 1] = sw.y; X.l[G::O_SW + G::SS * i + 2] = sw.z;
    X.l[G::O_SV + G::SS * i] = sv.x; X.l[G::O_SV + G::SS * i + 1] = sv.y; X.l[G::O_SV + G::SS * i + 2] = sv.z;
  }
  PBG_GANG_SYNC
  STAMP(1)
  // composites: leaf-to-root over the levels (a body adds its children's sums)
  static_for<0, NLEV - 1>([&](auto k_c) {
    constexpr int lv = NLEV - 2 - decltype(k_c)::value;
    using GC = GangComp<R>;
    constexpr int NBL = GC::v.cnt[lv];
    static_for<0, (NBL + T - 1) / T>([&](auto r_c) {
      constexpr int K0 = decltype(r_c)::value * T, KN = NBL - K0 < T ? NBL - K0 : T;
      constexpr int MC = GC::maxch(lv, K0, KN);
      using S = CompSrc<R, lv, K0>;
      const int t = opaque_lane(X.t);
      if (t < KN) {
        const int b = ksel<S, KN, int>(t, [&](auto bc) { return decltype(bc)::value; });
        LW* C = X.l + G::O_CP + G::CW * b;
        Sc acc[G::CW];
        if constexpr (G::AL) lds_ld4<G::CW>(C, acc);
        else {
#pragma unroll
          for (int i = 0; i < G::CW; i++) acc[i] = C[i];
        }
        static_for<0, MC>([&](auto j_c) {
          constexpr int j = decltype(j_c)::value;
          const int c = ksel<S, KN, int>(t, [&](auto bc) { return j < GC::v.nch[decltype(bc)::value] ? GC::v.ch[decltype(bc)::value][j] : -1; });
          if (c >= 0) {
            const LW* K = X.l + G::O_CP + G::CW * c;
            Sc kv[G::CW];
            if constexpr (G::AL) lds_ld4<G::CW>(K, kv);
            else {
#pragma unroll
              for (int i = 0; i < G::CW; i++) kv[i] = K[i];
            }
#pragma unroll
            for (int i = 0; i < G::CW; i++) acc[i] += kv[i];
          }
        });
        if constexpr (G::AL) lds_st4<G::CW>(C, acc);
        else {
#pragma unroll
          for (int i = 0; i < G::CW; i++) C[i] = acc[i];
        }
      }
    });
    PBG_GANG_SYNC
  });
  STAMP(2)
  // per generalized index k (one per lane): f_k = I^c s_k of its composite (angular |
  // linear part) into the dead kinematic area past the reference body's record (gang_O
  // still reads that), and the bias C_k = s_k . (N, F) of the same composite
  constexpr int O_FK = G::O_KV + G::KW * (Dims<R>::REF_BODY + 1);
  static_assert((G::O_KV - G::FIXED) + G::KW * (Dims<R>::REF_BODY + 1) + 6 * N <= G::MIN_CONTACT_WORDS, "f_k past the kinematic area");
#pragma unroll
  for (int r_ = 0; r_ < (N + T - 1) / T; r_++) {
    const int k = r_ * T + X.t;
    if (k >= N) continue;
    const int bk = TD.g_body[k], d = TD.g_dof[k];
    const LW* Cp = X.l + G::O_CP + G::CW * bk;
    Sc C[G::CW];
    if constexpr (G::AL) lds_ld4<G::CW>(Cp, C);
    else {
#pragma unroll
      for (int i = 0; i < G::CW; i++) C[i] = Cp[i];
    }
    S6<Sc> J;
#pragma unroll
    for (int i = 0; i < 6; i++) J.a[i] = C[i];
    const V3<Sc> p1 = mk3<Sc>(C[6], C[7], C[8]);
    const Sc cm = C[15];
    const V3<Sc> swk = mk3<Sc>(X.l[G::O_SW + G::SS * k], X.l[G::O_SW + G::SS * k + 1], X.l[G::O_SW + G::SS * k + 2]);
    const V3<Sc> svk = mk3<Sc>(X.l[G::O_SV + G::SS * k], X.l[G::O_SV + G::SS * k + 1], X.l[G::O_SV + G::SS * k + 2]);
    const V3<Sc> Jw_ = mul(J, swk) + cross3(p1, svk);
    const V3<Sc> Fv = cm * svk - cross3(p1, swk);
    LW* f = X.l + O_FK + 6 * k;
    f[0] = Jw_.x; f[1] = Jw_.y; f[2] = Jw_.z; f[3] = Fv.x; f[4] = Fv.y; f[5] = Fv.z;
    const V3<Sc> F = mk3<Sc>(C[9], C[10], C[11]), Nn = mk3<Sc>(C[12], C[13], C[14]);
    Sc r = -(dot3(swk, Nn) + dot3(svk, F));
    if (d >= 0) {
      r += X.l[G::O_TAU + d] - TD.damping[d] * X.l[G::O_QD + d];
      if constexpr (has_springs<R>()) r -= TD.stiffness[d] * X.l[G::O_Q + d];  // mjcf.py B7
    }
    X.l[G::O_RHS + k] = r;
  }
  PBG_GANG_SYNC
  // packed lower triangle of M: M_ik = s_i . f_k (+ armature)
#pragma unroll
  for (int r_ = 0; r_ < (D::NNZ + T - 1) / T; r_++) {
    const int j = r_ * T + X.t;
    if (j >= D::NNZ) continue;
    const int gi = TD.me_i[j], gk = TD.me_k[j];
    const LW* f = X.l + O_FK + 6 * gk;
    const V3<Sc> Jw_ = mk3<Sc>(f[0], f[1], f[2]), Fv = mk3<Sc>(f[3], f[4], f[5]);
    const V3<Sc> swi = mk3<Sc>(X.l[G::O_SW + G::SS * gi], X.l[G::O_SW + G::SS * gi + 1], X.l[G::O_SW + G::SS * gi + 2]);
    const V3<Sc> svi = mk3<Sc>(X.l[G::O_SV + G::SS * gi], X.l[G::O_SV + G::SS * gi + 1], X.l[G::O_SV + G::SS * gi + 2]);
    X.l[G::O_L + j] = (dot3(swi, Jw_) + dot3(svi, Fv)) + TD.me_arm[j];
  }
  PBG_GANG_SYNC
}

// ------------------------------------------------------------------ front-parallel linear algebra
// (pbg_fronts.h).  Lane t of a gang works on front q = t % FP (lanes q >= NF only add zeros to
// the group sums); the group of FP lanes sums the fronts' Schur terms and trunk right-hand
// sides by DPP; the trunk is factored and solved replicated.  The gang's first FP lanes store
// the fronts' words, lane 0 the trunk's.
template <class R>
struct TrunkTab {
  static constexpr int NT = FP<R>::NT;
  static constexpr int count() {
    int c = 0;
    for (int t1 = 0; t1 < NT; t1++)
      for (int t2 = 0; t2 <= t1; t2++) c += Dims<R>::coupled(FP<R>::v.tg[t1], FP<R>::v.tg[t2]);
    return c;
  }
  static constexpr int NT2 = count() > 0 ? count() : 1;
  // word of trunk pair (t1 >= t2) within the trunk block (-1: structurally zero)
  static constexpr int pos(int t1, int t2) {
    return Dims<R>::coupled(FP<R>::v.tg[t1], FP<R>::v.tg[t2]) ? FP<R>::v.idx[FP<R>::v.tg[t1]][FP<R>::v.tg[t2]] - FP<R>::v.toff
                                                                : -1;
  }
  static constexpr int BMAX() {
    int m = 1;
    for (int f = 0; f < FP<R>::NF; f++) m = FP<R>::v.bsz[f] > m ? FP<R>::v.bsz[f] : m;
    return m;
  }
  static constexpr int NMAX() {
    int m = 1;
    for (int f = 0; f < FP<R>::NF; f++) m = FP<R>::v.n[f] > m ? FP<R>::v.n[f] : m;
    return m;
  }
};
// per-lane pick of a compile-time front quantity fn(f) (f = the lane's front; -1 when q >= NF)
template <class R>
struct FrontSrc {
  static constexpr int at(int k) { return k; }
};
template <class R, class F>
PBG_DEV int front_pick(int q, F&& fn) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  return ksel<FrontSrc<R>, FP<R>::NF, int>(q, [&](auto fc) { return fn(decltype(fc)::value); });
}
// the trunk index t's joint velocity / base velocity from the env's LDS state (compile-time t)
template <class R, int T, int t>
PBG_DEV real_t<R> trunk_nu(const GangCtx<R>& X) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
  constexpr int g = FP<R>::v.tg[t], d = Dims<R>::dof_of(g);
  if constexpr (d >= 0) return X.l[G::O_QD + d];
  else return X.l[G::O_BS + 7 + (g - R::NJ)];  // v 3 | w 3
}

// Front-parallel replacement of dyn_solve: M (front-major words at O_L) and the right-hand side
// (O_RHS) from LDS; factor, nu_pred = clamp(nu + dt M^-1 rhs), u = L^T nu_pred; stages L (in
// place, the same word order), 1 / diag(L) (O_LD), u (O_U) and the limit positions (O_LP).
template <class R, int T>
PBG_DEV void gang_front_solve(const State<R>& s, const GangCtx<R>& X) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using D = Dims<R>;
  using G = Gang<R, T>;
  using TT = TrunkTab<R>;
  constexpr int NF = FP<R>::NF, GRP = FP<R>::GRP, NT = FP<R>::NT, NT2 = TT::NT2, BM = TT::BMAX(), NM = TT::NMAX();
  const Sc dt = X.P.dt;
  const int q = opaque_lane(X.t) % GRP;
  const int cls = q < NF ? front_pick<R>(q, [](int f) { return FP<R>::v.cls[f]; }) : -1;
  const int boff = front_pick<R>(q, [](int f) { return FP<R>::v.off[f]; });
  const int g0 = front_pick<R>(q, [](int f) { return FP<R>::v.g0[f]; });
  const LW* blk = X.l + G::O_L + boff;
  Sc Fb[BM], Fd[NM], Fy[NM];  // the lane's front block (factored in place), 1 / diag, forward solve
  Sc S[NT2], z[NT];           // Schur terms W W^T (trunk pairs) and trunk right-hand-side terms
#pragma unroll
  for (int i = 0; i < NT2; i++) S[i] = 0.f;
#pragma unroll
  for (int i = 0; i < NT; i++) z[i] = 0.f;
  // --- fronts: factor, forward solve ---------------------------------------------------------
  static_for<0, FP<R>::v.ncls>([&](auto c_c) {
    constexpr int C = decltype(c_c)::value;
    using FC = FrontCls<R, C>;
    constexpr int n = FC::n;
    if (cls != C) return;
    constexpr int bs = FP<R>::v.bsz[FC::f];
#pragma unroll
    for (int i = 0; i < bs; i++) Fb[i] = blk[i];
    static_for<0, n>([&](auto a_c) {
      constexpr int a = decltype(a_c)::value;
      const Sc d = fast_sqrt(Fb[FC::a_off(a, a)]);
      const Sc r = fast_rcp(d);
      Fb[FC::a_off(a, a)] = d;
      Fd[a] = r;
      static_for<a + 1, n>([&](auto b_c) {
        constexpr int b = decltype(b_c)::value;
        if constexpr (FC::cpl(b, a)) Fb[FC::a_off(b, a)] *= r;
      });
      static_for<0, NT>([&](auto t_c) {
        constexpr int t = decltype(t_c)::value;
        if constexpr (FC::tc(t)) Fb[FC::c_off(a, t)] *= r;
      });
      static_for<a + 1, n>([&](auto b_c) {
        constexpr int b = decltype(b_c)::value;
        if constexpr (FC::cpl(b, a)) {
          static_for<a + 1, b + 1>([&](auto b2_c) {
            constexpr int b2 = decltype(b2_c)::value;
            if constexpr (FC::cpl(b2, a) && FC::cpl(b, b2)) Fb[FC::a_off(b, b2)] -= Fb[FC::a_off(b, a)] * Fb[FC::a_off(b2, a)];
          });
          static_for<0, NT>([&](auto t_c) {
            constexpr int t = decltype(t_c)::value;
            if constexpr (FC::tc(t)) Fb[FC::c_off(b, t)] -= Fb[FC::c_off(a, t)] * Fb[FC::a_off(b, a)];
          });
        }
      });
      static_for<0, NT>([&](auto t1_c) {
        constexpr int t1 = decltype(t1_c)::value;
        if constexpr (FC::tc(t1)) {
          static_for<0, t1 + 1>([&](auto t2_c) {
            constexpr int t2 = decltype(t2_c)::value;
            if constexpr (FC::tc(t2)) S[TT::pos(t1, t2)] += Fb[FC::c_off(a, t1)] * Fb[FC::c_off(a, t2)];
          });
        }
      });
    });
    // forward solve L_f y_f = rhs_f; trunk terms z_t += L_(t,a) y_a
    static_for<0, n>([&](auto a_c) {
      constexpr int a = decltype(a_c)::value;
      Sc v = X.l[G::O_RHS + g0 + a];
      static_for<0, a>([&](auto b_c) {
        constexpr int b = decltype(b_c)::value;
        if constexpr (FC::cpl(a, b)) v -= Fb[FC::a_off(a, b)] * Fy[b];
      });
      Fy[a] = v * Fd[a];
      static_for<0, NT>([&](auto t_c) {
        constexpr int t = decltype(t_c)::value;
        if constexpr (FC::tc(t)) z[t] += Fb[FC::c_off(a, t)] * Fy[a];
      });
    });
  });
  // --- trunk: T - sum_f W_f W_f^T, factor, forward + backward solve ---------------------------
  const LW* tb = X.l + G::O_L + FP<R>::v.toff;
  Sc Lt[NT2], Ldt[NT], yt[NT], xt[NT];
#pragma unroll
  for (int i = 0; i < NT2; i++) Lt[i] = tb[i] - gang_sum<GRP>(S[i]);
  static_for<0, NT>([&](auto j_c) {
    constexpr int j = decltype(j_c)::value;
    const Sc d = fast_sqrt(Lt[TT::pos(j, j)]);
    const Sc r = fast_rcp(d);
    Lt[TT::pos(j, j)] = d;
    Ldt[j] = r;
    static_for<j + 1, NT>([&](auto i_c) {
      constexpr int i = decltype(i_c)::value;
      if constexpr (TT::pos(i, j) >= 0) Lt[TT::pos(i, j)] *= r;
    });
    static_for<j + 1, NT>([&](auto i_c) {
      constexpr int i = decltype(i_c)::value;
      if constexpr (TT::pos(i, j) >= 0) {
        static_for<j + 1, i + 1>([&](auto k_c) {
          constexpr int k = decltype(k_c)::value;
          if constexpr (TT::pos(k, j) >= 0 && TT::pos(i, k) >= 0) Lt[TT::pos(i, k)] -= Lt[TT::pos(i, j)] * Lt[TT::pos(k, j)];
        });
      }
    });
  });
  static_for<0, NT>([&](auto t_c) {
    constexpr int t = decltype(t_c)::value;
    Sc v = X.l[G::O_RHS + FP<R>::v.tg[t]] - gang_sum<GRP>(z[t]);
    static_for<0, t>([&](auto k_c) {
      constexpr int k = decltype(k_c)::value;
      if constexpr (TT::pos(t, k) >= 0) v -= Lt[TT::pos(t, k)] * yt[k];
    });
    yt[t] = v * Ldt[t];
  });
  static_for<0, NT>([&](auto r_c) {
    constexpr int t = NT - 1 - decltype(r_c)::value;
    Sc v = yt[t];
    static_for<t + 1, NT>([&](auto k_c) {
      constexpr int k = decltype(k_c)::value;
      if constexpr (TT::pos(k, t) >= 0) v -= Lt[TT::pos(k, t)] * xt[k];
    });
    xt[t] = v * Ldt[t];
  });
  // trunk nu_pred and u_t = L_t^T nu_t
  Sc nut[NT];
  static_for<0, NT>([&](auto t_c) {
    constexpr int t = decltype(t_c)::value;
    nut[t] = clampf(trunk_nu<R, T, t>(X) + dt * xt[t], -(Sc)PBG_MAX_COORD_VELOCITY, (Sc)PBG_MAX_COORD_VELOCITY);
  });
  const bool wf = X.t < GRP && q < NF;  // the gang's front writers
  // --- fronts: backward solve, nu_pred, u_f; store --------------------------------------------
  static_for<0, FP<R>::v.ncls>([&](auto c_c) {
    constexpr int C = decltype(c_c)::value;
    using FC = FrontCls<R, C>;
    constexpr int n = FC::n;
    if (cls != C) return;
    Sc xf[n], nuf[n];
    static_for<0, n>([&](auto r_c) {
      constexpr int a = n - 1 - decltype(r_c)::value;
      Sc v = Fy[a];
      static_for<a + 1, n>([&](auto b_c) {
        constexpr int b = decltype(b_c)::value;
        if constexpr (FC::cpl(b, a)) v -= Fb[FC::a_off(b, a)] * xf[b];
      });
      static_for<0, NT>([&](auto t_c) {
        constexpr int t = decltype(t_c)::value;
        if constexpr (FC::tc(t)) v -= Fb[FC::c_off(a, t)] * xt[t];
      });
      xf[a] = v * Fd[a];
    });
    // joint dof of local a: NJ - 1 - (g0 + a); its velocity from the gang's LDS copy of qd
    const LW* qd = X.l + G::O_QD + (R::NJ - 1 - g0);
    static_for<0, n>([&](auto a_c) {
      constexpr int a = decltype(a_c)::value;
      nuf[a] = clampf(qd[-a] + dt * xf[a], -(Sc)PBG_MAX_COORD_VELOCITY, (Sc)PBG_MAX_COORD_VELOCITY);
    });
    if (wf) {
      LW* wb = X.l + G::O_L + boff;
      constexpr int bs = FP<R>::v.bsz[FC::f];
#pragma unroll
      for (int i = 0; i < bs; i++) wb[i] = Fb[i];
      static_for<0, n>([&](auto a_c) {
        constexpr int a = decltype(a_c)::value;
        Sc u = 0.f;
        static_for<a, n>([&](auto b_c) {
          constexpr int b = decltype(b_c)::value;
          if constexpr (FC::cpl(b, a)) u += Fb[FC::a_off(b, a)] * nuf[b];
        });
        static_for<0, NT>([&](auto t_c) {
          constexpr int t = decltype(t_c)::value;
          if constexpr (FC::tc(t)) u += Fb[FC::c_off(a, t)] * nut[t];
        });
        X.l[G::O_LD + g0 + a] = Fd[a];
        X.l[G::O_U + g0 + a] = u;
      });
    }
  });
  if (X.t == 0) {
    LW* wt = X.l + G::O_L + FP<R>::v.toff;
#pragma unroll
    for (int i = 0; i < NT2; i++) wt[i] = Lt[i];
    static_for<0, NT>([&](auto t_c) {
      constexpr int t = decltype(t_c)::value;
      Sc u = 0.f;
      static_for<t, NT>([&](auto k_c) {
        constexpr int k = decltype(k_c)::value;
        if constexpr (TT::pos(k, t) >= 0) u += Lt[TT::pos(k, t)] * nut[k];
      });
      X.l[G::O_LD + FP<R>::v.tg[t]] = Ldt[t];
      X.l[G::O_U + FP<R>::v.tg[t]] = u;
    });
    if constexpr (R::harder) {
      // the cube (block-diagonal, factor diag(sqrt m x3, sqrt I x3)): u_c = L_c^T nu_c of its
      // free-body unconstrained velocity (cube_unconstrained on the LDS copy of its state)
      State<R> cs;
#pragma unroll
      for (int i = 0; i < 3; i++) { cs.cube.v[i] = X.l[G::O_CS + 7 + i]; cs.cube.w[i] = X.l[G::O_CS + 10 + i]; }
      Sc uc[6];
      cube_unconstrained<R>(cs, uc, X.P);
#pragma unroll
      for (int i = 0; i < 6; i++) X.l[G::O_U + R::NDOF + i] = uc[i];
    }
#pragma unroll
    for (int i = D::NY; i < G::YS; i++) X.l[G::O_U + i] = 0.f;
    static_for<0, D::NLIM>([&](auto li_c) {
      constexpr int li = decltype(li_c)::value;
      constexpr int d = D::LIM.v[li][0];
      X.l[G::O_LP + 2 * li] = X.l[G::O_Q + d] - (Sc)R::dof_lower[d];
      X.l[G::O_LP + 2 * li + 1] = (Sc)R::dof_upper[d] - X.l[G::O_Q + d];
    });
  }
  (void)NM;
  (void)s;
}

// The staged factor (word order pbg_fronts.h) and 1 / diag(L) into registers, as 16-byte LDS loads
template <class R, int T>
PBG_DEV void gang_load_factor(const GangCtx<R>& X, real_t<R>* L, real_t<R>* Ld) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
  typedef Sc v4f __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) const v4f lds_v4f;
  const lds_v4f* pl = (const lds_v4f*)(X.l + G::O_L);
#pragma unroll
  for (int k = 0; k < G::NNZ4 / 4; k++) {
    const v4f a = pl[k];
    L[4 * k] = a.x; L[4 * k + 1] = a.y; L[4 * k + 2] = a.z; L[4 * k + 3] = a.w;
  }
  const lds_v4f* pd = (const lds_v4f*)(X.l + G::O_LD);
#pragma unroll
  for (int k = 0; k < G::N4 / 4; k++) {
    const v4f a = pd[k];
    Ld[4 * k] = a.x; Ld[4 * k + 1] = a.y; Ld[4 * k + 2] = a.z; Ld[4 * k + 3] = a.w;
  }
}

// The front path's integration: nu = L^-T u, front-parallel like gang_front_solve (the trunk's
// back-substitution replicated, then lane q < NF of each group its front's, with the trunk terms
// last: the same summation order as a dense back-substitution over the leaf-first order),
// clamped; the env's LDS state advanced by semi-implicit Euler (the first group's front lanes
// their fronts' joints, lane 0 the trunk joints, the base and the cube; the next sub-step reads
// them after its first gang sync)
template <class R, int T>
PBG_DEV void gang_front_integrate(State<R>& s, const GangCtx<R>& X) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
  using D = Dims<R>;
  using TT = TrunkTab<R>;
  constexpr int NJ = R::NJ, N = R::NDOF, NF = FP<R>::NF, GRP = FP<R>::GRP, NT = FP<R>::NT, NT2 = TT::NT2;
  const Sc dt = X.P.dt;
  const Sc vmax = (Sc)PBG_MAX_COORD_VELOCITY;
  // --- trunk ---------------------------------------------------------------------------------
  const LW* tb = X.l + G::O_L + FP<R>::v.toff;
  Sc Lt[NT2], xt[NT];
#pragma unroll
  for (int i = 0; i < NT2; i++) Lt[i] = tb[i];
  static_for<0, NT>([&](auto r_c) {
    constexpr int t = NT - 1 - decltype(r_c)::value;
    constexpr int g = FP<R>::v.tg[t];
    Sc v = X.l[G::O_U + g];
    static_for<t + 1, NT>([&](auto k_c) {
      constexpr int k = decltype(k_c)::value;
      if constexpr (TT::pos(k, t) >= 0) v -= Lt[TT::pos(k, t)] * xt[k];
    });
    xt[t] = v * X.l[G::O_LD + g];
  });
  Sc nut[NT];
#pragma unroll
  for (int t = 0; t < NT; t++) nut[t] = clampf(xt[t], -vmax, vmax);
  // --- fronts --------------------------------------------------------------------------------
  const int q = opaque_lane(X.t) % GRP;
  const int cls = q < NF ? front_pick<R>(q, [](int f) { return FP<R>::v.cls[f]; }) : -1;
  const int boff = front_pick<R>(q, [](int f) { return FP<R>::v.off[f]; });
  const int g0 = front_pick<R>(q, [](int f) { return FP<R>::v.g0[f]; });
  const bool wf = X.t < GRP && q < NF;  // the gang's front writers
  static_for<0, FP<R>::v.ncls>([&](auto c_c) {
    constexpr int C = decltype(c_c)::value;
    using FC = FrontCls<R, C>;
    constexpr int n = FC::n;
    if (cls != C) return;
    const LW* blk = X.l + G::O_L + boff;
    Sc xf[n];
    static_for<0, n>([&](auto r_c) {
      constexpr int a = n - 1 - decltype(r_c)::value;
      Sc v = X.l[G::O_U + g0 + a];
      static_for<a + 1, n>([&](auto b_c) {
        constexpr int b = decltype(b_c)::value;
        if constexpr (FC::cpl(b, a)) v -= blk[FC::a_off(b, a)] * xf[b];
      });
      static_for<0, NT>([&](auto t_c) {
        constexpr int t = decltype(t_c)::value;
        if constexpr (FC::tc(t)) v -= blk[FC::c_off(a, t)] * xt[t];
      });
      xf[a] = v * X.l[G::O_LD + g0 + a];
    });
    if (wf) {
      // joint dof of local a: NJ - 1 - (g0 + a) (leaf-first order)
      LW* qd = X.l + G::O_QD + (NJ - 1 - g0);
      LW* qq = X.l + G::O_Q + (NJ - 1 - g0);
      static_for<0, n>([&](auto a_c) {
        constexpr int a = decltype(a_c)::value;
        const Sc v = clampf(xf[a], -vmax, vmax);
        qd[-a] = v;
        qq[-a] += dt * v;
      });
    }
  });
  Sc nu[N];  // the trunk part (compile-time indices; the fronts' entries are not used below)
  static_for<0, NT>([&](auto t_c) {
    constexpr int t = decltype(t_c)::value;
    nu[FP<R>::v.tg[t]] = nut[t];
  });
  if (X.t == 0) {
    static_for<0, NT>([&](auto t_c) {
      constexpr int t = decltype(t_c)::value;
      constexpr int d = D::dof_of(FP<R>::v.tg[t]);
      if constexpr (d >= 0) {
        X.l[G::O_QD + d] = nut[t];
        X.l[G::O_Q + d] += dt * nut[t];
      }
    });
  }
  if (X.t == 0) {
    if constexpr (R::floating) {
      Sc bq[4];
#pragma unroll
      for (int i = 0; i < 4; i++) bq[i] = X.l[G::O_BS + 3 + i];
#pragma unroll
      for (int i = 0; i < 3; i++) {
        X.l[G::O_BS + 7 + i] = nu[NJ + i];
        X.l[G::O_BS + 10 + i] = nu[NJ + 3 + i];
        X.l[G::O_BS + i] += dt * nu[NJ + i];
      }
      free_body_quat(bq, mk3<Sc>(nu[NJ + 3], nu[NJ + 4], nu[NJ + 5]), X.P);
#pragma unroll
      for (int i = 0; i < 4; i++) X.l[G::O_BS + 3 + i] = bq[i];
    }
    if constexpr (R::harder) {  // the cube: nu_c = L_c^-T u_c, clamp, semi-implicit Euler (cube_integrate)
      State<R> cs;
#pragma unroll
      for (int i = 0; i < 3; i++) cs.cube.p[i] = X.l[G::O_CS + i];
#pragma unroll
      for (int i = 0; i < 4; i++) cs.cube.q[i] = X.l[G::O_CS + 3 + i];
      Sc uc[6];
#pragma unroll
      for (int i = 0; i < 6; i++) uc[i] = X.l[G::O_U + N + i];
      cube_integrate<R>(cs, uc, X.P);
#pragma unroll
      for (int i = 0; i < 3; i++) { X.l[G::O_CS + i] = cs.cube.p[i]; X.l[G::O_CS + 7 + i] = cs.cube.v[i]; X.l[G::O_CS + 10 + i] = cs.cube.w[i]; }
#pragma unroll
      for (int i = 0; i < 4; i++) X.l[G::O_CS + 3 + i] = cs.cube.q[i];
    }
  }
  (void)s;
}
// the env's state record between registers and its LDS copy (front path)
template <class R, int T>
PBG_DEV void gang_put_state(const State<R>& s, const GangCtx<R>& X) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
  if (X.t == 0) {
#pragma unroll
    for (int d = 0; d < R::NJ; d++) { X.l[G::O_Q + d] = s.q[d]; X.l[G::O_QD + d] = s.qd[d]; }
#pragma unroll
    for (int i = 0; i < 3; i++) { X.l[G::O_BS + i] = s.bp[i]; X.l[G::O_BS + 7 + i] = s.bv[i]; X.l[G::O_BS + 10 + i] = s.bw[i]; }
#pragma unroll
    for (int i = 0; i < 4; i++) X.l[G::O_BS + 3 + i] = s.bq[i];
    if constexpr (R::harder) {
#pragma unroll
      for (int i = 0; i < 3; i++) { X.l[G::O_CS + i] = s.cube.p[i]; X.l[G::O_CS + 7 + i] = s.cube.v[i]; X.l[G::O_CS + 10 + i] = s.cube.w[i]; }
#pragma unroll
      for (int i = 0; i < 4; i++) X.l[G::O_CS + 3 + i] = s.cube.q[i];
    }
  }
}
template <class R, int T>
PBG_DEV void gang_get_state(State<R>& s, const GangCtx<R>& X) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using G = Gang<R, T>;
#pragma unroll
  for (int d = 0; d < R::NJ; d++) { s.q[d] = X.l[G::O_Q + d]; s.qd[d] = X.l[G::O_QD + d]; }
#pragma unroll
  for (int i = 0; i < 3; i++) { s.bp[i] = X.l[G::O_BS + i]; s.bv[i] = X.l[G::O_BS + 7 + i]; s.bw[i] = X.l[G::O_BS + 10 + i]; }
#pragma unroll
  for (int i = 0; i < 4; i++) s.bq[i] = X.l[G::O_BS + 3 + i];
  if constexpr (R::harder) {
#pragma unroll
    for (int i = 0; i < 3; i++) { s.cube.p[i] = X.l[G::O_CS + i]; s.cube.v[i] = X.l[G::O_CS + 7 + i]; s.cube.w[i] = X.l[G::O_CS + 10 + i]; }
#pragma unroll
    for (int i = 0; i < 4; i++) s.cube.q[i] = X.l[G::O_CS + 3 + i];
  }
}

// HumanoidFlagrunHarder: the rows of the cube's corner contacts with the floor, one row per lane.
// Their Jacobian has only the cube's 6 columns, so the robot's part of y = L^-1 J^T is exactly zero:
// no Jacobian over the robot's dofs and no forward substitution, only the cube's
// (nd / sqrt m | (r x nd) / sqrt I).  The row is stored in the sliced layout of every row (the PGS
// reads it unchanged), with the same arithmetic as the general rows pass, bit for bit (that pass
// added exact zeros for the robot's part).
template <class R, int T>
PBG_DEV void cube_floor_rows(const GangCtx<R>& X, int nr, int ncf, const SimPT<real_t<R>>& P) {
  using Sc = real_t<R>;
  using G = Gang<R, T>;
#pragma unroll 1
  for (int j = X.t; wave_any(j < 3 * ncf); j += T) {
    if (j >= 3 * ncf) continue;
    const int c = nr + j / 3, dir = j % 3;
    V3<Sc> rA;
    Sc dist = 0.f;
    contact_at<R, T>(X, c, [&](auto p) { rA = mk3<Sc>(p[0], p[1], p[2]); dist = p[9]; });
    // the floor's normal and btPlaneSpace1 basis
    const V3<Sc> nd = dir == 0 ? mk3<Sc>(0, 0, 1) : (dir == 1 ? mk3<Sc>(0, -1, 0) : mk3<Sc>(1, 0, 0));
    const V3<Sc> mc = cross3(rA, nd);
    const Sc rm = Sc(1) / CubeK<Sc>::sm(), rI = Sc(1) / CubeK<Sc>::sI();
    const V3<Sc> ycl = Sc(1) * rm * nd, cubes = Sc(1) * rI * mc;
    const Sc D2 = dot3(ycl, ycl) + dot3(cubes, cubes);
    const Sc meff = D2 > Sc(1e-12) ? fast_rcp(D2) : 0.f;
    const Sc tgt = dir == 0 ? (pos_target(dist, P.k_contact, P.k_sep)) : 0.f;
    contact_at<R, T>(X, c, [&](auto p0) {
      auto p = p0 + G::RW0 + dir * G::CRW;
      const Sc yc[6] = {ycl.x, ycl.y, ycl.z, cubes.x, cubes.y, cubes.z};
#pragma unroll
      for (int i = 0; i < G::YS; i++) p[G::yw(i)] = i >= G::N && i < G::NY ? yc[i - G::N] : Sc(0);
      p[G::YS] = meff;
      p[G::YS + 1] = tgt;
      p[G::YS + 2] = 0.f;
    });
  }
}

// ------------------------------------------------------------------ one physics sub-step
template <class R, int T, bool DIST>
PBG_DEV int gang_substep(State<R>& s, const real_t<R>* tau, const GangCtx<R>& X, uint64_t& slot_bits, uint32_t sub,
                         uint32_t& csig SUB_STAMP_ARGS) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  using D = Dims<R>;
  using G = Gang<R, T>;
  auto& TB = GangTabs<R>::tab(X.tabs);
  constexpr int N = R::NDOF, NB = D::NB, NLIM = D::NLIM, NSL = G::NSL, YS = G::YS;
  const SimPT<Sc>& P = X.P;
  const bool w0 = X.t == 0;  // the gang's writer for replicated values
  // L (Dims<R>::lidx order) into the factor's LDS word order (pbg_fronts.h)
  auto stage_solution = [&](const Sc* L, const Sc* Ld, const Sc* u) {
    if (w0) {
      static_for<0, N>([&](auto i_c) {
        constexpr int i = decltype(i_c)::value;
        static_for<0, i + 1>([&](auto k_c) {
          constexpr int k = decltype(k_c)::value;
          if constexpr (D::coupled(i, k)) X.l[G::O_L + FP<R>::idx(i, k)] = L[D::lidx(i, k)];
        });
      });
#pragma unroll
      for (int i = 0; i < N; i++) { X.l[G::O_LD + i] = Ld[i]; X.l[G::O_U + i] = u[i]; }
#pragma unroll
      for (int i = N; i < YS; i++) X.l[G::O_U + i] = 0.f;
      static_for<0, NLIM>([&](auto li_c) {
        constexpr int li = decltype(li_c)::value;
        constexpr int d = D::LIM.v[li][0];
        X.l[G::O_LP + 2 * li] = s.q[d] - (Sc)R::dof_lower[d];
        X.l[G::O_LP + 2 * li + 1] = (Sc)R::dof_upper[d] - s.q[d];
      });
    }
  };
  // the replicated path keeps its factor in registers from the factorisation through the rows pass
  // (the distributed path loads it from its LDS staging before the rows pass)
  Sc Lr[G::NNZ4], Ldr[G::N4];
  if constexpr (DIST) {
    // --- distributed dynamics (M, rhs, frames, motion vectors in LDS) ----------------------
#ifndef PBG_DEV_NODYN
    gang_dyn_mass<R, T>(s, X SUB_STAMP_PASS);
#endif
    STAMP(3)
  } else {
    // --- replicated dynamics (compile-time folded; short trees), staged into LDS ---------
    {
      Sc nu[N], u[N];
      dynamics<R>(s, tau, Lr, Ldr, nu, u, P SUB_STAMP_PASS);
      STAMP(3)
      stage_solution(Lr, Ldr, u);
    }
    Kin<R> k;
    V3<Sc> sw[N], sv[N], O0;
    kin_motion<R>(s, k, sw, sv, O0);
    if (w0) {
#pragma unroll
      for (int i = 0; i < N; i++) {
        X.l[G::O_SW + G::SS * i] = sw[i].x; X.l[G::O_SW + G::SS * i + 1] = sw[i].y; X.l[G::O_SW + G::SS * i + 2] = sw[i].z;
        X.l[G::O_SV + G::SS * i] = sv[i].x; X.l[G::O_SV + G::SS * i + 1] = sv[i].y; X.l[G::O_SV + G::SS * i + 2] = sv[i].z;
      }
#pragma unroll
      for (int b = 0; b < D::NB; b++) {
        LW* p = body_word<R, T>(X.l, b, 0);
#pragma unroll
        for (int i = 0; i < 9; i++) p[i] = k.Rm[b].m[i];
        p[9] = k.x[b].x; p[10] = k.x[b].y; p[11] = k.x[b].z;
        LW* pk = body_word<R, T>(X.l, b, G::FW);
        pk[0] = k.c[b].x; pk[1] = k.c[b].y; pk[2] = k.c[b].z;
      }
    }
  }
  PBG_GANG_SYNC
  const V3<Sc> O = gang_O<R, T>(X);
  PBG_GANG_SYNC
  STAMP(10)
  auto frame = [&](int b, M3<Sc>& Rm, V3<Sc>& x) {
    const LW* p = body_word<R, T>(X.l, b, 0);
#pragma unroll
    for (int i = 0; i < 9; i++) Rm.m[i] = p[i];
    x = mk3<Sc>(p[9], p[10], p[11]);
  };
  // descriptor: rA | rB | n | dist | fA (body A carries the base dofs) | fB (body B does) | chain masks of
  // A and B | floor | cube (+1: A is HumanoidFlagrunHarder's cube, -1: B is, 0: no cube; its lever
  // arm from the cube's centre is then rA, resp. rB)
  auto put_desc = [&](int c, V3<Sc> rA, V3<Sc> rB, V3<Sc> n, Sc dist, Sc fB, uint32_t mA, uint32_t mB, Sc floor_, Sc mu,
                      Sc fA = 1.f, Sc cube = 0.f) {
    const Sc v[G::DW] = {rA.x, rA.y, rA.z, rB.x, rB.y, rB.z, n.x, n.y, n.z, dist, fA, fB,
                            mask_word<Sc>(mA), mask_word<Sc>(mB), floor_, cube};
    contact_at<R, T>(X, c, [&](auto p) {
#pragma unroll
      for (int w = 0; w < G::DW; w++) p[w] = v[w];
      p[G::DW] = mu;
    });
  };
  const uint64_t gang_mask = ((T == 64) ? ~0ull : ((1ull << T) - 1ull)) << (X.le * T);
  const uint64_t below = (1ull << (X.le * T + X.t)) - 1ull;
  int nc = 0;
  // HumanoidFlagrunHarder: contacts [nr, nr + ncf) are the cube's corners on the floor (their rows:
  // cube_floor_rows); the robot's floor / self contacts come before them, the robot-cube ones after
  int nr = 0, ncf = 0;
  // --- distributed: capsule ends of the self-collision geoms in world coordinates, one geom
  // per lane, in the limit-row area (dead until the rows pass); read by the pair pass ------
  constexpr int O_GE = G::O_LR;
  static_assert(R::NPAIR == 0 || 6 * R::NG <= G::LRSZ, "geom ends exceed the limit-row area");
  if constexpr (R::NPAIR > 0) {
    static_for<0, (R::NG + T - 1) / T>([&](auto r_c) {
      const int g = decltype(r_c)::value * T + X.t;
      if (g < R::NG) {
        M3<Sc> Rm; V3<Sc> x;
        frame(TB.geom_body[g], Rm, x);
        const V3<Sc> e0 = x + mul(Rm, mk3<Sc>(TB.gp0[g][0], TB.gp0[g][1], TB.gp0[g][2]));
        const V3<Sc> e1 = x + mul(Rm, mk3<Sc>(TB.gp1[g][0], TB.gp1[g][1], TB.gp1[g][2]));
        LW* e = X.l + O_GE + 6 * g;
        e[0] = e0.x; e[1] = e0.y; e[2] = e0.z; e[3] = e1.x; e[4] = e1.y; e[5] = e1.z;
      }
    });
  }
  // --- distributed: floor slots (slot order) ---------------------------------------------
  uint64_t sb = 0;
  // ST: the slot table in the workgroup's LDS copy, or (gang_big) the __constant__ table
  auto slot_pass = [&](const auto& ST) {
  static_for<0, G::ROUNDS_S>([&](auto r_c) {
    constexpr int r = decltype(r_c)::value;
    const int sl = r * T + X.t;
    bool act = false;
    V3<Sc> cc;
    Sc rad = 0.f;
    if (sl < R::NS) {
      M3<Sc> Rm; V3<Sc> x;
      frame(ST.slot_body[sl], Rm, x);
      cc = x + mul(Rm, mk3<Sc>(ST.slot[sl][0], ST.slot[sl][1], ST.slot[sl][2]));
      rad = ST.slot[sl][3];
      act = cc.z - rad < (Sc)PBG_CONTACT_THRESHOLD;
    }
    const uint64_t bal = __ballot(act);
    const uint64_t mine = bal & gang_mask;
    if constexpr (r * T < 64) sb |= (mine >> (X.le * T)) << (r * T);  // the feet's slots come first
    if (act) {
      csig += pbg_contact_hash(sub, (uint32_t)sl);  // this lane's share of the signature
      const int c = nc + __popcll(bal & gang_mask & below);
      const V3<Sc> cp = mk3<Sc>(cc.x, cc.y, cc.z - rad);
      put_desc(c, cp - O, mk3<Sc>(0, 0, 0), mk3<Sc>(0, 0, 1), cc.z - rad, 0.f, TB.chain[ST.slot_body[sl]], 0u, 1.f, ST.slot_mu[sl]);
    }
    nc += __popcll(mine);
  });
  };
  if constexpr (gang_big<R>()) slot_pass(g_gang_tab<R>);
  else slot_pass(TB);
  slot_bits = sb;
  // --- distributed: self-collision pairs (pair order) ------------------------------------
  if constexpr (R::NPAIR > 0) {
    PBG_GANG_SYNC  // the geom ends
#pragma unroll
    for (int r = 0; r < (R::NPAIR + T - 1) / T; r++) {  // rounds unrolled: their loads overlap
      const int pp = r * T + X.t;
      bool act = false;
      V3<Sc> PA, PB, nrm;
      Sc dist = 0.f;
      int ga = 0, gb = 0;
      if (pp < R::NPAIR) {
        ga = TB.pga[pp]; gb = TB.pgb[pp];
        const LW* ea = X.l + O_GE + 6 * ga;
        const LW* eb = X.l + O_GE + 6 * gb;
        const V3<Sc> a0 = mk3<Sc>(ea[0], ea[1], ea[2]), a1 = mk3<Sc>(ea[3], ea[4], ea[5]);
        const V3<Sc> b0 = mk3<Sc>(eb[0], eb[1], eb[2]), b1 = mk3<Sc>(eb[3], eb[4], eb[5]);
        const V3<Sc> dc = (a0 + a1) - (b0 + b1);
        if (dot3(dc, dc) <= TB.pbound2[pp]) {
          // closest points of two segments (same branch structure as the lane kernel)
          const V3<Sc> d1 = a1 - a0, d2 = b1 - b0, r0 = a0 - b0;
          const Sc aa = dot3(d1, d1), ee = dot3(d2, d2), ff = dot3(d2, r0);
          Sc ss, tt;
          const Sc eps = Sc(1e-12);
          if (aa <= eps && ee <= eps) { ss = tt = 0.f; }
          else if (aa <= eps) { ss = 0.f; tt = tmin(tmax(ff / ee, 0.f), 1.f); }
          else {
            const Sc cc2 = dot3(d1, r0);
            if (ee <= eps) { tt = 0.f; ss = tmin(tmax(-cc2 / aa, 0.f), 1.f); }
            else {
              const Sc bb2 = dot3(d1, d2), den = aa * ee - bb2 * bb2;
              ss = den > eps ? tmin(tmax((bb2 * ff - cc2 * ee) / den, 0.f), 1.f) : 0.f;
              tt = (bb2 * ss + ff) / ee;
              if (tt < 0.f) { tt = 0.f; ss = tmin(tmax(-cc2 / aa, 0.f), 1.f); }
              else if (tt > 1.f) { tt = 1.f; ss = tmin(tmax((bb2 - cc2) / aa, 0.f), 1.f); }
            }
          }
          const V3<Sc> ca = a0 + ss * d1, cb = b0 + tt * d2;
          const V3<Sc> dv = ca - cb;
          const Sc dd = norm3(dv);
          const Sc ra = TB.gp0[ga][3], rb = TB.gp0[gb][3];
          dist = dd - ra - rb;
          act = dist < (Sc)PBG_CONTACT_THRESHOLD;
          nrm = dd > Sc(1e-9) ? fast_rcp(dd) * dv : mk3<Sc>(0, 0, 1);
          PA = ca - ra * nrm;
          PB = cb + rb * nrm;
        }
      }
      const uint64_t bal = __ballot(act);
      if (act) {
        csig += pbg_contact_hash(sub, (uint32_t)(R::NS + pp));
        const int c = nc + __popcll(bal & gang_mask & below);
        put_desc(c, PA - O, PB - O, nrm, dist, 1.f, TB.chain[TB.geom_body[ga]], TB.chain[TB.geom_body[gb]], 0.f, TB.pmu[pp]);
      }
      nc += __popcll(bal & gang_mask);
    }
  }
  // --- distributed: HumanoidFlagrunHarder's cube -- its 8 corners vs the floor, then every robot
  // collision geom vs the box (oracle detect_cube_contacts / the lane kernel's cube_contacts), one
  // candidate per lane, compacted in candidate order ------------------------------------------
  if constexpr (R::harder) {
    constexpr int NCC = 8 + R::NCG;
    const Sc h = (Sc)PBG_CUBE_HALF, thr = (Sc)PBG_CONTACT_THRESHOLD;
    const M3<Sc> Rc = quat_to_m3(X.l[G::O_CS + 3], X.l[G::O_CS + 4], X.l[G::O_CS + 5], X.l[G::O_CS + 6]);
    const V3<Sc> xc = mk3<Sc>(X.l[G::O_CS], X.l[G::O_CS + 1], X.l[G::O_CS + 2]);
    static_assert(T >= 8, "the corners are the first round's lanes");
    nr = nc;
#pragma unroll
    for (int r = 0; r < (NCC + T - 1) / T; r++) {
      const int k = r * T + X.t;
      bool act = false;
      V3<Sc> rA, rB, nrm;
      Sc dist = 0.f, mu = 0.f, fA = 1.f, cube = 0.f, flo = 0.f;
      uint32_t mA = 0u;
      if (k < 8) {  // corner k vs the floor: A = the cube, normal +z
        const V3<Sc> lc = mk3<Sc>((k & 1) ? h : -h, (k & 2) ? h : -h, (k & 4) ? h : -h);
        const V3<Sc> pp = xc + mul(Rc, lc);
        act = pp.z < thr;
        rA = pp - xc; rB = mk3<Sc>(0, 0, 0); nrm = mk3<Sc>(0, 0, 1);
        dist = pp.z; mu = (Sc)R::cube_floor_mu; fA = 0.f; cube = 1.f; flo = 1.f;
      } else if (k < NCC) {  // robot geom g vs the box: A = the robot link, B = the cube
        const int g = k - 8;
        int lnk = 0;
        Sc gp0[3], gp1[3], rr = 0.f, gmu = 0.f;
        static_for<0, R::NCG>([&](auto g_c) {  // the geom's constants by selects (no table loads)
          constexpr int gg = decltype(g_c)::value;
          if (g == gg) {
            lnk = R::cgeom_link[gg];
#pragma unroll
            for (int i = 0; i < 3; i++) { gp0[i] = (Sc)R::cgeom_p0[gg][i]; gp1[i] = (Sc)R::cgeom_p1[gg][i]; }
            rr = (Sc)R::cgeom_r[gg];
            gmu = (Sc)R::cgeom_mu[gg];
          }
        });
        M3<Sc> Rm; V3<Sc> x;
        frame(lnk + 1, Rm, x);
        const V3<Sc> e0 = x + mul(Rm, mk3<Sc>(gp0[0], gp0[1], gp0[2])), e1 = x + mul(Rm, mk3<Sc>(gp1[0], gp1[1], gp1[2]));
        M3<Sc> Rt;
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
          for (int j = 0; j < 3; j++) Rt.m[3 * i + j] = Rc.m[3 * j + i];
        const V3<Sc> p0 = mul(Rt, e0 - xc), p1 = mul(Rt, e1 - xc), d = p1 - p0;
        const Sc dd = dot3(d, d);
        const Sc t0 = dd > Sc(1e-12) ? tmin(tmax(-dot3(p0, d) / dd, 0.f), 1.f) : 0.f;
        const Sc bound = (Sc)(1.7320508075688772 * PBG_CUBE_HALF);  // circumradius
        if (norm3(p0 + t0 * d) < bound + rr + thr) {
          Sc t = 0.f;
          if (dd > Sc(1e-12)) {  // golden-section minimisation of the box's signed distance along the segment
            const Sc phi = Sc(0.6180339887498949);
            Sc a = 0.f, bb = 1.f;
            Sc x1 = bb - phi * (bb - a), x2 = a + phi * (bb - a);
            Sc f1 = box_sd(p0 + x1 * d, h), f2 = box_sd(p0 + x2 * d, h);
#pragma unroll 1
            for (int it = 0; it < PBG_CUBE_GS_ITERS; it++) {
              if (f1 <= f2) { bb = x2; x2 = x1; f2 = f1; x1 = bb - phi * (bb - a); f1 = box_sd(p0 + x1 * d, h); }
              else { a = x1; x1 = x2; f1 = f2; x2 = a + phi * (bb - a); f2 = box_sd(p0 + x2 * d, h); }
            }
            t = 0.5f * (a + bb);
          }
          const V3<Sc> ps = p0 + t * d;
          dist = box_sd(ps, h) - rr;
          act = dist < thr;
          V3<Sc> nb, qb;
          const Sc qx = tabs(ps.x) - h, qy = tabs(ps.y) - h, qz = tabs(ps.z) - h;
          if (tmax(qx, tmax(qy, qz)) > 0.f) {
            qb = mk3<Sc>(tmin(tmax(ps.x, -h), h), tmin(tmax(ps.y, -h), h), tmin(tmax(ps.z, -h), h));
            const V3<Sc> dv = ps - qb;
            const Sc l = norm3(dv);
            nb = l > Sc(1e-9) ? (1.f / l) * dv : mk3<Sc>(0, 0, 1);
          } else {
            const int ax = (qx >= qy && qx >= qz) ? 0 : (qy >= qz ? 1 : 2);
            const Sc cc = ax == 0 ? ps.x : (ax == 1 ? ps.y : ps.z);
            const Sc sg = cc < 0.f ? -1.f : 1.f;
            nb = mk3<Sc>(ax == 0 ? sg : 0.f, ax == 1 ? sg : 0.f, ax == 2 ? sg : 0.f);
            qb = mk3<Sc>(ax == 0 ? sg * h : ps.x, ax == 1 ? sg * h : ps.y, ax == 2 ? sg * h : ps.z);
          }
          nrm = mul(Rc, nb);
          const V3<Sc> PA = xc + mul(Rc, ps) - rr * nrm, PB = xc + mul(Rc, qb);
          rA = PA - O; rB = PB - xc;
          mu = gmu; cube = -1.f;
          mA = lnk >= 0 ? TB.chain[lnk + 1] : 0u;
        }
      }
      const uint64_t bal = __ballot(act);
      if (r == 0) ncf = __popcll(bal & gang_mask & (0xFFull << (X.le * T)));
      if (act) {
        csig += pbg_contact_hash(sub, (uint32_t)(R::NS + R::NPAIR + k));
        const int c = nc + __popcll(bal & gang_mask & below);
        put_desc(c, rA, rB, nrm, dist, 0.f, mA, 0u, flo, mu, fA, cube);
      }
      nc += __popcll(bal & gang_mask);
    }
  }
  PBG_GANG_SYNC
  STAMP(4)
  if constexpr (DIST) {
    if constexpr (FP<R>::NF > 0) {
      // --- front-parallel factorisation and unconstrained velocity (pbg_fronts.h) -----------
      gang_front_solve<R, T>(s, X);
    } else {
      // --- replicated: factorisation and the unconstrained velocity, staged for the PGS ----
      // (the factor stays in Lr / Ldr for the rows pass: no reload from LDS)
      Sc rhs[N], nu[N], u[N];
#pragma unroll
      for (int i = 0; i < D::NNZ; i++) Lr[i] = X.l[G::O_L + i];
#pragma unroll
      for (int i = 0; i < N; i++) rhs[i] = X.l[G::O_RHS + i];
      dyn_solve<R>(s, Lr, rhs, Ldr, nu, u, P);
      stage_solution(Lr, Ldr, u);
    }
    PBG_GANG_SYNC
    STAMP(10)
  }
  // --- distributed: constraint rows (limits first, then 3 rows per contact) --------------
#ifdef PBG_DEV_NOROWS
  const int njobs = 0;
#else
  // (HumanoidFlagrunHarder: the cube's floor contacts are built by cube_floor_rows below)
  const int njobs = NLIM + G::NRC * (nc - ncf);
#endif
  // the front path holds its staged factor in registers for the rows pass unless it is too big to
  // (Atlas: the register copy spilled 1.2 KB per lane; its rows read the LDS words instead) or the
  // gang is 32 lanes wide (two waves per SIMD, 256 registers: 148 -> 12 bytes of spills, Humanoid
  // -1.2 %, FlagrunHarder -13 % on 32-lane gangs; r04_ab_gang32_lds_factor.txt)
  constexpr bool LREG = !DIST || FP<R>::NF == 0 || (T == 16 && G::NNZ4 + G::N4 <= 240);
  if constexpr (DIST && FP<R>::NF > 0 && LREG) gang_load_factor<R, T>(X, Lr, Ldr);
#pragma unroll 1
  for (int j = X.t; wave_any(j < njobs); j += T) {
    if (j >= njobs) continue;
    Sc J[N];
    const bool is_lim = j < NLIM;
    int c = 0, dir = 0;
    Sc dist = 0.f;
    Sc cubef = 0.f;            // HumanoidFlagrunHarder: the contact's cube side (descriptor word 15)
    V3<Sc> ycl = mk3<Sc>(0, 0, 0), cubes = mk3<Sc>(0, 0, 0);  // and the cube part of y (linear | angular)
    if (is_lim) {
      const int g = TB.lim_g[j];
#pragma unroll
      for (int i = 0; i < N; i++) J[i] = i == g ? 1.f : 0.f;
    } else {
      c = (j - NLIM) / G::NRC;
      dir = (j - NLIM) - G::NRC * c;
      if constexpr (R::harder) c += c >= nr ? ncf : 0;
      Sc v[G::DW];
      contact_at<R, T>(X, c, [&](auto p) {
#pragma unroll
        for (int w = 0; w < G::DW; w++) v[w] = p[w];
      });
      const V3<Sc> rA = mk3<Sc>(v[0], v[1], v[2]), rB = mk3<Sc>(v[3], v[4], v[5]), nrm = mk3<Sc>(v[6], v[7], v[8]);
      dist = v[9];
      const Sc fB = v[11];
      const uint32_t mA = word_mask(v[12]), mB = word_mask(v[13]);
      V3<Sc> t1, t2;  // btPlaneSpace1(nrm); the floor's (+z) gives (0,-1,0), (1,0,0)
      if (v[14] != 0.f) { t1 = mk3<Sc>(0, -1, 0); t2 = mk3<Sc>(1, 0, 0); }
      else if (tabs(nrm.z) > Sc(0.7071067811865476)) {
        const Sc a2 = nrm.y * nrm.y + nrm.z * nrm.z, kinv = fast_rsq(a2);
        t1 = mk3<Sc>(0, -nrm.z * kinv, nrm.y * kinv);
        t2 = mk3<Sc>(a2 * kinv, -nrm.x * t1.z, nrm.x * t1.y);
      } else {
        const Sc a2 = nrm.x * nrm.x + nrm.y * nrm.y, kinv = fast_rsq(a2);
        t1 = mk3<Sc>(-nrm.y * kinv, nrm.x * kinv, 0);
        t2 = mk3<Sc>(-nrm.z * t1.y, nrm.z * t1.x, a2 * kinv);
      }
      // rows 3-5 (NRC = 6): spinning about n, rolling about t1, t2 -- angular Jacobians
      const int ax = G::NRC == 6 && dir >= 3 ? dir - 3 : dir;
      const V3<Sc> nd = ax == 0 ? nrm : (ax == 1 ? t1 : t2);
      const V3<Sc> mmA = cross3(rA, nd), mmB = cross3(rB, nd);
      cubef = v[15];
      cubes = mk3<Sc>(0, 0, 0);
      if constexpr (R::harder) {  // the cube's columns: +-(nd / sqrt m, (r x nd) / sqrt I), r its lever arm
        const V3<Sc> rc = cubef > 0.f ? rA : rB;
        const V3<Sc> mc = cross3(rc, nd);
        const Sc rm = Sc(1) / CubeK<Sc>::sm(), rI = Sc(1) / CubeK<Sc>::sI();
        ycl = cubef * rm * nd;
        cubes = cubef * rI * mc;
      }
      const Sc fA = v[10];
#pragma unroll
      for (int i = 0; i < N; i++) {
        const int di = D::dof_of(i);
        const bool inA = di < 0 ? fA != 0.f : ((mA >> di) & 1u) != 0u, inB = di < 0 ? fB != 0.f : ((mB >> di) & 1u) != 0u;
        const V3<Sc> sw = mk3<Sc>(X.l[G::O_SW + G::SS * i], X.l[G::O_SW + G::SS * i + 1], X.l[G::O_SW + G::SS * i + 2]);
        const V3<Sc> sv = mk3<Sc>(X.l[G::O_SV + G::SS * i], X.l[G::O_SV + G::SS * i + 1], X.l[G::O_SV + G::SS * i + 2]);
        Sc tj = 0.f;
        if (G::NRC == 6 && dir >= 3) {
          if (inA) tj += dot3(nd, sw);
          if (inB) tj -= dot3(nd, sw);
        } else {
          if (inA) tj += dot3(nd, sv) + dot3(mmA, sw);
          if (inB) tj -= dot3(nd, sv) + dot3(mmB, sw);
        }
        J[i] = tj;
      }
    }
    // y = L^-1 J (forward substitution over the compile-time pattern of L, held in registers for
    // the pass: 16-byte loads of the staged factor before the job loop)
    Sc y[N];
    Sc D2 = 0.f;
#pragma unroll
    for (int i = 0; i < N; i++) {
      Sc tt = J[i];
#pragma unroll
      for (int kk = 0; kk < i; kk++)
        if (D::coupled(i, kk)) tt -= (LREG ? Lr[DIST ? FP<R>::idx(i, kk) : D::lidx(i, kk)] : X.l[G::O_L + FP<R>::idx(i, kk)]) * y[kk];
      y[i] = tt * (LREG ? Ldr[i] : X.l[G::O_LD + i]);
      D2 += y[i] * y[i];
    }
    if constexpr (R::harder) D2 += dot3(ycl, ycl) + dot3(cubes, cubes);
    const Sc meff = D2 > Sc(1e-12) ? fast_rcp(D2) : 0.f;
    if (is_lim) {
      const Sc plo = X.l[G::O_LP + 2 * j], phi = X.l[G::O_LP + 2 * j + 1];
      limit_at<R, T>(X, j, [&](auto p) {
#pragma unroll
        for (int i = 0; i < YS; i++) p[i] = i < N ? y[i] : 0.f;
        p[YS] = meff;
        p[YS + 1] = pos_target(plo, P.k_limit, P.k_sep);
        p[YS + 2] = pos_target(phi, P.k_limit, P.k_sep);
      });
    } else {
      const int w0r = G::RW0 + dir * G::CRW;
      Sc tgt = dir == 0 ? (pos_target(dist, P.k_contact, P.k_sep)) : 0.f;
      if constexpr (R::restitution > 0.0) {
        // restitution (sim_params.h): e (-v_n) when |v_n| >= the threshold, v_n = J nu = y.u before the solve
        static_assert(R::NPAIR == 0 && !R::harder, "restitution: robot-floor contacts only");
        if (dir == 0) {
          Sc vn = 0.f;
#pragma unroll
          for (int i = 0; i < N; i++) vn += y[i] * X.l[G::O_U + i];
          const Sc rest = tabs(vn) < Sc(PBG_RESTITUTION_VELOCITY_THRESHOLD) ? Sc(0) : Sc(R::restitution) * -vn;
          tgt += rest > Sc(0) ? rest : Sc(0);
        }
      }
      contact_at<R, T>(X, c, [&](auto p0) {
        auto p = p0 + w0r;
        const Sc yc[6] = {ycl.x, ycl.y, ycl.z, cubes.x, cubes.y, cubes.z};
#pragma unroll
        for (int i = 0; i < YS; i++) p[G::yw(i)] = i < N ? y[i] : (i < G::NY ? yc[(i - N) % 6] : 0.f);
        p[YS] = meff;
        p[YS + 1] = tgt;
        p[YS + 2] = 0.f;
      });
    }
  }
  if constexpr (R::harder) cube_floor_rows<R, T>(X, nr, ncf, P);
  PBG_GANG_SYNC
  STAMP(11)
  // --- PGS: 5 sweeps, Bullet order (scene_bases.py:65 numSolverIterations=5) -------------
  Sc us[NSL];
#pragma unroll
  for (int m = 0; m < NSL; m++) us[m] = X.l[G::O_U + X.t + m * T];
  {
    // joint-limit rows stay in registers for the whole solve
#ifdef PBG_DEV_NOLIM
    constexpr int NLIM = 0;
#endif
    constexpr int NL1 = NLIM > 0 ? NLIM : 1;
    Sc ly[NL1][NSL], lm[NL1], lrm[NL1], ltl[NL1], lth[NL1], llo[NL1], lhi[NL1];
#pragma unroll
    for (int li = 0; li < NLIM; li++) {
      limit_at<R, T>(X, li, [&](auto p) {
#pragma unroll
        for (int m = 0; m < NSL; m++) ly[li][m] = p[X.t + m * T];
        lm[li] = p[YS]; ltl[li] = p[YS + 1]; lth[li] = p[YS + 2];
      });
      lrm[li] = lm[li] > 0.f ? fast_rcp(lm[li]) : 0.f;  // off the sweeps' dependency chain
      llo[li] = 0.f; lhi[li] = 0.f;
    }
    const bool all_lds = !wave_any(nc > X.cap);  // every contact row of the wave in LDS
    constexpr int NWF = (G::MAXC + 31) / 32;
    const bool few = NWF == 1 || !wave_any(nc > 32);  // a one-word positive-impulse mask suffices
    for (int it = 0; it < P.iterations; it++) {
#pragma unroll
      for (int li = 0; li < NLIM; li++) {
        Sc part = 0.f;
#pragma unroll
        for (int m = 0; m < NSL; m++) part += ly[li][m] * us[m];
        const Sc yu = gang_sum<T>(part);
        const Sc meff = lm[li];
        const Sc nlo = clampf(llo[li] + meff * (ltl[li] - yu), 0.f, (Sc)PBG_LIMIT_MAX_IMPULSE);
        const Sc dlo = nlo - llo[li];
        // upper row sees u after the lower update: (-y).u' = -(yu + dlo / meff)
        // lrm = 0 when meff = 0: no select on the chain (Atlas keeps it: without it the allocator
        // spilled 48 bytes of its 512 registers)
        const Sc yu2 = G::NSL > 2 && !(meff > 0.f) ? yu : yu + dlo * lrm[li];
        const Sc nhi = clampf(lhi[li] + meff * (lth[li] + yu2), 0.f, (Sc)PBG_LIMIT_MAX_IMPULSE);
        const Sc dhi = nhi - lhi[li];
        llo[li] = nlo;
        lhi[li] = nhi;
        const Sc dl = dlo - dhi;
#pragma unroll
        for (int m = 0; m < NSL; m++) us[m] += ly[li][m] * dl;
      }
      if (few) {
        if (all_lds) gang_contact_sweep<R, T, true, 1>(X, nc, us);
        else gang_contact_sweep<R, T, false, 1>(X, nc, us);
      } else {
        if (all_lds) gang_contact_sweep<R, T, true, NWF>(X, nc, us);
        else gang_contact_sweep<R, T, false, NWF>(X, nc, us);
      }
    }
  }
  // --- replicated: gather u, back-substitute, integrate ----------------------------------
  STAMP(5)
#pragma unroll
  for (int m = 0; m < NSL; m++) X.l[G::O_U + X.t + m * T] = us[m];
  PBG_GANG_SYNC
  if constexpr (DIST && G::LST) {
    gang_front_integrate<R, T>(s, X);
  } else {
    Sc L[D::NNZ], Ld[N], u[N], nu[N];
    // the staged factor in Dims<R>::lidx order (a compile-time permutation of its LDS words)
    static_for<0, N>([&](auto i_c) {
      constexpr int i = decltype(i_c)::value;
      static_for<0, i + 1>([&](auto k_c) {
        constexpr int k = decltype(k_c)::value;
        if constexpr (D::coupled(i, k)) L[D::lidx(i, k)] = X.l[G::O_L + FP<R>::idx(i, k)];
      });
    });
#pragma unroll
    for (int i = 0; i < N; i++) { Ld[i] = X.l[G::O_LD + i]; u[i] = X.l[G::O_U + i]; }
    integrate<R>(s, L, Ld, u, nu, P);
  }
  PBG_GANG_SYNC  // the next sub-step's staging overwrites this one's LDS
  STAMP(6)
  return nc;
}

// The env's final stores dealt over the gang (state and obs are bitwise identical in every
// lane): lane t writes state words t, t+T, ... ([word][env]) and observation entries t,
// t+T, ... ([env][D]) -- a few full-wave stores instead of one partial store per word from
// lane 0, whose queue of ~100 outstanding stores stalled the wave.
template <class R, int T>
PBG_DEV void gang_store(const State<R>& s, const float (&obs)[R::OBS], real_t<R>* __restrict__ st, int n,
                        float* __restrict__ obs_out, int e, int t) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  constexpr int SW = PBG_STATE_WORDS(R::NJ, R::harder);
  Sc w[SW];  // store_state's word order
#pragma unroll
  for (int i = 0; i < 3; i++) { w[i] = s.bp[i]; w[7 + i] = s.bv[i]; w[10 + i] = s.bw[i]; }
#pragma unroll
  for (int i = 0; i < 4; i++) w[3 + i] = s.bq[i];
#pragma unroll
  for (int d = 0; d < R::NJ; d++) { w[PBG_BASE_WORDS + d] = s.q[d]; w[PBG_BASE_WORDS + R::NJ + d] = s.qd[d]; }
  if constexpr (R::harder) {  // the cube's words after the robot's (sim_params.h)
    constexpr int c0 = PBG_BASE_WORDS + 2 * R::NJ;
#pragma unroll
    for (int i = 0; i < 3; i++) { w[c0 + i] = s.cube.p[i]; w[c0 + 7 + i] = s.cube.v[i]; w[c0 + 10 + i] = s.cube.w[i]; }
#pragma unroll
    for (int i = 0; i < 4; i++) w[c0 + 3 + i] = s.cube.q[i];
  }
  static_for<0, (SW + T - 1) / T>([&](auto m_c) {
    constexpr int m = decltype(m_c)::value;
    const Sc v = lanes_pick<T, m, SW>(w, t);
    if (m * T + t < SW) st[(size_t)(m * T + t) * n + e] = v;
  });
  lanes_store_row<R, T>(obs, obs_out, e, t);
}

template <class R, int T, bool DIST>
__global__ __launch_bounds__((gang_block<R, T>()), (gang_waves_per_simd<R, T>())) void gang_step_kernel(Buffers B, StepIO io, float* __restrict__ scratch, int cap,
                                                       int env_words) {
  using Sc = real_t<R>;
  using LW = lds_t<Sc>;
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  using G = Gang<R, T>;
  using TT = GangTabs<R>;
  constexpr int BLK = gang_block<R, T>();
  constexpr int EPB = BLK / T;  // envs per workgroup
  lds_float* lds = (lds_float*)lds_dyn;  // the model tables (4-byte words), then the env regions
  {
    const uint32_t* src0 = (const uint32_t*)&g_gang_tab<R>;
    const uint32_t* src1 = (const uint32_t*)&g_gang_dyn<R>;
    __attribute__((address_space(3))) uint32_t* dst = (__attribute__((address_space(3))) uint32_t*)lds;
    for (int i = threadIdx.x; i < TT::TAB_COPY; i += BLK) dst[i] = src0[i];
    for (int i = threadIdx.x; i < (int)(sizeof(GangDynTab<R>) / 4); i += BLK) dst[TT::TAB_WORDS + i] = src1[i];
  }
  __syncthreads();
  GangCtx<R> X;
  X.tabs = lds;
  X.t = threadIdx.x % T;
  X.le = threadIdx.x / T;
  const int e = xcd_block() * EPB + X.le;
  if (e >= B.n) return;  // whole gangs only (no workgroup barrier below)
  X.le &= 64 / T - 1;     // gang within the wave (ballot masks)
  // (env_words is a multiple of REGION_ALIGN: saying so lets the compiler prove the 8 / 16-byte
  // alignment of the region's fixed words and use b64 / b128 LDS accesses with offsets instead
  // of ds_read2_b32 pairs, whose 8-bit offsets needed a v_add_u32 for every address)
  X.l = (LW*)(lds + TT::WORDS) + (threadIdx.x / T) * (env_words & ~(G::REGION_ALIGN - 1));
  X.g = (Sc*)scratch + (size_t)e * G::GWORDS;
  X.cap = cap;
#ifdef PBG_DEV_CHECKS
  X.env_words = env_words;
#endif
  X.P = sp_of<R>(B);
  const bool w0 = X.t == 0;
  STAMP_DECL
  State<R> s;
  load_state<R>(s, st_of<R>(B), B.n, e);
  float act[R::NA];
#pragma unroll
  for (int i = 0; i < R::NA; i++) act[i] = io.act[(size_t)e * R::NA + i];
  constexpr bool LST = DIST && G::LST;  // the front path: the state in LDS through the sub-steps
  if constexpr (LST) gang_put_state<R, T>(s, X);
  // apply_action: tau = power * power_coef * clip(a, -1, 1)   (robot_locomotors.py:26-29)
  Sc tau[R::NJ];
#pragma unroll
  for (int d = 0; d < R::NJ; d++) tau[d] = 0.f;
#pragma unroll
  for (int i = 0; i < R::NA; i++) {
    const float c = fminf(fmaxf(act[i], -1.f), 1.f);
    tau[R::act_dof[i]] += (Sc)(R::act_gain[i] * (double)c);
  }
  if (w0) {
#pragma unroll
    for (int d = 0; d < R::NJ; d++) X.l[G::O_TAU + d] = tau[d];
  }
  uint64_t slot_bits = 0;
  int nc = 0;
  uint32_t csig = 0;  // per-lane share; gang-summed below
  STAMP(7)
  for (int sub = 0; sub < X.P.substeps; sub++)
    nc = gang_substep<R, T, DIST>(s, tau, X, slot_bits, (uint32_t)sub, csig SUB_STAMP_PASS);
  if constexpr (LST) {
    gang_get_state<R, T>(s, X);  // (the sub-step ends with a gang sync)
    // the raw action again for the pack (electricity), instead of holding it through the physics
#pragma unroll
    for (int i = 0; i < R::NA; i++) act[i] = io.act[(size_t)e * R::NA + i];
  }
  if (io.ncontact && w0) io.ncontact[e] = nc;
  if (io.csig) {
    const uint32_t sig = gang_sum_u32<T>(csig);
    if (w0) io.csig[e] = sig;
  }
  // the pack's bookkeeping loads after the physics (issued before it: HalfCheetah -0.5 %, Humanoid
  // +1.9 %, Walker2D +1.1 %, Hopper +0.5 % -- round-4 A/B, r04e; round 3 likewise)
  const int el = B.elapsed[e] + 1;
  uint32_t flags = B.flags[e];
  const double pot_old = B.pot[e];
  const Sc z0_old = z0_of<R>(B)[e];
  float obs[R::OBS];
  PackOut po;
  double pot_new = 0.0;
  Flag fl = load_flag<R>(B, e);
  HarderBk hb = load_harder<R>(B, e);
  STAMPX(13)
  if constexpr (R::kind == 1) {
    pendulum_pack<R>(s, obs, po);
  } else if constexpr (R::kind == 2) {
    mujoco_planar_pack_state<R>(s, pot_old, act, obs, po, B.sp.env_dt);
    pot_new = po.potential;
  } else {
    PackIn<R> in;
    in.env_dt = B.sp.env_dt;
#ifdef PBG_DEV_NOPACK
    for (int i = 0; i < R::OBS; i++) obs[i] = 0.f;
    po = PackOut{};
    if (0)
#endif
    gather<R>(s, flags & 1u, in, [&](auto c) { STAMPX(decltype(c)::value) });
    STAMPX(12)
    uint32_t fnew = 0;
    static_assert(feet_slots_below_64<R>(), "a foot slot past the gang kernel's 64-slot contact mask");
#pragma unroll
    for (int f = 0; f < R::NF; f++) {
      uint64_t fm = 0;
#pragma unroll
      for (int sl = 0; sl < (R::NS < 64 ? R::NS : 64); sl++)
        if (R::slot_link[sl] == R::foot_link[f]) fm |= 1ull << sl;
      fnew |= ((slot_bits & fm) ? 1u : 0u) << f;
      in.feet_prev[f] = ((flags >> (8 + f)) & 1u) ? 1.f : 0.f;
    }
    in.feet_new = fnew;
    in.potential_old = pot_old;
    in.initial_z = z0_old;
#ifdef PBG_DEV_NOPACK
    if (0)
#endif
    {
    if constexpr (R::kind == 3) mujoco3d_pack<R>(in, act, obs, po);
    else flag_pack<R, 4>(in, act, obs, po, fl, [&](Flag& f) { flag_draw(B, e, f); }, X.t, R::harder ? &hb : nullptr);
    }
    if constexpr (R::harder) {  // HumanoidFlagrunHarder's _step half (robot_locomotors.py:251-302)
      double pos[3], vel[3];
      if (harder_step<R>(B, e, in, obs, po, hb, pos, vel, nullptr)) {  // resetBasePosition / Velocity
#pragma unroll
        for (int i = 0; i < 3; i++) { s.cube.p[i] = (Sc)pos[i]; s.cube.v[i] = (Sc)vel[i]; s.cube.w[i] = 0.f; }
      }
    }
    pot_new = po.potential;
    flags = (flags & 0xFFu) | (po.feet_out << 8);
  }
  STAMP(8)
  const bool term = po.done;
  const bool trunc = el >= R::max_episode_steps;  // gym TimeLimit (envs/__init__.py max_episode_steps)
  if (w0) {
    io.rew[e] = (float)po.reward;
    if (io.rew64) io.rew64[e] = po.reward;
    if (io.rew_terms) {
#pragma unroll
      for (int i = 0; i < 5; i++) io.rew_terms[(size_t)e * 5 + i] = po.terms[i];
    }
    io.done[e] = term || trunc;
    if (io.trunc) io.trunc[e] = trunc && !term;
  }
  if (io.autoreset && (term || trunc)) {
    if (io.term_obs) lanes_store_row<R, T>(obs, io.term_obs, e, X.t);
    bool has_floor = flags & 1u;
    double pot;
    Sc z0;
    // every lane reads the episode counter (one load instruction) before the writer bumps it
    const uint32_t epi = B.episode[e];
    if (w0) B.episode[e] = epi + 1;
    // the reset's pack deals its transcendentals over the quad as the step's does (the gang's
    // 16 lanes take the branch together): Hopper, Walker2D and HalfCheetah reset often
    reset_env_epi<R, 4>(B, e, s, nullptr, obs, has_floor, pot, z0, epi, fl, R::harder ? &hb : nullptr, X.t);
    if (w0) {
      B.pot[e] = pot;
      z0_of<R>(B)[e] = z0;
      B.elapsed[e] = 0;
      B.flags[e] = has_floor ? 1u : 0u;
    }
  } else if (w0) {
    B.pot[e] = pot_new;
    B.elapsed[e] = el;
    B.flags[e] = flags;
  }
  if (w0) {
    store_flag<R>(B, e, fl);
    if constexpr (R::harder) store_harder<R>(B, e, hb);
  }
  gang_store<R, T>(s, obs, st_of<R>(B), B.n, io.obs, e, X.t);
  STAMP(9)
  STAMP_FLUSH
}

}  // namespace pbg
