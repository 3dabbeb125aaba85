// pbg_fronts.h -- compile-time branch ("front") decomposition of a robot's mass matrix for the
// gang kernel's factorisation and triangular solves (pbg_gang.hip).  Included by pbg_gang.hip.
//
// The generalized velocity is ordered leaf-first (reverse preorder of the joint dofs, base
// last: Dims<R>::gj), so M's Cholesky factor has no fill-in and every subtree's dofs are a
// contiguous range.  The TRUNK is the root path to the deepest branch point -- the links that
// are an ancestor-or-self of some link (or the base) with two or more dof-carrying child
// subtrees -- plus the floating base's 6 coordinates.  Every other dof belongs to a FRONT: a
// maximal dof-carrying subtree hanging off the trunk (Humanoid: two legs of 4 dofs below the
// pelvis and two arms of 3 dofs below the torso; trunk = the 3 abdomen dofs + the base).  In
// that order M is block-arrow shaped:
//
//       [ A_1              C_1^T ]          A_f   front f's own block
//   M = [      ...         ...   ]          C_f   trunk x front coupling (zero rows for the
//       [          A_F     C_F^T ]                trunk dofs that are not the front's ancestors)
//       [ C_1 ... C_F      T     ]          T     the trunk block
//
// so L_f = chol(A_f), W_f = C_f L_f^-T, L_T = chol(T - sum_f W_f W_f^T), and the fronts are
// independent: lane q of a group of FP lanes (FP = 4 or 8 >= F) factors front q, the Schur
// contributions W_f W_f^T are summed over the group by DPP, and the small trunk block is
// factored replicated.  Isomorphic fronts (same size, same internal coupling, same trunk
// coupling -- left / right leg, left / right arm) form one CLASS and run one unrolled code path
// with a per-lane base offset.
//
// The packed factor in LDS is front-major so that a lane addresses its own front with one base
// and compile-time offsets: block f = A_f's coupled lower triangle (row-major, local indices)
// then C_f (front column a major, trunk rows of the front's coupling set), ...; then the trunk
// block's coupled lower triangle.  idx(i, k) maps a coupled generalized pair i >= k to its word.
// Robots without a branch point (Hopper) or with more than 8 fronts keep nf = 0 and the plain
// lower-triangle order (idx == Dims<R>::lidx).
#pragma once

namespace pbg {

constexpr int FRONTS_MAX = 8;
constexpr int FRONT_MIN_DOF = 14;  // generalized coordinates from which a robot takes the front path
constexpr int FRONT_DOF_MAX = 40;

template <class R>
struct FrontPlan {
  static constexpr int N = R::NDOF;
  int nf = 0;                      // fronts (0: no decomposition)
  int fp = 1;                      // lanes per front group (power of two >= nf; 4 or 8)
  int g0[FRONTS_MAX] = {}, n[FRONTS_MAX] = {};  // front f: generalized range g0 .. g0 + n - 1
  int cls[FRONTS_MAX] = {};        // class of front f
  int ncls = 0;
  int crep[FRONTS_MAX] = {};       // representative (first) front of class c
  int nt = 0;                      // trunk size
  int tg[FRONT_DOF_MAX] = {};      // trunk generalized indices, ascending
  bool tcpl[FRONTS_MAX][FRONT_DOF_MAX] = {};  // front f couples with trunk local t
  int off[FRONTS_MAX] = {};        // word offset of front f's block
  int bsz[FRONTS_MAX] = {};        // words in front f's block
  int toff = 0;                    // word offset of the trunk block
  int idx[FRONT_DOF_MAX][FRONT_DOF_MAX] = {};  // word of coupled (i >= k)
  int front_of[FRONT_DOF_MAX] = {};  // generalized index -> front (-1: trunk)
  int tloc[FRONT_DOF_MAX] = {};    // generalized index -> trunk local (-1: front)
};

template <class R>
constexpr bool link_has_dof_subtree(int l) {  // l = -1: the base
  if (l >= 0 && R::link_dof[l] >= 0) return true;
  for (int c = 0; c < R::NL; c++)
    if (R::link_parent[c] == l && link_has_dof_subtree<R>(c)) return true;
  return false;
}
template <class R>
constexpr int dof_children(int l) {
  int k = 0;
  for (int c = 0; c < R::NL; c++)
    if (R::link_parent[c] == l && link_has_dof_subtree<R>(c)) k++;
  return k;
}
// link a (-1 = base) is an ancestor-or-self of link b
template <class R>
constexpr bool link_anc_or_self(int a, int b) {
  if (a == -1) return true;
  while (b >= 0) {
    if (b == a) return true;
    b = R::link_parent[b];
  }
  return false;
}
template <class R>
constexpr bool link_in_trunk(int l) {
  for (int b = -1; b < R::NL; b++)
    if (dof_children<R>(b) >= 2 && link_anc_or_self<R>(l, b)) return true;
  return false;
}

template <class R>
constexpr FrontPlan<R> make_front_plan() {
  using D = Dims<R>;
  constexpr int N = R::NDOF;
  FrontPlan<R> p{};
  for (int i = 0; i < N; i++)
    for (int k = 0; k < N; k++) p.idx[i][k] = D::NNZ;
  bool any_branch = false;
  for (int b = -1; b < R::NL; b++) any_branch = any_branch || dof_children<R>(b) >= 2;
  // fronts: non-trunk dof-carrying children of the base or of trunk links
  int nf = 0;
  // small trees (Walker2D, HalfCheetah: 9 dofs, a 36-entry factor) keep the replicated algebra:
  // there the group sums and the staging cost more than the factorisation they split (round-4
  // A/B: Walker2D +2.6 %, HalfCheetah +1 % on the front path)
  bool ok = any_branch && N <= FRONT_DOF_MAX && N >= FRONT_MIN_DOF;
  for (int c = 0; c < R::NL && ok; c++) {
    const int par = R::link_parent[c];
    if (link_in_trunk<R>(c) || !link_has_dof_subtree<R>(c)) continue;
    if (par != -1 && !link_in_trunk<R>(par)) continue;
    if (nf >= FRONTS_MAX) { ok = false; break; }
    // the subtree's dofs: a contiguous generalized range
    int lo = N, hi = -1;
    for (int d = 0; d < R::NJ; d++)
      if (link_anc_or_self<R>(c, R::dof_link[d])) {
        const int g = D::gj(d);
        lo = g < lo ? g : lo;
        hi = g > hi ? g : hi;
      }
    p.g0[nf] = lo;
    p.n[nf] = hi - lo + 1;
    nf++;
  }
  if (!ok || nf < 2) {  // no decomposition: the plain lower triangle
    for (int i = 0; i < N; i++)
      for (int k = 0; k <= i; k++) p.idx[i][k] = D::lidx(i, k);
    for (int g = 0; g < N; g++) { p.front_of[g] = -1; p.tloc[g] = -1; }
    return p;
  }
  p.nf = nf;
  p.fp = nf <= 4 ? 4 : 8;
  for (int g = 0; g < N; g++) { p.front_of[g] = -1; p.tloc[g] = -1; }
  for (int f = 0; f < nf; f++)
    for (int a = 0; a < p.n[f]; a++) p.front_of[p.g0[f] + a] = f;
  for (int g = 0; g < N; g++)
    if (p.front_of[g] < 0) { p.tloc[g] = p.nt; p.tg[p.nt++] = g; }
  for (int f = 0; f < nf; f++)
    for (int t = 0; t < p.nt; t++) p.tcpl[f][t] = D::coupled(p.tg[t], p.g0[f]);
  // classes
  for (int f = 0; f < nf; f++) {
    int c = -1;
    for (int f2 = 0; f2 < f && c < 0; f2++) {
      bool same = p.n[f2] == p.n[f];
      for (int a = 0; a < p.n[f] && same; a++)
        for (int b = 0; b < p.n[f] && same; b++)
          same = D::coupled(p.g0[f] + a, p.g0[f] + b) == D::coupled(p.g0[f2] + a, p.g0[f2] + b);
      for (int t = 0; t < p.nt && same; t++) same = p.tcpl[f][t] == p.tcpl[f2][t];
      if (same) c = p.cls[f2];
    }
    if (c < 0) { c = p.ncls++; p.crep[c] = f; }
    p.cls[f] = c;
  }
  // front-major layout
  int w = 0;
  for (int f = 0; f < nf; f++) {
    p.off[f] = w;
    for (int a = 0; a < p.n[f]; a++)
      for (int b = 0; b <= a; b++)
        if (D::coupled(p.g0[f] + a, p.g0[f] + b)) p.idx[p.g0[f] + a][p.g0[f] + b] = w++;
    for (int a = 0; a < p.n[f]; a++)
      for (int t = 0; t < p.nt; t++)
        if (p.tcpl[f][t]) p.idx[p.tg[t]][p.g0[f] + a] = w++;
    p.bsz[f] = w - p.off[f];
  }
  p.toff = w;
  for (int t1 = 0; t1 < p.nt; t1++)
    for (int t2 = 0; t2 <= t1; t2++)
      if (D::coupled(p.tg[t1], p.tg[t2])) p.idx[p.tg[t1]][p.tg[t2]] = w++;
  return p;
}

template <class R>
struct FP {
  static constexpr FrontPlan<R> v = make_front_plan<R>();
  static constexpr int NF = v.nf, GRP = v.fp, NT = v.nt;
  // every coupled pair has exactly one word, words 0 .. NNZ - 1
  static constexpr bool layout_ok() {
    using D = Dims<R>;
    int cnt = 0;
    bool seen[D::NNZ + 1] = {};
    for (int i = 0; i < R::NDOF; i++)
      for (int k = 0; k <= i; k++) {
        if (!D::coupled(i, k)) continue;
        const int x = v.idx[i][k];
        if (x < 0 || x >= D::NNZ || seen[x]) return false;
        seen[x] = true;
        cnt++;
      }
    return cnt == D::NNZ;
  }
  static_assert(layout_ok(), "front layout is not a permutation of the packed factor");
  static constexpr int idx(int i, int k) { return v.idx[i][k]; }
};

// Front class C: the representative's local patterns (shared by every front of the class)
template <class R, int C>
struct FrontCls {
  using D = Dims<R>;
  static constexpr int f = FP<R>::v.crep[C];
  static constexpr int g0 = FP<R>::v.g0[f], n = FP<R>::v.n[f], NT = FP<R>::NT;
  static constexpr bool cpl(int a, int b) { return D::coupled(g0 + a, g0 + b); }
  static constexpr bool tc(int t) { return FP<R>::v.tcpl[f][t]; }
  // word offsets within the front's block
  static constexpr int a_off(int a, int b) { return FP<R>::v.idx[g0 + a][g0 + b] - FP<R>::v.off[f]; }
  static constexpr int c_off(int a, int t) { return FP<R>::v.idx[FP<R>::v.tg[t]][g0 + a] - FP<R>::v.off[f]; }
  static constexpr int members() {
    int k = 0;
    for (int q = 0; q < FP<R>::NF; q++) k += FP<R>::v.cls[q] == C;
    return k;
  }
};

}  // namespace pbg
