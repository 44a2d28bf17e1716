// aw_tree.h -- the joint-space inertia's tree-sparse LDL' (MuJoCo 2.1 mj_factorM / mj_solveM),
// with the dof tree of the task known at compile time (aw_trees.h, TreeDef<task_kind>).
//
// M[i][k] is nonzero only when dof k is dof i, an ancestor or a descendant of it (the hand: five
// finger chains under the wrist; the object and the nail: separate chains).  MuJoCo factors
// M = L' D L (L unit lower triangular, L[k][i] nonzero only for i an ancestor of k) by
// eliminating the dofs from the leaves up; there is no fill-in.  Here the dofs of one tree level
// are eliminated together -- they are independent -- so the sequential chain is the tree depth
// (hammer 9, door 11, pen 7, relocate 13 levels) instead of nv = 30..36 pivots of a dense
// Cholesky, and the work is the tree's nonzeros (hammer: 147 off-diagonal entries instead of
// 528).  Lane i holds row i of M in registers (float r[NV], as stage_crb builds it); every index
// below is a compile-time constant, and the values of another lane arrive by v_readlane (SGPR
// broadcast), so no stage touches LDS.
//
// Factor layout on return, lane i (entries kept unscaled, the solves scale them where used):
// r[k] = M'[i][k] with L[i][k] = M'[i][k] / D[i] for k an ancestor of i; r[j] = M'[i][j] with
// L[j][i] = M'[i][j] / D[j] for j a descendant of i (M' = M as updated up to that elimination);
// invd = 1 / D[i]; entries of unrelated dofs stay 0.
#pragma once
#include <utility>

#include "aw_common.h"
#include "aw_trees.h"

namespace aw {

template <int TASK> struct Tree {
  using D = TreeDef<TASK>;
  static constexpr int NV = D::NV;
  static constexpr int depth(int j) {
    int d = 0;
    for (int p = D::parent[j]; p >= 0; p = D::parent[p]) d++;
    return d;
  }
  // a-th strict ancestor of j (a = 0: the parent), a < depth(j)
  static constexpr int anc(int j, int a) {
    int p = D::parent[j];
    for (int t = 0; t < a; t++) p = D::parent[p];
    return p;
  }
  static constexpr int maxdepth() {
    int m = 0;
    for (int j = 0; j < NV; j++) m = depth(j) > m ? depth(j) : m;
    return m;
  }
  static constexpr int NLEV = maxdepth() + 1;
  // first dof of the object block: the smallest p > 0 such that no dof in [p, NV) descends from
  // a dof in [0, p) (the hand's tree; M is then block-diagonal across p).  0 = no split.
  static constexpr int split() {
    for (int p = 1; p < NV; p++) {
      bool ok = D::parent[p] < 0;
      for (int j = p; j < NV; j++)
        if (D::parent[j] >= 0 && D::parent[j] < p) ok = false;
      if (ok) return p;
    }
    return 0;
  }
  static constexpr int SPLIT = split();
  static constexpr bool ordered() {   // ancestors before descendants (MuJoCo's dof order)
    for (int j = 0; j < NV; j++)
      if (D::parent[j] >= j) return false;
    return true;
  }
};
// constants forced at compile time (template arguments of every register index below)
template <int TASK, int J> struct TDepth { static constexpr int v = Tree<TASK>::depth(J); };
template <int TASK, int J, int A> struct TAnc { static constexpr int v = Tree<TASK>::anc(J, A); };

namespace tree {
template <int TASK> using Row = float[Tree<TASK>::NV];

// Lane masks as arithmetic on the lane id held as a float (lf = lane): a 0/1 factor costs two
// VALU ops where it is used; a v_cmp mask per dof would be hoisted into dozens of live SGPR pairs.
template <int J> AW_DEV float below(float lf) { return __builtin_amdgcn_fmed3f((float)J - lf, 0.f, 1.f); }  // lane < J
template <int J> AW_DEV float above(float lf) { return __builtin_amdgcn_fmed3f(lf - (float)J, 0.f, 1.f); }  // lane > J
template <int J> AW_DEV float is(float lf) { return fmaxf(1.f - fabsf((float)J - lf), 0.f); }              // lane == J

// eliminate pivot J (1 / D[J] in lane J's inv): for every pair (i, k) of ancestors of J,
// M[i][k] -= M[i][J] M[J][k] / D[J].  Lanes i < J are ancestors of J or unrelated (M[i][J] = 0).
// The entries M[i][J] (lanes i < J) and M[J][k] (lane J) are left unscaled: the solves scale them
// by 1 / D[J] and 1 / D[i] where they use them.
template <int TASK, int J, int... A>
AW_DEV void col(Row<TASK>& r, float inv, float lf, std::integer_sequence<int, A...>) {
  const float c = r[J] * rlane(inv, J) * below<J>(lf);   // M[lane][J] / D[J] on ancestor lanes, else 0
  // lane J's own row is untouched (c = 0 there), so rlane(r[k], J) is M[J][k] throughout
  ((r[TAnc<TASK, J, A>::v] = fmaf(-c, rlane(r[TAnc<TASK, J, A>::v], J), r[TAnc<TASK, J, A>::v])), ...);
}
template <int TASK, int L, int J>
AW_DEV void col_at(Row<TASK>& r, float inv, float lf) {
  if constexpr (TDepth<TASK, J>::v == L && L > 0) col<TASK, J>(r, inv, lf, std::make_integer_sequence<int, L>{});
}
template <int TASK, int L, int J>
AW_DEV void piv_at(const Row<TASK>& r, float lf, float& d, float& e) {
  if constexpr (TDepth<TASK, J>::v == L) {
    const float f = is<J>(lf);
    d = fmaf(r[J], f, d);   // exact: one term is nonzero
    e += f;
  }
}
template <int TASK, int L, int... J>
AW_DEV void level(Row<TASK>& r, float& invd, float lf, std::integer_sequence<int, J...>) {
  float d = 0.f, e = 0.f;   // this level's pivot lanes: their diagonal, and e = 1
  (piv_at<TASK, L, J>(r, lf, d, e), ...);
  const float inv = __builtin_amdgcn_rcpf(fmaxf(d, MINVAL));   // mj_factorI: D < mjMINVAL -> mjMINVAL
  invd = fmaf(inv, e, invd);   // each lane is a pivot at exactly one level: invd = 0 + inv, exactly
  (col_at<TASK, L, J>(r, inv, lf), ...);
}
template <int TASK, int... Ls>
AW_DEV void levels_down(Row<TASK>& r, float& invd, float lf, std::integer_sequence<int, Ls...>) {
  constexpr int NL = Tree<TASK>::NLEV;
  (level<TASK, NL - 1 - Ls>(r, invd, lf, std::make_integer_sequence<int, Tree<TASK>::NV>{}), ...);
}

// x <- inv(L') x: dof J's entry is final once its subtree is done, then leaves its ancestors
// (L[J][i] = M[i][J] / D[J], lanes i < J)
template <int TASK, int L, int J>
AW_DEV void up_at(const Row<TASK>& r, float invd, float& x, float lf) {
  if constexpr (TDepth<TASK, J>::v == L) x = fmaf(-r[J] * below<J>(lf), rlane(x * invd, J), x);
}
template <int TASK, int L, int... J>
AW_DEV void up_level(const Row<TASK>& r, float invd, float& x, float lf, std::integer_sequence<int, J...>) {
  (up_at<TASK, L, J>(r, invd, x, lf), ...);
}
template <int TASK, int... Ls>
AW_DEV void solve_up(const Row<TASK>& r, float invd, float& x, float lf, std::integer_sequence<int, Ls...>) {
  constexpr int NL = Tree<TASK>::NLEV;
  (up_level<TASK, NL - 1 - Ls>(r, invd, x, lf, std::make_integer_sequence<int, Tree<TASK>::NV>{}), ...);
}
// x <- inv(L) x: dof K's entry is final once its ancestors are done, then reaches its descendants
// (L[i][K] = M[i][K] / D[i], lanes i > K)
template <int TASK, int L, int K>
AW_DEV void down_at(const Row<TASK>& r, float invd, float& x, float lf) {
  if constexpr (TDepth<TASK, K>::v == L) x = fmaf(-r[K] * invd * above<K>(lf), rlane(x, K), x);
}
template <int TASK, int L, int... K>
AW_DEV void down_level(const Row<TASK>& r, float invd, float& x, float lf, std::integer_sequence<int, K...>) {
  (down_at<TASK, L, K>(r, invd, x, lf), ...);
}
template <int TASK, int... Ls>
AW_DEV void solve_down(const Row<TASK>& r, float invd, float& x, float lf, std::integer_sequence<int, Ls...>) {
  (down_level<TASK, Ls>(r, invd, x, lf, std::make_integer_sequence<int, Tree<TASK>::NV>{}), ...);
}

// multi-RHS: lane i holds X = column i of inv(M) (a register vector over dofs); the factor's
// entries are uniform here (readlane of the owning lane: M[J][a] unscaled, and 1 / D[J])
template <int TASK, int J, int... A>
AW_DEV void inv_up_col(const Row<TASK>& r, float invd, Row<TASK>& X, std::integer_sequence<int, A...>) {
  const float t = X[J] * rlane(invd, J);   // L[J][a] X[J] = M[J][a] (X[J] / D[J])
  ((X[TAnc<TASK, J, A>::v] = fmaf(-rlane(r[TAnc<TASK, J, A>::v], J), t, X[TAnc<TASK, J, A>::v])), ...);
}
template <int TASK, int J, int... A>
AW_DEV void inv_down_col(const Row<TASK>& r, float invd, Row<TASK>& X, std::integer_sequence<int, A...>) {
  float acc = 0.f;
  ((acc = fmaf(rlane(r[TAnc<TASK, J, A>::v], J), X[TAnc<TASK, J, A>::v], acc)), ...);
  X[J] = fmaf(-rlane(invd, J), acc, X[J]);
}
template <int TASK, int... J>
AW_DEV void inverse_cols(const Row<TASK>& r, float invd, Row<TASK>& X, float lf, std::integer_sequence<int, J...>) {
  constexpr int NV = Tree<TASK>::NV;
  ((X[J] = is<J>(lf)), ...);
  // inv(L'): dofs in decreasing index = leaves before their ancestors (ordered tree)
  ((inv_up_col<TASK, NV - 1 - J>(r, invd, X, std::make_integer_sequence<int, TDepth<TASK, NV - 1 - J>::v>{})), ...);
  ((X[J] *= rlane(invd, J)), ...);
  // inv(L): increasing index = ancestors first
  ((inv_down_col<TASK, J>(r, invd, X, std::make_integer_sequence<int, TDepth<TASK, J>::v>{})), ...);
}
}  // namespace tree

// In-place factor of the dense symmetric row r (lane = dof); lanes >= NV carry garbage.
template <int TASK>
AW_DEV void tree_factor(float (&r)[Tree<TASK>::NV], float& invd, int lane) {
  static_assert(Tree<TASK>::ordered(), "dof tree must list ancestors before descendants");
  invd = 0.f;
  tree::levels_down<TASK>(r, invd, opaque((float)lane), std::make_integer_sequence<int, Tree<TASK>::NLEV>{});
}
// x = inv(M) b, b and x lane-distributed (lanes >= NV return 0)
template <int TASK>
AW_DEV float tree_solve(const float (&r)[Tree<TASK>::NV], float invd, float b, int lane) {
  constexpr int NV = Tree<TASK>::NV, NL = Tree<TASK>::NLEV;
  const float lf = opaque((float)lane);
  float x = lane < NV ? b : 0.f;
  tree::solve_up<TASK>(r, invd, x, lf, std::make_integer_sequence<int, NL>{});
  x *= invd;
  tree::solve_down<TASK>(r, invd, x, lf, std::make_integer_sequence<int, NL>{});
  return lane < NV ? x : 0.f;
}
// lane i: X = row i (= column i) of inv(M); lanes >= NV: garbage
template <int TASK>
AW_DEV void tree_inverse(const float (&r)[Tree<TASK>::NV], float invd, int lane, float (&X)[Tree<TASK>::NV]) {
  tree::inverse_cols<TASK>(r, invd, X, opaque((float)lane), std::make_integer_sequence<int, Tree<TASK>::NV>{});
}

}  // namespace aw
