// aw_dynamics.h -- position/velocity stages of mj_step for one env per wave (fp32).
//
// Lane maps: bodies (kinematics in tree-level order, subtree sums over DFS ranges), dofs
// (cdof, M rows, RNE projections), geoms / sites.  Restates MuJoCo 2.1 mj_kinematics,
// mj_comPos, mj_tendon (fixed), mj_crb, mj_comVel, mj_rne (flg_acc = 0), mj_passive,
// mj_fwdActuation (see oracle/mjstep.cc for the fp64 statement of the same stages).
#pragma once
#include "aw_common.h"
#include "aw_sincos64.h"

namespace aw {

// subtree sums over DFS ranges: the loads of this many bodies are issued together
#ifndef AW_SUB_UNROLL
#define AW_SUB_UNROLL 4
#endif

// ---------------------------------------------------------------------------------------
// this env's parameters + the per-env copies of the overridable fields read in hot loops
// (geom_size: every collider; body_mass: subtree sums); other overrides are applied where
// the field is read (apply_ovr)
AW_DEV void stage_model(const DModel& m, Env& s, const float* params, int lane) {
  if (lane < m.nparam) s.prm[lane] = params ? params[lane] : MD(param_default, lane);
  for (int b = lane; b < m.nbody; b += 64) s.bmass[b] = MD(body_mass, b);
  for (int g = lane; g < m.ngeom; g += 64)
    for (int k = 0; k < 3; k++) s.gsize[g][k] = MD(geom_size, 3 * g + k);
  wsync();
  if (lane == 0) {
    for (int p = 0; p < m.nparam; p++) {
      int o = MD(param_obj, p), c = MD(param_comp, p);
      if (MD(param_field, p) == 3) s.bmass[o] = s.prm[p];
      else if (MD(param_field, p) == 5) s.gsize[o][c] = s.prm[p];
    }
  }
  wsync();
}
// v[0..N) = model field (field code, object) with this env's overrides applied
template <int N>
AW_DEV void apply_ovr(const DModel& m, const Env& s, int field, int obj, float (&v)[N]) {
  for (int p = 0; p < m.nparam; p++)
    if (MD(param_field, p) == field && MD(param_obj, p) == obj) {
      const int c = MD(param_comp, p);
      const float x = s.prm[p];
#pragma unroll
      for (int k = 0; k < N; k++) v[k] = k == c ? x : v[k];
    }
}

// mj_kinematics (+ local2global for geoms, sites).  Frames are kept as quaternions only: every
// position update rotates by the (normalised) quaternion instead of a stored rotation matrix.
AW_DEV void stage_kinematics(const DModel& m, Env& s, int lane) {
  if (lane == 0) {
    s.xpos[0][0] = s.xpos[0][1] = s.xpos[0][2] = 0;
    s.xquat[0][0] = 1; s.xquat[0][1] = s.xquat[0][2] = s.xquat[0][3] = 0;
  }
  wsync();
  // Body frames without a level sweep.  (A) Lane b composes its body offset and its joints into
  // ONE rigid transform T_b in the parent's frame -- every lane at once, nothing read from another
  // lane -- and leaves its joints' axes / anchors in that frame.  (B) Global frames by pointer
  // jumping on the tree: each round replaces (T, target) with (T_target o T, target's target),
  // so the dependent chain is log2(depth) compositions instead of depth.  (C) Lane = dof: the
  // joint axes / anchors to the world frame with the parent's global frame.  Same transforms as
  // mj_kinematics, composed in a different order (fp32 rounding only).
  {
    const bool own = lane > 0 && lane < m.nbody;
    const int b = own ? lane : 0;
    const int p = MD(body_parentid, b), da = MD(body_dofadr, b), dn = own ? MD(body_dofnum, b) : 0;
    float tp[3], tq[4];
    for (int k = 0; k < 3; k++) tp[k] = MD(body_pos, 3 * b + k);
    for (int k = 0; k < 4; k++) tq[k] = MD(body_quat, 4 * b + k);
    if (own && MD(body_ovr, b)) { apply_ovr<3>(m, s, 0, b, tp); apply_ovr<4>(m, s, 1, b, tq); }
    // (A) branch-free joint steps: a slide is a hinge with ql = 1 and no anchor arm (exact)
#pragma unroll
    for (int k = 0; k < MAXJB; k++) {
      if (k < dn) {
        const int j = da + k;
        float axis[3], jp[3], xa[3], xn[3];
        for (int c = 0; c < 3; c++) { axis[c] = MD(jnt_axis, 3 * j + c); jp[c] = MD(jnt_pos, 3 * j + c); }
        const bool hinge = MD(jnt_type, j) != JNT_SLIDE;
        const float q = s.qpos[j];
        rotvq(xa, axis, tq);
        rotvq(xn, jp, tq);
        add3(xn, xn, tp);
        copy3(s.xaxis[j], xa);    // parent frame; (C) makes them global
        copy3(s.xanchor[j], xn);
        // hardware v_sin / v_cos on the half angle reduced to [-pi, pi]
        const float hq = hinge ? 0.5f * q : 0.f;
        const float hr = fmaf(-6.28318530717958648f, rintf(hq * 0.159154943091895336f), hq);
        const float sn = __sinf(hr), cs = __cosf(hr);
        const float ql[4] = {cs, axis[0] * sn, axis[1] * sn, axis[2] * sn};
        mulq(tq, tq, ql);
        float v[3];
        rotvq(v, jp, tq);
        for (int c = 0; c < 3; c++) tp[c] = hinge ? xn[c] - v[c] : fmaf(xa[c], q, tp[c]);
      }
    }
    // (B) pointer jumping; targets in the (not yet written) cinert storage
    int* tgt = reinterpret_cast<int*>(&s.cinert[0][0]);
    int t = own ? p : 0;
    if (own) {
      copy3(s.xpos[b], tp);
      for (int c = 0; c < 4; c++) s.xquat[b][c] = tq[c];
    }
    if (lane < m.nbody) tgt[lane] = t;
    wsync();
    while (__ballot(t != 0)) {
      float pp[3], pq[4];
      int tt = 0;
      if (t != 0) {
        copy3(pp, s.xpos[t]);
        for (int c = 0; c < 4; c++) pq[c] = s.xquat[t][c];
        tt = tgt[t];
      }
      wsync();
      if (t != 0) {
        float v[3];
        rotvq(v, tp, pq);
        add3(tp, pp, v);
        mulq(tq, pq, tq);
        t = tt;
        copy3(s.xpos[b], tp);
        for (int c = 0; c < 4; c++) s.xquat[b][c] = tq[c];
        tgt[b] = t;
      }
      wsync();
    }
    if (own) {
      normq(tq);
      for (int c = 0; c < 4; c++) s.xquat[b][c] = tq[c];
    }
    wsync();
    // (C) joint axes / anchors to the world frame (lane = dof)
    if (lane < m.nv) {
      const int j = lane, pb = MD(body_parentid, MD(dof_bodyid, j));
      float pq[4], v[3];
      for (int c = 0; c < 4; c++) pq[c] = s.xquat[pb][c];
      rotvq(v, s.xaxis[j], pq);
      copy3(s.xaxis[j], v);
      rotvq(v, s.xanchor[j], pq);
      add3(s.xanchor[j], v, s.xpos[pb]);
    }
    wsync();
  }
  // geoms (compact collidable list), sites, inertial frames
  for (int g = lane; g < m.ngeom; g += 64) {
    int b = MD(geom_bodyid, g);
    float v[3], q[4], gq[4], gp[3], bq[4];
    for (int c = 0; c < 3; c++) gp[c] = MD(geom_pos, 3 * g + c);
    if (MD(geom_ovr, g)) apply_ovr<3>(m, s, 4, g, gp);
    for (int c = 0; c < 4; c++) { gq[c] = MD(geom_quat, 4 * g + c); bq[c] = s.xquat[b][c]; }
    rotvq(v, gp, bq);
    add3(s.gxpos[g], v, s.xpos[b]);
    mulq(q, bq, gq);
    for (int c = 0; c < 4; c++) s.gxquat[g][c] = q[c];
  }
  for (int i = lane; i < m.nsite; i += 64) {
    int b = MD(site_bodyid, i);
    float v[3], sp[3], bq[4];
    for (int c = 0; c < 3; c++) sp[c] = MD(site_pos, 3 * i + c);
    if (MD(site_ovr, i)) apply_ovr<3>(m, s, 2, i, sp);
    for (int c = 0; c < 4; c++) bq[c] = s.xquat[b][c];
    rotvq(v, sp, bq);
    add3(s.sxpos[i], v, s.xpos[b]);
  }
  if (lane < m.ntouch) {
    int i = MD(touch_site, lane), b = MD(site_bodyid, i);
    float q[4], sq[4];
    for (int c = 0; c < 4; c++) sq[c] = MD(site_quat, 4 * i + c);
    mulq(q, s.xquat[b], sq);
    q2m(s.txmat[lane], q);
  }
  for (int b = lane; b < m.nbody; b += 64) {
    float v[3], ip[3], bq[4];
    for (int c = 0; c < 3; c++) ip[c] = MD(body_ipos, 3 * b + c);
    for (int c = 0; c < 4; c++) bq[c] = s.xquat[b][c];
    rotvq(v, ip, bq);
    add3(s.xipos[b], v, s.xpos[b]);
  }
  wsync();
}

// 1 / sqrt(x): the hardware estimate refined by Newton steps (fp64: two steps from v_rsq_f64 give
// full double precision for normal x, where the correctly rounded sqrt + divide expansions cost
// ~3x the instructions on the MPR's serial chain: -1.4 % k_step, r04m)
template <class T> AW_DEV T rsqrt_fast(T x) {
  if constexpr (sizeof(T) == 8) {
    double r = __builtin_amdgcn_rsq(x);
    const double hx = 0.5 * x;
    r = r * fma(-hx * r, r, 1.5);
    r = r * fma(-hx * r, r, 1.5);
    return r;
  }
  return T(1.0) / sqrt(x);
}

template <int N>
AW_DEV void apply_ovr64(const DModel& m, const Env& s, int field, int obj, double (&v)[N]) {
  for (int p = 0; p < m.nparam; p++)
    if (MD(param_field, p) == field && MD(param_obj, p) == obj) {
      const int c = MD(param_comp, p);
      const double x = (double)s.prm[p];
#pragma unroll
      for (int k = 0; k < N; k++) v[k] = k == c ? x : v[k];
    }
}

// sin / cos of a joint half-angle in fp64 (aw_sincos64.h, shared with the host check
// tests/sincos64_check.cc).  It replaces ocml's sincos, whose table-driven large-argument path left
// 64-bit table addresses hoisted out of the env loop and reloaded from scratch on every call; the
// constants live in constant memory and are read where they are used through a pointer the
// compiler cannot see through (as literals, LICM hoisted them into nine VGPR pairs that the
// allocator reloaded from scratch on every call as well).
static __constant__ double SINCOS64_K[15] = AW_SINCOS64_K;
AW_DEV void sincos64(double x, double* sn, double* cs) {
  const double* K = SINCOS64_K;
  asm volatile("" : "+s"(K));
  sincos64_k(x, K, sn, cs);
}

// mj_kinematics in fp64 for the bodies that carry the geometry of this substep's MPR (cylinder)
// pairs and their ancestors (s.kin64_mask), from the fp32 state with the model's fp64 constants
// (levels holding none of them are skipped): the oracle's
// operation order (oracle/mjstep.cc kinematics: parent xmat * body_pos, xquat chain, hinge
// axis-angle quaternions, normalised).  MPR contact points are ill-conditioned on line / face
// contacts (a cylinder lying on a box: rotating the cylinder by 1e-7 rad moves MuJoCo's point
// between the ends), so MPR runs on these fp64 frames, not on the fp32 ones.
AW_DEV void stage_kin64(const DModel& m, Env& s, int lane) {
  if (lane == 0) {
    double* X = kin64(s, 0);
    X[0] = X[1] = X[2] = 0.0;
    X[3] = 1.0; X[4] = X[5] = X[6] = 0.0;
  }
  // one joint per lane up front, for every joint of a needed body: its record in LDS -- the hinge
  // half-angle sin / cos, the axis and its kind (0 hinge at the body origin, 1 slide, 2 hinge with
  // an anchor arm).  The level loop below is left with the frame algebra on its serial chain and
  // reads LDS instead of waiting on model-table loads joint by joint (same sincos, same inputs:
  // bitwise the per-level evaluation; r04o A/B: -0.7 % random, -1.4 % DAPG for the sincos, r04r
  // -0.5 % random for the records)
  const int jl = lane < m.njnt ? lane : 0;
  if (lane < m.njnt && ((s.kin64_mask >> MD(jnt_bodyid, jl)) & 1ull)) {
    double* SC = kin64_sc(s, jl);
    const bool slide = MD(jnt_type, jl) == JNT_SLIDE;
    double sn = 0.0, cs = 1.0;
#ifdef AW_OCML_SINCOS
    if (!slide) sincos(qpos64(s, jl) * 0.5, &sn, &cs);
#else
    if (!slide) sincos64(qpos64(s, jl) * 0.5, &sn, &cs);
#endif
    const double p0 = MD(jnt_pos64, 3 * jl), p1 = MD(jnt_pos64, 3 * jl + 1), p2 = MD(jnt_pos64, 3 * jl + 2);
    SC[0] = sn;
    SC[1] = cs;
    SC[2] = MD(jnt_axis64, 3 * jl);
    SC[3] = MD(jnt_axis64, 3 * jl + 1);
    SC[4] = MD(jnt_axis64, 3 * jl + 2);
    SC[5] = slide ? 1.0 : (p0 == 0.0 && p1 == 0.0 && p2 == 0.0 ? 0.0 : 2.0);
  }
  wsync();
  const bool own = lane > 0 && lane < m.nbody && ((s.kin64_mask >> lane) & 1ull);
  const int b = own ? lane : 0;
  const int dep = own ? MD(body_depth, b) : -1;
  const int ntop = (int)wave_max((float)dep) + 1;   // deepest level holding a needed frame
  const int p = MD(body_parentid, b), da = MD(body_dofadr, b), dn = own ? MD(body_dofnum, b) : 0;
  double bp[3], bq[4];
  for (int k = 0; k < 3; k++) bp[k] = MD(body_pos64, 3 * b + k);
  for (int k = 0; k < 4; k++) bq[k] = MD(body_quat64, 4 * b + k);
  if (own && MD(body_ovr, b)) { apply_ovr64<3>(m, s, 0, b, bp); apply_ovr64<4>(m, s, 1, b, bq); }
  for (int lev = 1; lev < ntop; lev++) {
    if (dep == lev) {
      const double* P = kin64(s, p);
      double pq[4] = {P[3], P[4], P[5], P[6]}, pm[9], xp[3], xq[4];
      q2m(pm, pq);
      mulmv3(xp, pm, bp);
      xp[0] += P[0]; xp[1] += P[1]; xp[2] += P[2];
      mulq(xq, pq, bq);
      for (int k = 0; k < dn; k++) {
        const int j = da + k;
        double axis[3], jp[3], xanchor[3];
        const double* SCj = kin64_sc(s, j);
        for (int c = 0; c < 3; c++) axis[c] = SCj[2 + c];
        const double kind = SCj[5];
        if (kind == 1.0) {
          const double qj = qpos64(s, j);
          double xaxis[3];
          rotvq(xaxis, axis, xq);
          for (int c = 0; c < 3; c++) xp[c] += xaxis[c] * qj;
          continue;
        }
        const double qs[4] = {SCj[1], axis[0] * SCj[0], axis[1] * SCj[0], axis[2] * SCj[0]};
        if (kind == 0.0) {
          mulq(xq, xq, qs);
          continue;
        }
        // a hinge with an anchor arm (kind 2); a hinge at the body origin (kind 0, the free objects'
        // rotations) skipped both anchor rotations above: they are rotations of the zero vector
        double v[3];
        for (int c = 0; c < 3; c++) jp[c] = MD(jnt_pos64, 3 * j + c);
        rotvq(xanchor, jp, xq);
        add3(xanchor, xanchor, xp);
        mulq(xq, xq, qs);
        rotvq(v, jp, xq);
        sub3(xp, xanchor, v);
      }
      double* X = kin64(s, b);
      // normalised by one refined reciprocal square root (the oracle divides by the norm: the two
      // differ in the last fp64 bit)
      const double n2 = xq[0] * xq[0] + xq[1] * xq[1] + xq[2] * xq[2] + xq[3] * xq[3];
      if (n2 < 1e-30) { X[3] = 1.0; X[4] = X[5] = X[6] = 0.0; }
      else { const double in = rsqrt_fast(n2); for (int c = 0; c < 4; c++) X[3 + c] = xq[c] * in; }
      for (int c = 0; c < 3; c++) X[c] = xp[c];
    }
    wsync();
  }
}

// mj_comPos: subtree com (divided by the compile-time subtree mass), cinert, cdof
AW_DEV void stage_com(const DModel& m, Env& s, int lane) {
  for (int b = lane; b < m.nbody; b += 64) {
    float acc[3] = {0, 0, 0};
    const int de = MD(body_subtree_end, b);
#pragma unroll AW_SUB_UNROLL
    for (int d = b; d < de; d++) {
      float md = s.bmass[d];
      acc[0] += md * s.xipos[d][0]; acc[1] += md * s.xipos[d][1]; acc[2] += md * s.xipos[d][2];
    }
    float stm = MD(body_subtreemass, b);
    if (stm < MINVAL) copy3(s.subcom[b], s.xipos[b]);
    else scl3(s.subcom[b], acc, 1.0f / stm);
  }
  wsync();
  for (int b = lane; b < m.nbody; b += 64) {
    float* c = s.cinert[b];
    if (b == 0) { for (int k = 0; k < 10; k++) c[k] = 0; continue; }
    float q[4], iq[4], R[9], dif[3];
    for (int k = 0; k < 4; k++) iq[k] = MD(body_iquat, 4 * b + k);
    mulq(q, s.xquat[b], iq);
    q2m(R, q);
    const auto I = MDP(body_inertia, 3 * b);
    float mass = s.bmass[b];
    sub3(dif, s.xipos[b], s.subcom[MD(body_rootid, b)]);
    float T[9];
    for (int a = 0; a < 3; a++)
      for (int bb = 0; bb < 3; bb++)
        T[3 * a + bb] = R[3 * a] * I[0] * R[3 * bb] + R[3 * a + 1] * I[1] * R[3 * bb + 1] + R[3 * a + 2] * I[2] * R[3 * bb + 2];
    c[0] = T[0] + mass * (dif[1] * dif[1] + dif[2] * dif[2]);
    c[1] = T[4] + mass * (dif[0] * dif[0] + dif[2] * dif[2]);
    c[2] = T[8] + mass * (dif[0] * dif[0] + dif[1] * dif[1]);
    c[3] = T[1] - mass * dif[0] * dif[1];
    c[4] = T[2] - mass * dif[0] * dif[2];
    c[5] = T[5] - mass * dif[1] * dif[2];
    c[6] = mass * dif[0]; c[7] = mass * dif[1]; c[8] = mass * dif[2];
    c[9] = mass;
  }
  if (lane < m.nv) {
    int j = lane, b = MD(dof_bodyid, j);
    float* cd = s.cdof[j];
    const float* axis = s.xaxis[j];
    if (MD(jnt_type, j) == JNT_SLIDE) {
      cd[0] = cd[1] = cd[2] = 0;
      copy3(cd + 3, axis);
    } else {
      float off[3];
      sub3(off, s.subcom[MD(body_rootid, b)], s.xanchor[j]);
      copy3(cd, axis);
      cross3(cd + 3, axis, off);
    }
  }
  wsync();
}

// mj_crb -> M row per lane (registers).  Runs after RNE: the composite inertias overwrite
// cinert in place.  M[i][k] = cdof_k . (crb_{body i} cdof_i) for k an ancestor of i, symmetric
// for descendants, + armature on the diagonal.
template <int NV>
AW_DEV void stage_crb(const DModel& m, Env& s, int lane, float (&Mrow)[NV]) {
  float acc[10];
  for (int k = 0; k < 10; k++) acc[k] = 0;
  const int bb = lane < m.nbody ? lane : 0;
  if (lane < m.nbody && lane > 0)
#pragma unroll AW_SUB_UNROLL
    for (int d = bb; d < MD(body_subtree_end, bb); d++)
      for (int k = 0; k < 10; k++) acc[k] += s.cinert[d][k];
  wsync();
  if (lane < m.nbody)
    for (int k = 0; k < 10; k++) s.cinert[bb][k] = acc[k];
  wsync();
  const int li = lane < NV ? lane : NV - 1;
  float ci[6], bi[6];
  for (int k = 0; k < 6; k++) ci[k] = s.cdof[li][k];
  mul_inert_vec(bi, s.cinert[MD(dof_bodyid, li)], ci);
  for (int k = 0; k < 6; k++) s.buf[li][k] = bi[k];
  wsync();
  const unsigned long long anc = MD(dof_ancmask, li);
  const float arm = MD(dof_armature, li);
  // P = B C' on the matrix cores (B: rows b_i = crb_{body i} cdof_i, C: rows cdof_k; K = 6 padded
  // to two K-steps of v_mfma_f32_16x16x4_f32), lower tiles only.  M[i][k] = P[i][k] for k an
  // ancestor of i and P[k][i] for a descendant, so each lower entry is stored at (i, k) and
  // (k, i) of a square staging block in the dense-J rows (dead from the narrowphase to the
  // constraint rows; the pair list / fp64 frames there are consumed) and lane i reads its row
  // back with 16-byte reads: ~24 LDS ops + 12 MFMAs instead of 33 x (12 broadcast reads + 12 fma).
  {
    typedef float f4 __attribute__((ext_vector_type(4)));
    constexpr int NT = (NV + 15) / 16, SS = VS;
    static_assert(offsetof(Env, rowbuf) == offsetof(Env, J) + sizeof(float) * JL * VS &&
                  MAXV * SS <= JL * VS + MAXEFC, "CRB staging block does not fit the dense-J rows + rowbuf");
    float* S = &s.J[0][0];
    const int sub = lane >> 4, col = lane & 15;
    f4 acc[NT][NT];
#pragma unroll
    for (int ti = 0; ti < NT; ti++)
#pragma unroll
      for (int tj = 0; tj <= ti; tj++) acc[ti][tj] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ks++) {
      const int c = 4 * ks + sub;
      const bool cv = c < 6;
      const int cc = cv ? c : 0;
      float a[NT], b[NT];
#pragma unroll
      for (int t = 0; t < NT; t++) {
        const int i = 16 * t + col;
        const bool v = cv && i < NV;
        const int ii = i < NV ? i : NV - 1;
        const float av = s.buf[ii][cc], bv = s.cdof[ii][cc];   // valid (ii, cc): load, then select
        a[t] = v ? av : 0.f;
        b[t] = v ? bv : 0.f;
      }
#pragma unroll
      for (int ti = 0; ti < NT; ti++)
#pragma unroll
        for (int tj = 0; tj <= ti; tj++)
          acc[ti][tj] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ti], b[tj], acc[ti][tj], 0, 0, 0);
    }
    wsync();
#pragma unroll
    for (int ti = 0; ti < NT; ti++)
#pragma unroll
      for (int tj = 0; tj <= ti; tj++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int i = 16 * ti + 4 * sub + r, k = 16 * tj + col;
          if (i < NV && k <= i) {
            S[i * SS + k] = acc[ti][tj][r];
            S[k * SS + i] = acc[ti][tj][r];
          }
        }
    wsync();
    const float* Sr = S + li * SS;
#pragma unroll
    for (int q = 0; q < (NV + 3) / 4; q++) {
      const float4 v4 = *reinterpret_cast<const float4*>(Sr + 4 * q);
      const float vv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const int k = 4 * q + t;
        if (k >= NV) continue;
        const bool rel = ((anc >> k) | (MD(dof_ancmask, k) >> li)) & 1ull;   // no short-circuit branch
        Mrow[k] = k == li ? vv[t] + arm : (rel ? vv[t] : 0.f);
      }
    }
    wsync();
    return;
  }
#pragma unroll
  for (int k = 0; k < NV; k++) {
    float ck[6], bk[6];
    for (int c = 0; c < 6; c++) { ck[c] = s.cdof[k][c]; bk[c] = s.buf[k][c]; }
    const unsigned long long anck = MD(dof_ancmask, k);
    float v;
    if (k == li) v = dot6(ci, bi) + arm;
    else if ((anc >> k) & 1ull) v = dot6(ck, bi);
    else if ((anck >> li) & 1ull) v = dot6(ci, bk);
    else v = 0.f;
    Mrow[k] = v;
  }
  wsync();
}

// mj_comVel + mj_rne(flg_acc=0) + mj_passive + mj_fwdActuation -> qfrc_smooth (lane = dof)
AW_DEV float stage_velocity(const DModel& m, Env& s, int lane) {
  float (*cvel)[6] = s.cvel;
  float (*cacc)[6] = s.cacc;
  if (lane == 0) {
    for (int k = 0; k < 6; k++) { cvel[0][k] = 0; cacc[0][k] = 0; }
    if (!(m.disableflags & DSBL_GRAVITY)) { cacc[0][3] = -m.gravity[0]; cacc[0][4] = -m.gravity[1]; cacc[0][5] = -m.gravity[2]; }
  }
  wsync();
  // cvel / cacc as tree prefix sums (pointer jumping, log2(depth) rounds) of per-body local terms:
  // cvel_b = cvel_parent + sum_j cdof_j qvel_j; cacc_b = cacc_parent + sum_j (cv_j x cdof_j) qvel_j
  // with cv_j the velocity before joint j (mj_comVel's per-joint order inside the body)
  {
    const bool own = lane > 0 && lane < m.nbody;
    const int b = own ? lane : 0;
    const int p = MD(body_parentid, b), da = MD(body_dofadr, b), dn = own ? MD(body_dofnum, b) : 0;
    int* tgt = reinterpret_cast<int*>(s.rowbuf);   // dead until the constraint rows
    auto tree_prefix = [&](float (*arr)[6], float (&v)[6]) {
      int t = own ? p : -1;
      if (own)
        for (int k = 0; k < 6; k++) arr[b][k] = v[k];
      if (lane < m.nbody) tgt[lane] = t;
      wsync();
      while (__ballot(t >= 0)) {
        float u[6];
        int tt = -1;
        if (t >= 0) {
          for (int k = 0; k < 6; k++) u[k] = arr[t][k];
          tt = tgt[t];
        }
        wsync();
        if (t >= 0) {
          for (int k = 0; k < 6; k++) { v[k] += u[k]; arr[b][k] = v[k]; }
          tgt[b] = tt;
          t = tt;
        }
        wsync();
      }
    };
    float lv[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < MAXJB; k++)
      if (k < dn) {
        const int j = da + k;
        const float qv = s.qvel[j];
        for (int c = 0; c < 6; c++) lv[c] = fmaf(s.cdof[j][c], qv, lv[c]);
      }
    tree_prefix(cvel, lv);
    float w[6], la[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < 6; c++) w[c] = cvel[p][c];
#pragma unroll
    for (int k = 0; k < MAXJB; k++)
      if (k < dn) {
        const int j = da + k;
        float cd[6], cdd[6];
        const float qv = s.qvel[j];
        for (int c = 0; c < 6; c++) cd[c] = s.cdof[j][c];
        cross_motion(cdd, w, cd);
        for (int c = 0; c < 6; c++) { la[c] = fmaf(cdd[c], qv, la[c]); w[c] = fmaf(cd[c], qv, w[c]); }
      }
    tree_prefix(cacc, la);
  }
  // local body force: cinert*cacc + cvel x* (cinert*cvel), written over cacc
  for (int b = 1 + lane; b < m.nbody; b += 64) {
    float f[6], t1[6], t2[6];
    mul_inert_vec(f, s.cinert[b], cacc[b]);
    mul_inert_vec(t1, s.cinert[b], cvel[b]);
    cross_force(t2, cvel[b], t1);
    for (int k = 0; k < 6; k++) f[k] += t2[k];
    // each lane reads and writes only its own body -> in place is safe
    for (int k = 0; k < 6; k++) cacc[b][k] = f[k];
  }
  wsync();
  // subtree sum (DFS range) -> cvel storage (cvel no longer needed)
  float sub[6];
  const int bb = lane < m.nbody ? lane : 0;
  for (int k = 0; k < 6; k++) sub[k] = 0;
  if (lane < m.nbody && lane > 0)
#pragma unroll AW_SUB_UNROLL
    for (int d = bb; d < MD(body_subtree_end, bb); d++)
      for (int k = 0; k < 6; k++) sub[k] += cacc[d][k];
  wsync();
  if (lane < m.nbody)
    for (int k = 0; k < 6; k++) cvel[bb][k] = sub[k];
  wsync();
  float qfrc = 0.f;
  if (lane < m.nv) {
    int j = lane;
    float bias = dot6(s.cdof[j], cvel[MD(dof_bodyid, j)]);
    float pas = (m.disableflags & DSBL_PASSIVE) ? 0.f : -MD(dof_damping, j) * s.qvel[j];
    float act = 0.f;
    int u = MD(dof_act, j);
    if (u >= 0 && !(m.disableflags & DSBL_ACTUATION)) {
      float ctrl = s.ctrl[u];
      if (MD(act_ctrllimited, u) && !(m.disableflags & DSBL_CLAMPCTRL))
        ctrl = clampf(ctrl, MD(act_ctrlrange, 2 * u), MD(act_ctrlrange, 2 * u + 1));
      float gear = MD(act_gear, u);
      float len = gear * s.qpos[j], vel = gear * s.qvel[j];
      const auto bp = MDP(act_bias, 3 * u);
      float f = MD(act_gain, u) * ctrl + bp[0] + bp[1] * len + bp[2] * vel;
      if (MD(act_forcelimited, u)) f = clampf(f, MD(act_forcerange, 2 * u), MD(act_forcerange, 2 * u + 1));
      act = gear * f;
    }
    qfrc = pas - bias + act;
  }
  wsync();
  return qfrc;
}

}  // namespace aw
