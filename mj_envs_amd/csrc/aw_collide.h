// aw_collide.h -- lane-per-pair narrowphase (fp32) for the Adroit primitive set.
//
// Restates MuJoCo 2.1 mj_collision (see oracle/collide.cc for the fp64 statement of the same
// algorithms): bounding-sphere test (rbound + margin, planes exempt), analytic plane/sphere/
// capsule/box colliders, SAT + fixed-order candidate points for box-box, libccd MPR (as used by
// mjc_Convex) for every pair involving a cylinder.  Each lane owns one geom pair and appends
// its contacts to the env's LDS list through an LDS atomic counter; the list is then sorted by
// (pair index, emission index) so contact order -- and hence constraint row order -- is the
// oracle's order.
#pragma once
#include "aw_common.h"
#include "aw_dynamics.h"

namespace aw {

struct GV {
  float pos[3];
  float mat[9];
  float size[3];
  int type;
};

struct Emit {
  Env* s;
  int pair;
  int cnt;
  double* out64 = nullptr;   // test hook (aw_collide_test): the MPR's fp64 (dist, pos, normal) per contact
};

AW_DEV void axis_of(float* a, const float* m, int k) { a[0] = m[k]; a[1] = m[3 + k]; a[2] = m[6 + k]; }

// Contact activation in fp64.  Resting and grasping contacts sit AT their margin (MuJoCo's reference
// acceleration drives dist -> margin), where fp32 geometry (~1e-7 m) decides on rounding whether a
// contact exists -- the dominant class of teacher-forced misses in the DAPG grasp (r05c: 150 of 293
// misses within 1e-6 of the margin, fingers / palm on the hammer handle).  So the sphere / capsule
// colliders (classes 1, 2) emit candidates up to DEC_EPS past the margin, and every contact within
// DEC_EPS of its margin is decided on its fp64 distance from fp64 geometry (refine_contacts64 below,
// the frames from stage_kin64): dropped when beyond the margin, kept with the fp64 distance otherwise.
constexpr float DEC_EPS = 2e-6f;

// aux: the contact's segment parameter t (capsule - box: the sphere-box contact at axis point t),
// kept in con_efc until the constraint rows reuse it
AW_DEV void emit(Emit& e, float dist, const float* pos, const float* n, float aux = 0.f) {
  if (e.cnt >= MAXPAIRCON) return;
  int slot = atomicAdd(&e.s->ncon, 1);
  if (slot < MAXCON) {
    e.s->con_key[slot] = e.pair * MAXPAIRCON + e.cnt;
    e.s->con_efc[slot] = __builtin_bit_cast(int, aux);
    e.s->con_pair[slot] = e.pair;
    e.s->con_dist[slot] = dist;
    copy3(e.s->con_pos[slot], pos);
    copy3(e.s->con_nrm[slot], n);
  } else {
    atomicOr(&e.s->status, (unsigned)ST_CON_OVERFLOW);
  }
  e.cnt++;
}

// ---------------------------------------------------------------------------------------
AW_DEV void c_plane_sphere(const float* p1, const float* m1, const float* p2, float r, float margin, Emit& e) {
  float n[3], dif[3];
  axis_of(n, m1, 2);
  sub3(dif, p2, p1);
  float dist = dot3(n, dif) - r;
  if (dist > margin) return;
  float pos[3];
  for (int k = 0; k < 3; k++) pos[k] = p2[k] - n[k] * (r + dist / 2);
  emit(e, dist, pos, n);
}

AW_DEV void c_plane_capsule(const GV& a, const GV& b, float margin, Emit& e) {
  float ax[3], p[3];
  axis_of(ax, b.mat, 2);
  for (int s = 1; s >= -1; s -= 2) {
    for (int k = 0; k < 3; k++) p[k] = b.pos[k] + s * ax[k] * b.size[1];
    c_plane_sphere(a.pos, a.mat, p, b.size[0], margin, e);
  }
}

AW_DEV void c_plane_box(const GV& a, const GV& b, float margin, Emit& e) {
  float n[3], dif[3];
  axis_of(n, a.mat, 2);
  sub3(dif, b.pos, a.pos);
  float dist = dot3(n, dif);
  int cnt = 0;
  for (int i = 0; i < 8; i++) {
    float v[3] = {(i & 1) ? b.size[0] : -b.size[0], (i & 2) ? b.size[1] : -b.size[1], (i & 4) ? b.size[2] : -b.size[2]};
    float corner[3];
    mulmv3(corner, b.mat, v);
    float ld = dot3(n, corner);
    if (dist + ld > margin || ld > 0) continue;
    float dd = dist + ld, pos[3];
    for (int k = 0; k < 3; k++) pos[k] = corner[k] + b.pos[k] - n[k] * dd / 2;
    emit(e, dd, pos, n);
    if (++cnt >= 4) return;
  }
}

AW_DEV void c_plane_cylinder(const GV& a, const GV& b, float margin, Emit& e) {
  float n[3], axis[3], dif[3], vec[3];
  axis_of(n, a.mat, 2);
  axis_of(axis, b.mat, 2);
  sub3(dif, b.pos, a.pos);
  float dist0 = dot3(dif, n);
  float prjaxis = dot3(n, axis);
  if (prjaxis > 0) { scl3(axis, axis, -1); prjaxis = -prjaxis; }
  for (int k = 0; k < 3; k++) vec[k] = axis[k] * prjaxis - n[k];
  float len = norm3(vec);
  if (len < MINVAL) axis_of(vec, b.mat, 0);
  else scl3(vec, vec, 1.0f / len);
  float r = b.size[0], h = b.size[1];
  scl3(vec, vec, r);
  float prjvec = dot3(vec, n);
  float ah[3];
  scl3(ah, axis, h);
  float pa = prjaxis * h;
  float pos[3], d;
  d = dist0 + pa + prjvec;
  if (d <= margin) {
    for (int k = 0; k < 3; k++) pos[k] = b.pos[k] + ah[k] + vec[k] - n[k] * d / 2;
    emit(e, d, pos, n);
  }
  d = dist0 - pa + prjvec;
  if (d <= margin) {
    for (int k = 0; k < 3; k++) pos[k] = b.pos[k] - ah[k] + vec[k] - n[k] * d / 2;
    emit(e, d, pos, n);
  }
  d = dist0 + pa - prjvec / 2;
  if (d <= margin) {
    float v1[3];
    cross3(v1, vec, axis);
    scl3(v1, v1, 0.86602540378443864676f);
    for (int s = -1; s <= 1; s += 2) {
      for (int k = 0; k < 3; k++) pos[k] = b.pos[k] + ah[k] - vec[k] / 2 + s * v1[k] - n[k] * d / 2;
      emit(e, d, pos, n);
    }
  }
}

AW_DEV void c_sphere_sphere(const float* p1, float r1, const float* p2, float r2, float margin, Emit& e) {
  float dif[3];
  sub3(dif, p2, p1);
  float cd = norm3(dif);
  float dist = cd - r1 - r2;
  if (dist > margin + DEC_EPS) return;   // candidates near the margin: decided in fp64
  float n[3] = {1, 0, 0};
  if (cd > MINVAL) scl3(n, dif, 1.0f / cd);
  float pos[3];
  for (int k = 0; k < 3; k++) pos[k] = p1[k] + n[k] * (r1 + dist / 2);
  emit(e, dist, pos, n);
}

AW_DEV void c_sphere_capsule(const GV& a, const GV& b, float margin, Emit& e) {
  float ax[3], dif[3], q[3];
  axis_of(ax, b.mat, 2);
  sub3(dif, a.pos, b.pos);
  float t = clampf(dot3(dif, ax), -b.size[1], b.size[1]);
  for (int k = 0; k < 3; k++) q[k] = b.pos[k] + ax[k] * t;
  c_sphere_sphere(a.pos, a.size[0], q, b.size[0], margin, e);
}

template <class T> AW_DEV T clampt(T x, T lo, T hi) { return x < lo ? lo : (x > hi ? hi : x); }
template <class T>
AW_DEV void seg_seg(const T* p1, const T* d1, const T* p2, const T* d2, T* c1, T* c2) {
  T r[3];
  sub3(r, p1, p2);
  T a = dot3(d1, d1), ee = dot3(d2, d2), f = dot3(d2, r);
  T s, t;
  const T mv = T(MINVAL), z = T(0), o = T(1);
  if (a <= mv && ee <= mv) { s = t = 0; }
  else if (a <= mv) { s = 0; t = clampt(f / ee, z, o); }
  else {
    T cc = dot3(d1, r);
    if (ee <= mv) { t = 0; s = clampt(-cc / a, z, o); }
    else {
      T b = dot3(d1, d2), den = a * ee - b * b;
      s = den > mv ? clampt((b * f - cc * ee) / den, z, o) : z;
      t = (b * s + f) / ee;
      if (t < 0) { t = 0; s = clampt(-cc / a, z, o); }
      else if (t > 1) { t = 1; s = clampt((b - cc) / a, z, o); }
    }
  }
  for (int k = 0; k < 3; k++) { c1[k] = p1[k] + d1[k] * s; c2[k] = p2[k] + d2[k] * t; }
}

AW_DEV void c_capsule_capsule(const GV& a, const GV& b, float margin, Emit& e) {
  float a1[3], a2[3], s1[3], s2[3], d1[3], d2[3], c1[3], c2[3];
  axis_of(a1, a.mat, 2);
  axis_of(a2, b.mat, 2);
  for (int k = 0; k < 3; k++) {
    s1[k] = a.pos[k] - a1[k] * a.size[1]; d1[k] = 2 * a1[k] * a.size[1];
    s2[k] = b.pos[k] - a2[k] * b.size[1]; d2[k] = 2 * a2[k] * b.size[1];
  }
  seg_seg<float>(s1, d1, s2, d2, c1, c2);
  c_sphere_sphere(c1, a.size[0], c2, b.size[0], margin, e);
}

AW_DEV void c_sphere_box_pt(const float* p, float r, const GV& b, float margin, Emit& e, float t = 0.f) {
  float dif[3], loc[3], cl[3];
  sub3(dif, p, b.pos);
  mulmtv3(loc, b.mat, dif);
  bool inside = true;
  for (int k = 0; k < 3; k++) {
    cl[k] = clampf(loc[k], -b.size[k], b.size[k]);
    if (fabsf(loc[k]) > b.size[k]) inside = false;
  }
  float n[3], dist;
  if (!inside) {
    float dl[3], dw[3];
    sub3(dl, cl, loc);
    float dd = norm3(dl);
    dist = dd - r;
    if (dist > margin + DEC_EPS) return;   // candidates near the margin: decided in fp64
    mulmv3(dw, b.mat, dl);
    scl3(n, dw, 1.0f / dd);
  } else {
    int kmin = 0;
    float pen = b.size[0] - fabsf(loc[0]);
    for (int k = 1; k < 3; k++) {
      float pk = b.size[k] - fabsf(loc[k]);
      if (pk < pen) { pen = pk; kmin = k; }
    }
    float nl[3];
#pragma unroll
    for (int k = 0; k < 3; k++) nl[k] = k == kmin ? (loc[k] >= 0 ? -1.0f : 1.0f) : 0.f;
    mulmv3(n, b.mat, nl);
    dist = -pen - r;
  }
  float pos[3];
  for (int k = 0; k < 3; k++) pos[k] = p[k] + n[k] * (r + dist / 2);
  emit(e, dist, pos, n, t);
}

// signed distance of the box-frame point c + t u to the box of half-sizes s (< 0 inside)
AW_DEV float seg_box_f(const float* c, const float* u, const float* s, float t) {
  float out = 0.f, mx = -1e30f;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float q = fabsf(fmaf(t, u[k], c[k])) - s[k];
    const float qp = fmaxf(q, 0.f);
    out = fmaf(qp, qp, out);
    mx = fmaxf(mx, q);
  }
  return sqrtf(out) + fminf(mx, 0.f);
}

// capsule (a) vs box (b): mjc_CapsuleBox's construction, the fp64 statement is
// oracle/collide.cc capsule_box (same steps, same candidates, same tie rules):
//  1. t* = exact minimiser of the convex piecewise signed distance along the segment: ends,
//     slab / zero crossings, stationary points of the 2- and 3-coordinate outside pieces,
//     crossings of two inside pieces; ties to the smallest t;
//  2. two or three coordinates outside at t* -> edge / corner -> one contact; otherwise face k;
//  3. face: the segment part over face k is [lo, hi]; t* moves to the nearer end when that end
//     is as close (parallel capsule) and the other end is the second point; both sphere-box
//     contacts within the margin (flat on a face: two contacts at the clipped ends).
// Step 1's candidates, 43 of them, spread over the 16 lanes of a DPP row (lane gl of the row
// takes candidates gl, gl + 16, gl + 32): 0, 1 the segment ends; 2..10 the slab / zero crossings
// of coordinate j = (k - 2) / 3; 11..30 the stationary points of the outside pieces with two or
// three coordinates outside (code digits cd_j: 0 inside, 1 above +s_j, 2 below -s_j); 31..42
// the crossings of two inside pieces (i, j, signs).  The minimiser is the lexicographic
// minimum of (f, t) over the candidates -- the sequential scan's "smaller f, ties to smaller
// t" -- so the row reduction below returns the scan's t* whatever the evaluation order.
// Three-digit codes with >= 2 nonzero digits, 6 bits each (cd0 | cd1 << 2 | cd2 << 4), in the
// scan's code order: codes 4 5 7 8 10..17 19..26 of 0..26.
constexpr unsigned long long CAPBOX_CODES_LO =
    0x05ull | 0x06ull << 6 | 0x09ull << 12 | 0x0Aull << 18 | 0x11ull << 24 | 0x12ull << 30 | 0x14ull << 36 |
    0x15ull << 42 | 0x16ull << 48 | 0x18ull << 54;
constexpr unsigned long long CAPBOX_CODES_HI =
    0x19ull | 0x1Aull << 6 | 0x21ull << 12 | 0x22ull << 18 | 0x24ull << 24 | 0x25ull << 30 | 0x26ull << 36 |
    0x28ull << 42 | 0x29ull << 48 | 0x2Aull << 54;
static_assert(CAPBOX_CODES_LO == 0x616554491289185ull && CAPBOX_CODES_HI == 0xaa9a269648a1699ull, "code table");
AW_DEV float sel3(const float* v, int j) { return j == 0 ? v[0] : (j == 1 ? v[1] : v[2]); }
AW_DEV void capbox_tstar_row(const float* c, const float* u, const float* sz, float h, int gl, float& best_f,
                             float& best_t) {
  float bf = 3.402823466e38f, bt = 3.402823466e38f;
#pragma unroll
  for (int rd = 0; rd < 3; rd++) {
    const int k = gl + 16 * rd;
    float t = -h;
    bool ok = k < 43;
    if (k == 1) {
      t = h;
    } else if (k >= 2 && k < 11) {
      const int j = (k - 2) / 3, w = (k - 2) - 3 * j;
      const float uj = sel3(u, j), cj = sel3(c, j), sj = sel3(sz, j);
      ok = fabsf(uj) > 1e-12f;
      const float iu = 1.0f / uj;
      t = (w == 0 ? sj - cj : (w == 1 ? -sj - cj : -cj)) * iu;
    } else if (k >= 11 && k < 31) {
      const int q = k - 11;
      const int code = (int)(((q < 10 ? CAPBOX_CODES_LO : CAPBOX_CODES_HI) >> (6 * (q < 10 ? q : q - 10))) & 63ull);
      float nu = 0.f, de = 0.f;
#pragma unroll
      for (int j = 0; j < 3; j++) {
        const int cdj = (code >> (2 * j)) & 3;
        const float sg = cdj == 1 ? 1.f : -1.f;
        const float tn = (sz[j] * sg - c[j]) * u[j], td = u[j] * u[j];
        nu = cdj ? nu + tn : nu;
        de = cdj ? de + td : de;
      }
      ok = de > 1e-24f;
      t = nu / de;
    } else if (k >= 31 && k < 43) {
      const int q = k - 31, pr = q >> 2, sc = q & 3;
      const int i = pr == 2 ? 1 : 0, j = pr == 0 ? 1 : 2;
      const float si = (sc & 1) ? -1.f : 1.f, sj = (sc & 2) ? -1.f : 1.f;
      const float ui = sel3(u, i), uj = sel3(u, j), ci = sel3(c, i), cj = sel3(c, j);
      const float den = si * ui - sj * uj;
      ok = fabsf(den) > 1e-12f;
      t = (sel3(sz, i) - sel3(sz, j) - si * ci + sj * cj) / den;
    }
    t = fminf(fmaxf(t, -h), h);
    const float f = ok ? seg_box_f(c, u, sz, t) : 3.402823466e38f;
    const bool take = ok && (f < bf || (f == bf && t < bt));
    bf = take ? f : bf;
    bt = take ? t : bt;
  }
  // lexicographic (f, t) minimum over the 16-lane row: xor 1, xor 2, half-row and row mirrors
  auto step = [&](float pf, float pt) {
    const bool take = pf < bf || (pf == bf && pt < bt);
    bf = take ? pf : bf;
    bt = take ? pt : bt;
  };
  step(dpp_f<0xB1>(0.f, bf), dpp_f<0xB1>(0.f, bt));
  step(dpp_f<0x4E>(0.f, bf), dpp_f<0x4E>(0.f, bt));
  step(dpp_f<0x141>(0.f, bf), dpp_f<0x141>(0.f, bt));
  step(dpp_f<0x140>(0.f, bf), dpp_f<0x140>(0.f, bt));
  best_f = bf;
  best_t = bt;
}

// one capsule-box pair on the 16 lanes of a DPP row (gl = lane in the row); every lane of the
// row computes the same contacts, the row's lane 0 emits them
AW_DEV void c_capsule_box(const GV& a, const GV& b, float margin, Emit& e, int gl) {
  float ax[3];
  axis_of(ax, a.mat, 2);
  const float h = a.size[1], r = a.size[0];
  const float* sz = b.size;
  float dif[3], c[3], u[3];
  sub3(dif, a.pos, b.pos);
  mulmtv3(c, b.mat, dif);
  mulmtv3(u, b.mat, ax);
  float best_f, best_t;
  capbox_tstar_row(c, u, sz, h, gl, best_f, best_t);
  if (gl != 0) return;
  float ts = best_t;
  int nout = 0, kout = 0, kin = 0;
  float pen = 1e30f;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float q = fabsf(fmaf(ts, u[k], c[k]));
    if (q > sz[k]) { nout++; kout = k; }
    if (sz[k] - q < pen) { pen = sz[k] - q; kin = k; }
  }
  float t2 = ts;
  bool second = false;
  if (nout <= 1) {
    const int fk = nout == 1 ? kout : kin;
    float lo = -h, hi = h;
#pragma unroll
    for (int j = 0; j < 3; j++) {
      if (j == fk) continue;
      if (fabsf(u[j]) > 1e-12f) {
        float t0 = (-sz[j] - c[j]) / u[j], t1 = (sz[j] - c[j]) / u[j];
        const float mn = fminf(t0, t1), mx = fmaxf(t0, t1);
        lo = fmaxf(lo, mn);
        hi = fminf(hi, mx);
      } else if (fabsf(c[j]) > sz[j]) {
        hi = lo - 1.f;
      }
    }
    if (hi > lo) {
      const float tol = 1e-6f * (h + r);
      const float near_end = (ts - lo <= hi - ts) ? lo : hi, far_end = near_end == lo ? hi : lo;
      if (near_end != ts && seg_box_f(c, u, sz, near_end) <= best_f + tol) ts = near_end;
      t2 = far_end;
      second = fabsf(t2 - ts) > 1e-6f * h;
    }
  }
  float p[3];
  for (int k = 0; k < 3; k++) p[k] = a.pos[k] + ax[k] * ts;
  c_sphere_box_pt(p, r, b, margin, e, ts);
  if (second) {
    for (int k = 0; k < 3; k++) p[k] = a.pos[k] + ax[k] * t2;
    c_sphere_box_pt(p, r, b, margin, e, t2);
  }
}

AW_DEV void c_box_box(const GV& A, const GV& B, float margin, Emit& e) {
  float a[3][3], b[3][3], t[3];
  for (int k = 0; k < 3; k++) { axis_of(a[k], A.mat, k); axis_of(b[k], B.mat, k); }
  sub3(t, B.pos, A.pos);
  float best = -1e30f, bestn[3] = {0, 0, 0};
  int bestk = -1;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    float L[3];
    if (k < 3) copy3(L, a[k]);
    else if (k < 6) copy3(L, b[k - 3]);
    else {
      cross3(L, a[(k - 6) / 3], b[(k - 6) % 3]);
      float ln = norm3(L);
      if (ln < 1e-6f) continue;
      scl3(L, L, 1.0f / ln);
    }
    float ra = A.size[0] * fabsf(dot3(L, a[0])) + A.size[1] * fabsf(dot3(L, a[1])) + A.size[2] * fabsf(dot3(L, a[2]));
    float rb = B.size[0] * fabsf(dot3(L, b[0])) + B.size[1] * fabsf(dot3(L, b[1])) + B.size[2] * fabsf(dot3(L, b[2]));
    float tl = dot3(t, L);
    float sep = fabsf(tl) - ra - rb;
    if (sep > margin) return;
    float bias = k < 6 ? 0.f : 1e-6f;
    if (sep > best + bias) {
      best = sep; bestk = k;
      copy3(bestn, L);
      if (tl < 0) scl3(bestn, bestn, -1);
    }
  }
  if (bestk < 0) return;
  if (bestk < 6) {
    // face contact; every axis / size choice is a select so all arrays stay in VGPRs
    const bool refA = bestk < 3;
    const int fk = refA ? bestk : bestk - 3;
    const int ru = fk == 2 ? 0 : fk + 1;
    float Rpos[3], Ipos[3], Rs[3], Is[3], rN[3], rU[3], rV[3];
    float ra[3][3], ia[3][3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
      Rpos[k] = refA ? A.pos[k] : B.pos[k];
      Ipos[k] = refA ? B.pos[k] : A.pos[k];
      Rs[k] = refA ? A.size[k] : B.size[k];
      Is[k] = refA ? B.size[k] : A.size[k];
#pragma unroll
      for (int c = 0; c < 3; c++) { ra[k][c] = refA ? a[k][c] : b[k][c]; ia[k][c] = refA ? b[k][c] : a[k][c]; }
    }
    const int rvv = (fk + 2) % 3;
#pragma unroll
    for (int c = 0; c < 3; c++) {
      rN[c] = fk == 0 ? ra[0][c] : (fk == 1 ? ra[1][c] : ra[2][c]);
      rU[c] = ru == 0 ? ra[0][c] : (ru == 1 ? ra[1][c] : ra[2][c]);
      rV[c] = rvv == 0 ? ra[0][c] : (rvv == 1 ? ra[1][c] : ra[2][c]);
    }
    const float hF = fk == 0 ? Rs[0] : (fk == 1 ? Rs[1] : Rs[2]);
    const float hu = ru == 0 ? Rs[0] : (ru == 1 ? Rs[1] : Rs[2]);
    const float hv = rvv == 0 ? Rs[0] : (rvv == 1 ? Rs[1] : Rs[2]);
    float nr[3];
    copy3(nr, bestn);
    if (!refA) scl3(nr, nr, -1);
    const float sg = dot3(nr, rN) > 0 ? 1.f : -1.f;
    float fc[3];
#pragma unroll
    for (int k = 0; k < 3; k++) fc[k] = Rpos[k] + rN[k] * sg * hF;
    int ik = 0;
    float imin = 1e30f, isg = 1;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      float dd = dot3(ia[k], nr);
      if (dd < imin) { imin = dd; ik = k; isg = 1; }
      if (-dd < imin) { imin = -dd; ik = k; isg = -1; }
    }
    const int iu = ik == 2 ? 0 : ik + 1, iv = (ik + 2) % 3;
    float iN[3], iU[3], iV[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {
      iN[c] = ik == 0 ? ia[0][c] : (ik == 1 ? ia[1][c] : ia[2][c]);
      iU[c] = iu == 0 ? ia[0][c] : (iu == 1 ? ia[1][c] : ia[2][c]);
      iV[c] = iv == 0 ? ia[0][c] : (iv == 1 ? ia[1][c] : ia[2][c]);
    }
    const float sIk = ik == 0 ? Is[0] : (ik == 1 ? Is[1] : Is[2]);
    const float su = iu == 0 ? Is[0] : (iu == 1 ? Is[1] : Is[2]);
    const float sv = iv == 0 ? Is[0] : (iv == 1 ? Is[1] : Is[2]);
    float inn[3], ic[3];
    scl3(inn, iN, isg);
#pragma unroll
    for (int k = 0; k < 3; k++) ic[k] = Ipos[k] + inn[k] * sIk;
    float P[4][3], pu[4], pv[4];
    const float cs[4][2] = {{1, 1}, {-1, 1}, {-1, -1}, {1, -1}};
#pragma unroll
    for (int q = 0; q < 4; q++) {
#pragma unroll
      for (int k = 0; k < 3; k++) P[q][k] = ic[k] + iU[k] * cs[q][0] * su + iV[k] * cs[q][1] * sv;
      float dv[3];
      sub3(dv, P[q], fc);
      pu[q] = dot3(dv, rU);
      pv[q] = dot3(dv, rV);
    }
    auto em = [&](const float* p) {
      float dv[3];
      sub3(dv, p, fc);
      float dist = dot3(dv, nr);
      if (dist > margin) return;
      float pos[3];
      for (int k = 0; k < 3; k++) pos[k] = p[k] - nr[k] * dist / 2;
      emit(e, dist, pos, bestn);
    };
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (fabsf(pu[q]) <= hu && fabsf(pv[q]) <= hv) em(P[q]);
    float den = dot3(nr, inn);
    if (fabsf(den) > 1e-12f) {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        float Q[3], dq[3], Qp[3];
        for (int k = 0; k < 3; k++) Q[k] = fc[k] + rU[k] * cs[q][0] * hu + rV[k] * cs[q][1] * hv;
        sub3(dq, ic, Q);
        float tt = dot3(dq, inn) / den;
        for (int k = 0; k < 3; k++) Qp[k] = Q[k] + nr[k] * tt;
        sub3(dq, Qp, ic);
        if (fabsf(dot3(dq, iU)) <= su && fabsf(dot3(dq, iV)) <= sv) em(Qp);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int q2 = (q + 1) & 3;
      float du = pu[q2] - pu[q], dv = pv[q2] - pv[q];
#pragma unroll
      for (int side = 0; side < 4; side++) {
        float tt;
        if (side < 2) {
          float U = side == 0 ? hu : -hu;
          if (fabsf(du) < 1e-12f) continue;
          tt = (U - pu[q]) / du;
          if (!(tt > 0 && tt < 1)) continue;
          if (fabsf(pv[q] + tt * dv) > hv) continue;
        } else {
          float V = side == 2 ? hv : -hv;
          if (fabsf(dv) < 1e-12f) continue;
          tt = (V - pv[q]) / dv;
          if (!(tt > 0 && tt < 1)) continue;
          if (fabsf(pu[q] + tt * du) > hu) continue;
        }
        float X[3];
        for (int k = 0; k < 3; k++) X[k] = P[q][k] + (P[q2][k] - P[q][k]) * tt;
        em(X);
      }
    }
    return;
  }
  const int ea = (bestk - 6) / 3, eb = (bestk - 6) % 3;
  float pa[3], pb[3];
  copy3(pa, A.pos);
  copy3(pb, B.pos);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    if (k != ea) {
      float s1 = dot3(a[k], bestn) > 0 ? 1.f : -1.f;
      for (int q = 0; q < 3; q++) pa[q] += a[k][q] * s1 * A.size[k];
    }
    if (k != eb) {
      float s2 = dot3(b[k], bestn) > 0 ? -1.f : 1.f;
      for (int q = 0; q < 3; q++) pb[q] += b[k][q] * s2 * B.size[k];
    }
  }
  float aE[3], bE[3];
  const float sa = ea == 0 ? A.size[0] : (ea == 1 ? A.size[1] : A.size[2]);
  const float sb = eb == 0 ? B.size[0] : (eb == 1 ? B.size[1] : B.size[2]);
#pragma unroll
  for (int q = 0; q < 3; q++) {
    aE[q] = ea == 0 ? a[0][q] : (ea == 1 ? a[1][q] : a[2][q]);
    bE[q] = eb == 0 ? b[0][q] : (eb == 1 ? b[1][q] : b[2][q]);
  }
  float s1[3], d1[3], s2[3], d2[3], c1[3], c2[3], pos[3];
  for (int q = 0; q < 3; q++) {
    s1[q] = pa[q] - aE[q] * sa; d1[q] = 2 * aE[q] * sa;
    s2[q] = pb[q] - bE[q] * sb; d2[q] = 2 * bE[q] * sb;
  }
  seg_seg(s1, d1, s2, d2, c1, c2);
  for (int q = 0; q < 3; q++) pos[q] = 0.5f * (c1[q] + c2[q]);
  emit(e, best, pos, bestn);
}

// ---------------------------------------------------------------------------------------
// MPR (libccd ccdMPRPenetration), supports inflated by margin/2 (mjccd_support)
namespace mpr {
// Run in fp64 (T = double) on fp64 geometry (geom64): MuJoCo's libccd is double, and its contact
// point on line / face contacts (a cylinder lying on a box) moves between the ends of the line
// under 1e-7 rad of rotation, i.e. under fp32 kinematics.  (An fp32 path with fp32 inputs measured
// 81 % teacher-forced parity on pen and 99.4 % on hammer's C3 run; it was removed in round 3.)
//
// Operation order: libccd's, as the oracle states it (oracle/collide.cc namespace mpr) -- every
// product and sum rounded separately (no fused multiply-add: the pragma below holds for the MPR
// code and its local vector helpers), normalisation as 1 / sqrt(|v|^2) with the correctly rounded
// fp64 sqrt and divide, the cylinder's radial support as ld / |ld_xy| * r.  On identical inputs the
// kernel's portal, depth, normal and point are then bitwise the oracle's -- including the line /
// face contacts (a cylinder lying on a box), whose point is ill-conditioned along the line
// (tests/test_colliders.py test_gpu_mpr_pairs_match_oracle).
// every function body of this namespace starts with MPR_EXACT: no contraction in that scope
#ifdef AW_MPR_FAST
#define MPR_EXACT
#else
#define MPR_EXACT _Pragma("clang fp contract(off)")
#endif
// libccd's CCD_EPS of the matching build: DBL_EPSILON (MuJoCo's double build) / FLT_EPSILON
template <class T> constexpr T EPS_T = sizeof(T) == 8 ? T(2.220446049250313e-16) : T(1.1920928955078125e-07);
template <class T> struct GVdT {
  T pos[3], mat[9], size[3];
  int type;
};
// local vector helpers (compiled under the pragma above: no contraction)
template <class T> AW_DEV T dot3(const T* a, const T* b) { MPR_EXACT return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
template <class T> AW_DEV void cross3(T* r, const T* a, const T* b) { MPR_EXACT
  T t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
template <class T> AW_DEV void sub3(T* r, const T* a, const T* b) { MPR_EXACT r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2]; }
template <class T> AW_DEV void add3(T* r, const T* a, const T* b) { MPR_EXACT r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2]; }
template <class T> AW_DEV void scl3(T* r, const T* a, T s) { MPR_EXACT r[0] = a[0] * s; r[1] = a[1] * s; r[2] = a[2] * s; }
template <class T> AW_DEV void copy3(T* r, const T* a) { MPR_EXACT r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; }
template <class T> AW_DEV void mulmv3(T* r, const T* m, const T* v) { MPR_EXACT
  T t0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  T t1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  T t2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
template <class T> AW_DEV void mulmtv3(T* r, const T* m, const T* v) { MPR_EXACT
  T t0 = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  T t1 = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  T t2 = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
template <class T> AW_DEV bool is_zero(T x) { MPR_EXACT return fabs(x) < EPS_T<T>; }
template <class T> AW_DEV bool eq(T a, T b) { MPR_EXACT
  T ab = fabs(a - b);
  if (ab < EPS_T<T>) return true;
  T fa = fabs(a), fb = fabs(b);
  return fb > fa ? ab < EPS_T<T> * fb : ab < EPS_T<T> * fa;
}
template <class T> AW_DEV bool veq(const T* a, const T* b) { MPR_EXACT return eq(a[0], b[0]) && eq(a[1], b[1]) && eq(a[2], b[2]); }
template <class T> AW_DEV void vnorm(T* v) { MPR_EXACT
#ifdef AW_MPR_FAST
  T k = rsqrt_fast(dot3(v, v));
#else
  T k = T(1.0) / sqrt(dot3(v, v));   // ccdVec3Normalize
#endif
  scl3(v, v, k);
}
template <class T> AW_DEV T sgn(T x) { MPR_EXACT return x < 0 ? -T(1.0) : (x > 0 ? T(1.0) : T(0.0)); }

template <class T> struct SupT { T v[3], v1[3], v2[3]; };

// support point of a primitive in direction dir (world), inflated by margin / 2.  Branch-free:
// the lanes of one MPR round hold pairs of different geom types, and a type switch would run
// every shape's branch in turn.
template <class T> AW_DEV void gsupport(T* res, const GVdT<T>& g, const T* dir, T margin) { MPR_EXACT
  T ld[3], r[3];
  mulmtv3(ld, g.mat, dir);
  const T* s = g.size;
  const bool box = g.type == GEOM_BOX, cyl = g.type == GEOM_CYLINDER, cap = g.type == GEOM_CAPSULE;
  const bool round = g.type == GEOM_SPHERE || cap;
  const T sg0 = sgn(ld[0]), sg1 = sgn(ld[1]), sg2 = sgn(ld[2]);
#ifdef AW_MPR_FAST
  const T t2 = ld[0] * ld[0] + ld[1] * ld[1];   // the cylinder's radial direction: |ld_xy| > MINVAL
  const T ci = t2 > T(MINVAL) * T(MINVAL) ? s[0] * rsqrt_fast(t2) : T(0.0);
  const T cx = ld[0] * ci, cy = ld[1] * ci;
  const T rz = fma(ld[2], s[0], cap ? sg2 * s[1] : T(0.0));
#else
  // the oracle's (mjccd_support's) order: cylinder ld / |ld_xy| * r, capsule ld r + sign h
  const T tmp = sqrt(ld[0] * ld[0] + ld[1] * ld[1]);
  const bool rad = tmp > T(MINVAL);
  const T cx = rad ? ld[0] / tmp * s[0] : T(0.0), cy = rad ? ld[1] / tmp * s[0] : T(0.0);
  const T rz = ld[2] * s[0] + (cap ? sg2 * s[1] : T(0.0));
#endif
  r[0] = box ? sg0 * s[0] : (cyl ? cx : (round ? ld[0] * s[0] : T(0.0)));
  r[1] = box ? sg1 * s[1] : (cyl ? cy : (round ? ld[1] * s[0] : T(0.0)));
  r[2] = box ? sg2 * s[2] : (cyl ? sg2 * s[1] : (round ? rz : T(0.0)));
  for (int k = 0; k < 3; k++) r[k] += ld[k] * margin / 2;
  mulmv3(res, g.mat, r);
  add3(res, res, g.pos);
}

// two lanes per pair (lane 2p: the pair's first geom, lane 2p + 1: its second): each lane holds only
// its own geom and evaluates its own support function; the partner's point arrives by a DPP swap
// within the lane pair, and both lanes run the rest of MPR identically -- the same arithmetic as one
// lane evaluating both supports, half the support work on the chain and half the geometry
// registers (r04s A/B: -1.9 % random, -0.4 % DAPG)
AW_DEV double swap_pair(double x) { MPR_EXACT
  const long long b = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_update_dpp((int)b, (int)b, 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(b >> 32), (int)(b >> 32), 0xB1, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
template <class T> struct Ctx { const GVdT<T>* own; int half; T opos[3]; T margin, tol; int maxit; };

template <class T> AW_DEV void support(const Ctx<T>& c, const T* dir, SupT<T>& s) { MPR_EXACT
  T d[3], r[3], o[3];
  scl3(d, dir, c.half ? T(-1) : T(1));
  gsupport(r, *c.own, d, c.margin);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    o[k] = swap_pair(r[k]);
    s.v1[k] = c.half ? o[k] : r[k];
    s.v2[k] = c.half ? r[k] : o[k];
  }
  sub3(s.v, s.v1, s.v2);
}
// the portal is kept as four named vertices (no array) so every vertex stays in VGPRs
template <class T> struct PortalT { SupT<T> p0, p1, p2, p3; };
// element-wise copy (a whole-struct copy becomes a memcpy that keeps the portal in scratch)
template <class T> AW_DEV void setsup(SupT<T>& d, const SupT<T>& s) { MPR_EXACT
#pragma unroll
  for (int k = 0; k < 3; k++) { d.v[k] = s.v[k]; d.v1[k] = s.v1[k]; d.v2[k] = s.v2[k]; }
}

template <class T> AW_DEV void portal_dir(const PortalT<T>& P, T* dir) { MPR_EXACT
  T a[3], b[3];
  sub3(a, P.p2.v, P.p1.v);
  sub3(b, P.p3.v, P.p1.v);
  cross3(dir, a, b);
  vnorm(dir);
}
template <class T> AW_DEV bool reach_tol(const PortalT<T>& P, const SupT<T>& v4, const T* dir, T tol) { MPR_EXACT
  T dv1 = dot3(P.p1.v, dir), dv2 = dot3(P.p2.v, dir), dv3 = dot3(P.p3.v, dir), dv4 = dot3(v4.v, dir);
  T d1 = fmin(fmin(dv4 - dv1, dv4 - dv2), dv4 - dv3);
  return eq(d1, tol) || d1 < tol;
}
template <class T> AW_DEV void selsup(SupT<T>& d, bool c, const SupT<T>& s) { MPR_EXACT
#pragma unroll
  for (int k = 0; k < 3; k++) {
    d.v[k] = c ? s.v[k] : d.v[k]; d.v1[k] = c ? s.v1[k] : d.v1[k]; d.v2[k] = c ? s.v2[k] : d.v2[k];
  }
}
// branch-free vertex replacement: conditional struct stores through a selected pointer would
// pin the portal in scratch
template <class T> AW_DEV void expand(PortalT<T>& P, const SupT<T>& v4) { MPR_EXACT
  T v4v0[3];
  cross3(v4v0, v4.v, P.p0.v);
  const bool a1 = dot3(P.p1.v, v4v0) > 0;
  const bool a2 = dot3(P.p2.v, v4v0) > 0;
  const bool a3 = dot3(P.p3.v, v4v0) > 0;
  selsup(P.p1, (a1 && a2) || (!a1 && !a3), v4);
  selsup(P.p3, a1 && !a2, v4);
  selsup(P.p2, !a1 && a3, v4);
}
template <class T> AW_DEV int discover(const Ctx<T>& c, PortalT<T>& P) { MPR_EXACT
  T dir[3], va[3], vb[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    P.p0.v1[k] = c.half ? c.opos[k] : c.own->pos[k];
    P.p0.v2[k] = c.half ? c.own->pos[k] : c.opos[k];
  }
  sub3(P.p0.v, P.p0.v1, P.p0.v2);
  const T zero[3] = {0, 0, 0};
  if (veq(P.p0.v, zero)) P.p0.v[0] += EPS_T<T> * 10;
  scl3(dir, P.p0.v, T(-1));
  vnorm(dir);
  support(c, dir, P.p1);
  T d = dot3(P.p1.v, dir);
  if (is_zero(d) || d < 0) return -1;
  cross3(dir, P.p0.v, P.p1.v);
  if (is_zero(dot3(dir, dir))) return veq(P.p1.v, zero) ? 1 : 2;
  vnorm(dir);
  support(c, dir, P.p2);
  d = dot3(P.p2.v, dir);
  if (is_zero(d) || d < 0) return -1;
  sub3(va, P.p1.v, P.p0.v);
  sub3(vb, P.p2.v, P.p0.v);
  cross3(dir, va, vb);
  vnorm(dir);
  {
    const bool sw = dot3(dir, P.p0.v) > 0;
    SupT<T> t;
    setsup(t, P.p1);
    selsup(P.p1, sw, P.p2);
    selsup(P.p2, sw, t);
    if (sw) scl3(dir, dir, T(-1));
  }
  for (int it = 0; it < 1000; it++) {
    support(c, dir, P.p3);
    d = dot3(P.p3.v, dir);
    if (is_zero(d) || d < 0) return -1;
    cross3(va, P.p1.v, P.p3.v);
    d = dot3(va, P.p0.v);
    const bool r2 = d < 0 && !is_zero(d);
    cross3(va, P.p3.v, P.p2.v);
    d = dot3(va, P.p0.v);
    const bool r1 = !r2 && d < 0 && !is_zero(d);
    if (!r2 && !r1) return 0;
    selsup(P.p2, r2, P.p3);
    selsup(P.p1, r1, P.p3);
    sub3(va, P.p1.v, P.p0.v);
    sub3(vb, P.p2.v, P.p0.v);
    cross3(dir, va, vb);
    vnorm(dir);
  }
  return -1;
}
template <class T> AW_DEV int refine(const Ctx<T>& c, PortalT<T>& P) { MPR_EXACT
  T dir[3];
  SupT<T> v4;
  for (int it = 0; it <= c.maxit; it++) {
    portal_dir(P, dir);
    T d = dot3(dir, P.p1.v);
    if (is_zero(d) || d > 0) return 0;
    support(c, dir, v4);
    T d4 = dot3(v4.v, dir);
    if (!(is_zero(d4) || d4 > 0) || reach_tol(P, v4, dir, c.tol)) return -1;
    expand(P, v4);
  }
  return -1;
}
template <class T> AW_DEV T pseg2(const T* P, const T* x0, const T* b, T* w) { MPR_EXACT
  T dd[3], a[3];
  sub3(dd, b, x0);
  sub3(a, x0, P);
  T t = -dot3(a, dd) / dot3(dd, dd);
  const bool lo = t < 0 || is_zero(t), hi = !lo && (t > 1 || eq(t, T(1)));
  T df[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    w[k] = lo ? x0[k] : (hi ? b[k] : x0[k] + dd[k] * t);
    df[k] = w[k] - P[k];
  }
  return dot3(df, df);
}
template <class T> AW_DEV T ptri2(const T* P, const T* x0, const T* B, const T* C, T* w) { MPR_EXACT
  T d1[3], d2[3], a[3];
  sub3(d1, B, x0);
  sub3(d2, C, x0);
  sub3(a, x0, P);
  T v = dot3(d1, d1), ww = dot3(d2, d2), p = dot3(a, d1), q = dot3(a, d2), r = dot3(d1, d2);
  T dd = ww * v - r * r, s, t;
  if (is_zero(dd)) { s = t = -1; }
  else { s = (q * r - ww * p) / dd; t = (-s * r - q) / ww; }
  if ((is_zero(s) || s > 0) && (eq(s, T(1)) || s < 1) && (is_zero(t) || t > 0) && (eq(t, T(1)) || t < 1) &&
      (eq(t + s, T(1)) || t + s < 1)) {
    for (int k = 0; k < 3; k++) w[k] = x0[k] + d1[k] * s + d2[k] * t;
    T df[3];
    sub3(df, w, P);
    return dot3(df, df);
  }
  T w2[3];
  T dist = pseg2(P, x0, B, w);
  T d2s = pseg2(P, x0, C, w2);
  bool take = d2s < dist;
  dist = take ? d2s : dist;
#pragma unroll
  for (int k = 0; k < 3; k++) w[k] = take ? w2[k] : w[k];
  d2s = pseg2(P, B, C, w2);
  take = d2s < dist;
  dist = take ? d2s : dist;
#pragma unroll
  for (int k = 0; k < 3; k++) w[k] = take ? w2[k] : w[k];
  return dist;
}
template <class T> AW_DEV void find_pos(const PortalT<T>& P, T* pos) { MPR_EXACT
  T dir[3], vec[3], b0, b1, b2, b3;
  portal_dir(P, dir);
  cross3(vec, P.p1.v, P.p2.v); b0 = dot3(vec, P.p3.v);
  cross3(vec, P.p3.v, P.p2.v); b1 = dot3(vec, P.p0.v);
  cross3(vec, P.p0.v, P.p1.v); b2 = dot3(vec, P.p3.v);
  cross3(vec, P.p2.v, P.p1.v); b3 = dot3(vec, P.p0.v);
  T sum = b0 + b1 + b2 + b3;
  if (is_zero(sum) || sum < 0) {
    b0 = 0;
    cross3(vec, P.p2.v, P.p3.v); b1 = dot3(vec, dir);
    cross3(vec, P.p3.v, P.p1.v); b2 = dot3(vec, dir);
    cross3(vec, P.p1.v, P.p2.v); b3 = dot3(vec, dir);
    sum = b1 + b2 + b3;
  }
  T inv = T(1.0) / sum;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    T p1 = P.p0.v1[k] * b0 + P.p1.v1[k] * b1 + P.p2.v1[k] * b2 + P.p3.v1[k] * b3;
    T p2 = P.p0.v2[k] * b0 + P.p1.v2[k] * b1 + P.p2.v2[k] * b2 + P.p3.v2[k] * b3;
    pos[k] = T(0.5) * (p1 + p2) * inv;
  }
}
template <class T> AW_DEV int penetration(const Ctx<T>& c, T* depth, T* dir, T* pos) { MPR_EXACT
  PortalT<T> P;
  int res = discover(c, P);
  if (res < 0) return -1;
  if (res == 1) {
    *depth = 0;
    dir[0] = dir[1] = dir[2] = 0;
    for (int k = 0; k < 3; k++) pos[k] = T(0.5) * (P.p1.v1[k] + P.p1.v2[k]);
    return 0;
  }
  if (res == 2) {
    for (int k = 0; k < 3; k++) pos[k] = T(0.5) * (P.p1.v1[k] + P.p1.v2[k]);
    copy3(dir, P.p1.v);
    *depth = sqrt(dot3(dir, dir));
    vnorm(dir);
    return 0;
  }
  if (refine(c, P) < 0) return -1;
  SupT<T> v4;
  T pd[3];
  for (int it = 0;; it++) {
    portal_dir(P, pd);
    support(c, pd, v4);
    if (reach_tol(P, v4, pd, c.tol) || it > c.maxit) {
      const T zero[3] = {0, 0, 0};
      *depth = sqrt(ptri2(zero, P.p1.v, P.p2.v, P.p3.v, dir));
      if (is_zero(*depth)) dir[0] = dir[1] = dir[2] = 0;
      else vnorm(dir);
      find_pos(P, pos);
      return 0;
    }
    expand(P, v4);
  }
}
#undef MPR_EXACT
}  // namespace mpr

// fp64 pose of collidable geom g from the fp64 body frames (stage_kin64), as the oracle's
// mj_local2Global: geom_xpos = xmat[b] geom_pos + xpos[b], geom_xmat = quat2mat(xquat[b] geom_quat)
AW_DEV void geom64(const DModel& m, Env& s, int g, mpr::GVdT<double>& G) {
  const int b = MD(geom_bodyid, g);
  const double* X = kin64(s, b);
  double bq[4] = {X[3], X[4], X[5], X[6]}, bm[9], gp[3], gq[4], q[4], sz[3];
  for (int k = 0; k < 3; k++) { gp[k] = MD(geom_pos64, 3 * g + k); sz[k] = MD(geom_size64, 3 * g + k); }
  for (int k = 0; k < 4; k++) gq[k] = MD(geom_quat64, 4 * g + k);
  if (MD(geom_ovr, g)) { apply_ovr64<3>(m, s, 4, g, gp); apply_ovr64<3>(m, s, 5, g, sz); }
  q2m(bm, bq);
  mulmv3(G.pos, bm, gp);
  for (int k = 0; k < 3; k++) { G.pos[k] += X[k]; G.size[k] = sz[k]; }
  mulq(q, bq, gq);
  q2m(G.mat, q);
  G.type = MD(geom_type, g);
}

// mjc_Convex: MPR in fp64 on fp64 geometry (MuJoCo's double libccd on its double kinematics)
AW_DEV void c_convex64(const DModel& m, const mpr::GVdT<double>& own, int half, double margin, Emit& e) {
  mpr::Ctx<double> ctx{&own, half, {mpr::swap_pair(own.pos[0]), mpr::swap_pair(own.pos[1]), mpr::swap_pair(own.pos[2])},
                       margin, m.mpr_tolerance64, m.mpr_iterations};
  double depth, dir[3], pos[3];
  if (mpr::penetration(ctx, &depth, dir, pos) != 0) return;
  if (dir[0] == 0 && dir[1] == 0 && dir[2] == 0) return;
  const double dist = margin - depth;
  if (dist > margin) return;
  const float pf[3] = {(float)pos[0], (float)pos[1], (float)pos[2]};
  const float df[3] = {(float)dir[0], (float)dir[1], (float)dir[2]};
  if (half) return;
  if (e.out64 && e.cnt < MAXPAIRCON) {
    double* o = e.out64 + 7 * e.cnt;
    o[0] = dist;
    for (int k = 0; k < 3; k++) { o[1 + k] = pos[k]; o[4 + k] = dir[k]; }
  }
  emit(e, (float)dist, pf, df);
}

// fp64 signed distance of contact c of a class-1 / class-2 pair (sphere / capsule pairs, sphere /
// capsule - box) on fp64 geometry (geom64: the kin64 frames of both bodies must be staged), the same
// construction as the fp32 collider that emitted it: sphere-sphere / sphere-capsule / capsule-capsule
// closest points, or the sphere-box distance of the capsule axis point t the collider chose.
AW_DEV double contact_dist64(const DModel& m, Env& s, int c) {
  const int pair = s.con_pair[c];
  const int g1 = MD(cp_g1, pair), g2 = MD(cp_g2, pair);
  mpr::GVdT<double> A, B;
  geom64(m, s, g1, A);
  geom64(m, s, g2, B);
  double ax[3] = {A.mat[2], A.mat[5], A.mat[8]}, p[3], q[3];
  if (B.type != GEOM_BOX) {
    if (A.type == GEOM_SPHERE && B.type == GEOM_SPHERE) {
      copy3(p, A.pos);
      copy3(q, B.pos);
    } else if (A.type == GEOM_SPHERE) {
      const double bx[3] = {B.mat[2], B.mat[5], B.mat[8]};
      double dif[3];
      sub3(dif, A.pos, B.pos);
      const double t = clampt(dot3(dif, bx), -B.size[1], B.size[1]);
      copy3(p, A.pos);
      for (int k = 0; k < 3; k++) q[k] = B.pos[k] + bx[k] * t;
    } else {
      const double bx[3] = {B.mat[2], B.mat[5], B.mat[8]};
      double s1[3], d1[3], s2[3], d2[3];
      for (int k = 0; k < 3; k++) {
        s1[k] = A.pos[k] - ax[k] * A.size[1]; d1[k] = 2 * ax[k] * A.size[1];
        s2[k] = B.pos[k] - bx[k] * B.size[1]; d2[k] = 2 * bx[k] * B.size[1];
      }
      seg_seg<double>(s1, d1, s2, d2, p, q);
    }
    double dif[3];
    sub3(dif, q, p);
    return sqrt(dot3(dif, dif)) - A.size[0] - B.size[0];
  }
  // sphere / capsule (A) - box (B): the sphere at axis point t (0 for a sphere)
  const double t = A.type == GEOM_CAPSULE ? (double)__builtin_bit_cast(float, s.con_efc[c]) : 0.0;
  for (int k = 0; k < 3; k++) p[k] = A.pos[k] + ax[k] * t;
  double dif[3], loc[3];
  sub3(dif, p, B.pos);
  mulmtv3(loc, B.mat, dif);
  bool inside = true;
  double dd = 0.0, pen = 1e300;
  for (int k = 0; k < 3; k++) {
    const double cl = clampt(loc[k], -B.size[k], B.size[k]);
    if (fabs(loc[k]) > B.size[k]) inside = false;
    dd += (cl - loc[k]) * (cl - loc[k]);
    pen = fmin(pen, B.size[k] - fabs(loc[k]));
  }
  return (inside ? -pen : sqrt(dd)) - A.size[0];
}

// Conservative midphase of a sphere / capsule - box pair (class 2): false only when no point of
// the segment can be within the margin of the box -- then the collider emits nothing either.
AW_DEV bool capbox_may_touch(const DModel& m, const Env& s, int pair) {
  const int g1 = MD(cp_g1, pair), g2 = MD(cp_g2, pair);   // g1 the sphere / capsule, g2 the box
  const float h = MD(geom_type, g1) == GEOM_CAPSULE ? s.gsize[g1][1] : 0.f;
  float mat[9], q[4], dif[3], c[3];
  for (int k = 0; k < 4; k++) q[k] = s.gxquat[g2][k];
  q2m(mat, q);
  sub3(dif, s.gxpos[g1], s.gxpos[g2]);
  mulmtv3(c, mat, dif);
  const float zero[3] = {0.f, 0.f, 0.f};
  const float lb = seg_box_f(c, zero, s.gsize[g2], 0.f) - h - s.gsize[g1][0];
  return !(lb > MD(cp_margin, pair) + 1e-4f);
}

// Conservative midphase of a box - box pair (class 3): false only when the first box's bounding
// sphere stays farther than the margin from the second box.
AW_DEV bool boxbox_may_touch(const DModel& m, const Env& s, int pair) {
  const int g1 = MD(cp_g1, pair), g2 = MD(cp_g2, pair);
  float mat[9], q[4], dif[3], c[3];
  for (int k = 0; k < 4; k++) q[k] = s.gxquat[g2][k];
  q2m(mat, q);
  sub3(dif, s.gxpos[g1], s.gxpos[g2]);
  mulmtv3(c, mat, dif);
  const float zero[3] = {0.f, 0.f, 0.f};
  const float lb = seg_box_f(c, zero, s.gsize[g2], 0.f) - norm3(s.gsize[g1]);   // box 1's circumradius
  return !(lb > MD(cp_margin, pair) + 1e-4f);
}

// Conservative midphase of an MPR (cylinder) pair (class 4), on the fp32 frames: false only when
// the geoms provably stay farther apart than the margin.  A cylinder lies inside the capsule of
// its axis segment and radius, so with a box (always the second geom of its pair) the bound is
// the box's signed distance at the first geom's centre less its circumradius; otherwise the
// distance of the two axis segments less both radii (sphere: a point).
AW_DEV bool mpr_may_touch(const DModel& m, const Env& s, int pair) {
  const int g1 = MD(cp_g1, pair), g2 = MD(cp_g2, pair);
  const int t1 = MD(geom_type, g1), t2 = MD(geom_type, g2);
  const float* z1 = s.gsize[g1];
  const float h1 = t1 == GEOM_SPHERE ? 0.f : z1[1];
  float lb;
  if (t2 == GEOM_BOX) {
    float mat[9], q[4], dif[3], c[3];
    for (int k = 0; k < 4; k++) q[k] = s.gxquat[g2][k];
    q2m(mat, q);
    sub3(dif, s.gxpos[g1], s.gxpos[g2]);
    mulmtv3(c, mat, dif);
    const float zero[3] = {0.f, 0.f, 0.f};
    const float circ = t1 == GEOM_CYLINDER ? sqrtf(z1[0] * z1[0] + h1 * h1) : z1[0] + h1;
    lb = seg_box_f(c, zero, s.gsize[g2], 0.f) - circ;
#ifndef AW_NO_MPR_SAT
    if (t1 == GEOM_CYLINDER) {
      // separating axes: the box's three face normals and the cylinder's axis.  A gap between the
      // two shapes' projections on a unit axis is a lower bound on their distance, and unlike the
      // circumscribed sphere it is tight for a flat cylinder beside a face (the hammer's head over
      // the table or the board)
      float q1[4], m1[9], aw[3], a[3];
      for (int k = 0; k < 4; k++) q1[k] = s.gxquat[g1][k];
      q2m(m1, q1);
      for (int k = 0; k < 3; k++) aw[k] = m1[3 * k + 2];
      mulmtv3(a, mat, aw);                      // cylinder axis in the box frame
      const float* B = s.gsize[g2];
      float sep = -1e30f, bext = 0.f;
      for (int k = 0; k < 3; k++) {
        const float ak = fabsf(a[k]);
        const float ext = ak * h1 + z1[0] * sqrtf(fmaxf(0.f, 1.f - ak * ak));   // cylinder along e_k
        sep = fmaxf(sep, fabsf(c[k]) - B[k] - ext);
        bext = fmaf(B[k], ak, bext);                                             // box along the axis
      }
      sep = fmaxf(sep, fabsf(c[0] * a[0] + c[1] * a[1] + c[2] * a[2]) - h1 - bext);
      lb = fmaxf(lb, sep);
    }
#endif
  } else {
    const float* z2 = s.gsize[g2];
    const float h2 = t2 == GEOM_SPHERE ? 0.f : z2[1];
    float q1[4], q2[4], m1[9], m2[9];
    for (int k = 0; k < 4; k++) { q1[k] = s.gxquat[g1][k]; q2[k] = s.gxquat[g2][k]; }
    q2m(m1, q1);
    q2m(m2, q2);
    float s1[3], d1[3], s2[3], d2[3], c1[3], c2[3];
    for (int k = 0; k < 3; k++) {
      s1[k] = s.gxpos[g1][k] - m1[3 * k + 2] * h1; d1[k] = 2.f * m1[3 * k + 2] * h1;
      s2[k] = s.gxpos[g2][k] - m2[3 * k + 2] * h2; d2[k] = 2.f * m2[3 * k + 2] * h2;
    }
    seg_seg(s1, d1, s2, d2, c1, c2);
    float dd[3];
    sub3(dd, c1, c2);
    lb = norm3(dd) - z1[0] - z2[0];
  }
  return !(lb > MD(cp_margin, pair) + 1e-4f);
}

// ---------------------------------------------------------------------------------------
// narrowphase of one pair of collider class C (host: adroit_wave.hip build_model pcls):
// 0 plane-*, 1 sphere/capsule pairs, 2 sphere/capsule-box, 3 box-box, 4 anything with a
// cylinder (MPR).  The class is a template parameter so each class loop carries only its own
// colliders (no divergent merge of every collider's code and registers).
template <int C>
AW_DEV void collide_pair(const DModel& m, Env& s, int pair, int gl = 0) {
  int g1 = MD(cp_g1, pair), g2 = MD(cp_g2, pair);
  Emit e{&s, pair, 0};
  if constexpr (C == 4) {           // every non-plane pair with a cylinder: MPR (mjc_Convex)
    mpr::GVdT<double> own;            // gl: this lane's half of the pair (0: g1, 1: g2)
    geom64(m, s, gl ? g2 : g1, own);
    c_convex64(m, own, gl, MD(cp_margin64, pair), e);
    return;
  }
  GV a, b;
  a.type = MD(geom_type, g1);
  b.type = MD(geom_type, g2);
  for (int k = 0; k < 3; k++) {
    a.pos[k] = s.gxpos[g1][k]; b.pos[k] = s.gxpos[g2][k];
    a.size[k] = s.gsize[g1][k]; b.size[k] = s.gsize[g2][k];
  }
  float margin = MD(cp_margin, pair);   // the bounding-sphere test ran in the broadphase
  {
    float q1[4], q2[4];
    for (int k = 0; k < 4; k++) { q1[k] = s.gxquat[g1][k]; q2[k] = s.gxquat[g2][k]; }
    q2m(a.mat, q1);
    q2m(b.mat, q2);
  }
  if constexpr (C == 0) {
    if (b.type == GEOM_SPHERE) c_plane_sphere(a.pos, a.mat, b.pos, b.size[0], margin, e);
    else if (b.type == GEOM_CAPSULE) c_plane_capsule(a, b, margin, e);
    else if (b.type == GEOM_CYLINDER) c_plane_cylinder(a, b, margin, e);
    else if (b.type == GEOM_BOX) c_plane_box(a, b, margin, e);
  } else if constexpr (C == 1) {
    if (a.type == GEOM_SPHERE && b.type == GEOM_SPHERE) c_sphere_sphere(a.pos, a.size[0], b.pos, b.size[0], margin, e);
    else if (a.type == GEOM_SPHERE) c_sphere_capsule(a, b, margin, e);
    else c_capsule_capsule(a, b, margin, e);
  } else if constexpr (C == 2) {   // one pair per 16-lane row (narrow_class), lane gl of the row
    if (a.type == GEOM_SPHERE) {
      if (gl == 0) c_sphere_box_pt(a.pos, a.size[0], b, margin, e);
    } else {
      c_capsule_box(a, b, margin, e, gl);
    }
  } else {
    c_box_box(a, b, margin, e);
  }
}

}  // namespace aw
