/* collide.cc -- fp64 restatement of MuJoCo 2.1 mj_collision for the Adroit primitive set.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Physics parity with real MuJoCo is unpinned.
 *
 * Pipeline (mj_collision): explicit <pair>s first (their own params), then the static
 * candidate list built by mjcf.py (contype/conaffinity, weld, parent, <exclude> filters),
 * each through a bounding-sphere test (rbound + margin, skipped for planes) and the
 * type-dispatched narrowphase.  Contact params of dynamic pairs are mixed as in
 * mj_contactParam (max condim, max friction, solmix-weighted solref/solimp, max margin/gap).
 *
 * Narrowphase restatement choices (documented in DESIGN.md):
 *   plane-{sphere,capsule,box,cylinder}, sphere-{sphere,capsule,box}, capsule-capsule:
 *     analytic, as the corresponding mjc_* routines;
 *   capsule-box: exact minimum of the signed distance along the axis (golden section) plus
 *     the far endpoint as second contact when within margin (MuJoCo 2.1: analytic, <= 2);
 *   box-box: separating-axis test; face case -> fixed-order candidate points (incident
 *     corners, projected reference corners, edge crossings; <= 8), edge case -> 1 contact;
 *   any pair with a cylinder (and sphere-cylinder): MPR, restating libccd's
 *     ccdMPRPenetration as used by mjc_Convex (1 contact, support inflated by margin/2).
 */
#include <cfloat>
#include <cmath>
#include <cstring>

#include "oracle.h"

namespace orc {

static const num MINVAL = 1e-15;
static const int MAXPAIRCON = 8;

struct GeomView {
  const num* pos;
  const num* mat;
  const num* size;
  int type;
};

static inline void set_contact(Contact* c, num dist, const num* pos, const num* normal) {
  c->dist = dist;
  copy3(c->pos, pos);
  copy3(c->frame, normal);
  c->frame[3] = c->frame[4] = c->frame[5] = 0;
}

static inline void axis_of(num* a, const num* mat, int k) { a[0] = mat[k]; a[1] = mat[3 + k]; a[2] = mat[6 + k]; }

/* ------------------------------------------------------------------------------------- */
static int plane_sphere(const num* p1, const num* m1, const num* p2, num r, num margin, Contact* c) {
  num n[3], dif[3];
  axis_of(n, m1, 2);
  sub3(dif, p2, p1);
  num dist = dot3(n, dif) - r;
  if (dist > margin) return 0;
  num pos[3];
  for (int k = 0; k < 3; k++) pos[k] = p2[k] - n[k] * (r + dist / 2);
  set_contact(c, dist, pos, n);
  return 1;
}

static int plane_capsule(const GeomView& g1, const GeomView& g2, num margin, Contact* c) {
  num ax[3], e[3];
  axis_of(ax, g2.mat, 2);
  int n = 0;
  for (int s = 1; s >= -1; s -= 2) {
    for (int k = 0; k < 3; k++) e[k] = g2.pos[k] + s * ax[k] * g2.size[1];
    n += plane_sphere(g1.pos, g1.mat, e, g2.size[0], margin, c + n);
  }
  return n;
}

static int plane_box(const GeomView& g1, const GeomView& g2, num margin, Contact* c) {
  num n[3], dif[3];
  axis_of(n, g1.mat, 2);
  sub3(dif, g2.pos, g1.pos);
  num dist = dot3(n, dif);
  int cnt = 0;
  for (int i = 0; i < 8; i++) {
    num v[3] = {(i & 1) ? g2.size[0] : -g2.size[0], (i & 2) ? g2.size[1] : -g2.size[1],
                (i & 4) ? g2.size[2] : -g2.size[2]};
    num corner[3];
    mul_mat_vec3(corner, g2.mat, v);
    num ld = dot3(n, corner);
    if (dist + ld > margin || ld > 0) continue;
    num dd = dist + ld, pos[3];
    for (int k = 0; k < 3; k++) pos[k] = corner[k] + g2.pos[k] - n[k] * dd / 2;
    set_contact(c + cnt, dd, pos, n);
    if (++cnt >= 4) return 4;
  }
  return cnt;
}

static int plane_cylinder(const GeomView& g1, const GeomView& g2, num margin, Contact* c) {
  num n[3], axis[3], dif[3], vec[3];
  axis_of(n, g1.mat, 2);
  axis_of(axis, g2.mat, 2);
  sub3(dif, g2.pos, g1.pos);
  num dist0 = dot3(dif, n);
  num prjaxis = dot3(n, axis);
  if (prjaxis > 0) { scl3(axis, axis, -1); prjaxis = -prjaxis; }
  /* radial direction pointing against the normal */
  for (int k = 0; k < 3; k++) vec[k] = axis[k] * prjaxis - n[k];
  num len = norm3(vec);
  if (len < MINVAL) axis_of(vec, g2.mat, 0);
  else scl3(vec, vec, 1.0 / len);
  num r = g2.size[0], h = g2.size[1];
  scl3(vec, vec, r);
  num prjvec = dot3(vec, n);
  num ah[3];
  scl3(ah, axis, h);
  num pa = prjaxis * h;
  int cnt = 0;
  num pos[3], d;
  d = dist0 + pa + prjvec;
  if (d <= margin) {
    for (int k = 0; k < 3; k++) pos[k] = g2.pos[k] + ah[k] + vec[k] - n[k] * d / 2;
    set_contact(c + cnt++, d, pos, n);
  }
  d = dist0 - pa + prjvec;
  if (d <= margin) {
    for (int k = 0; k < 3; k++) pos[k] = g2.pos[k] - ah[k] + vec[k] - n[k] * d / 2;
    set_contact(c + cnt++, d, pos, n);
  }
  d = dist0 + pa - prjvec / 2;
  if (d <= margin) {
    num v1[3];
    cross3(v1, vec, axis);
    scl3(v1, v1, std::sqrt(3.0) / 2);
    for (int s = -1; s <= 1; s += 2) {
      for (int k = 0; k < 3; k++) pos[k] = g2.pos[k] + ah[k] - vec[k] / 2 + s * v1[k] - n[k] * d / 2;
      set_contact(c + cnt++, d, pos, n);
    }
  }
  return cnt;
}

static int sphere_sphere(const num* p1, num r1, const num* p2, num r2, num margin, Contact* c) {
  num dif[3];
  sub3(dif, p2, p1);
  num cd = norm3(dif);
  num dist = cd - r1 - r2;
  if (dist > margin) return 0;
  num n[3] = {1, 0, 0};
  if (cd > MINVAL) scl3(n, dif, 1.0 / cd);
  num pos[3];
  for (int k = 0; k < 3; k++) pos[k] = p1[k] + n[k] * (r1 + dist / 2);
  set_contact(c, dist, pos, n);
  return 1;
}

static void closest_on_segment(num* q, const num* p, const num* center, const num* axis, num h) {
  num dif[3];
  sub3(dif, p, center);
  num t = dot3(dif, axis);
  t = t < -h ? -h : (t > h ? h : t);
  for (int k = 0; k < 3; k++) q[k] = center[k] + axis[k] * t;
}

static int sphere_capsule(const GeomView& g1, const GeomView& g2, num margin, Contact* c) {
  num ax[3], q[3];
  axis_of(ax, g2.mat, 2);
  closest_on_segment(q, g1.pos, g2.pos, ax, g2.size[1]);
  return sphere_sphere(g1.pos, g1.size[0], q, g2.size[0], margin, c);
}

/* closest points between segments p1 + s d1, p2 + t d2 (s,t in [0,1]) -- Ericson 5.1.9 */
static void segment_segment(const num* p1, const num* d1, const num* p2, const num* d2, num* c1, num* c2) {
  num r[3];
  sub3(r, p1, p2);
  num a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
  num s, t;
  if (a <= MINVAL && e <= MINVAL) { s = t = 0; }
  else if (a <= MINVAL) { s = 0; t = f / e; t = t < 0 ? 0 : (t > 1 ? 1 : t); }
  else {
    num cc = dot3(d1, r);
    if (e <= MINVAL) { t = 0; s = -cc / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
    else {
      num b = dot3(d1, d2), denom = a * e - b * b;
      s = denom > MINVAL ? (b * f - cc * e) / denom : 0;
      s = s < 0 ? 0 : (s > 1 ? 1 : s);
      t = (b * s + f) / e;
      if (t < 0) { t = 0; s = -cc / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
      else if (t > 1) { t = 1; s = (b - cc) / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
    }
  }
  for (int k = 0; k < 3; k++) { c1[k] = p1[k] + d1[k] * s; c2[k] = p2[k] + d2[k] * t; }
}

static int capsule_capsule(const GeomView& g1, const GeomView& g2, num margin, Contact* c) {
  num a1[3], a2[3], s1[3], s2[3], d1[3], d2[3], c1[3], c2[3];
  axis_of(a1, g1.mat, 2);
  axis_of(a2, g2.mat, 2);
  for (int k = 0; k < 3; k++) {
    s1[k] = g1.pos[k] - a1[k] * g1.size[1]; d1[k] = 2 * a1[k] * g1.size[1];
    s2[k] = g2.pos[k] - a2[k] * g2.size[1]; d2[k] = 2 * a2[k] * g2.size[1];
  }
  segment_segment(s1, d1, s2, d2, c1, c2);
  return sphere_sphere(c1, g1.size[0], c2, g2.size[0], margin, c);
}

/* sphere (center p, radius r, geom1) vs box (geom2) */
static int sphere_box_pt(const num* p, num r, const GeomView& b, num margin, Contact* c) {
  num dif[3], loc[3];
  sub3(dif, p, b.pos);
  mul_matT_vec3(loc, b.mat, dif);
  bool inside = true;
  num cl[3];
  for (int k = 0; k < 3; k++) {
    cl[k] = loc[k] < -b.size[k] ? -b.size[k] : (loc[k] > b.size[k] ? b.size[k] : loc[k]);
    if (std::fabs(loc[k]) > b.size[k]) inside = false;
  }
  num n[3], dist;
  if (!inside) {
    num dl[3], dw[3];
    sub3(dl, cl, loc);
    num dd = norm3(dl);
    dist = dd - r;
    if (dist > margin) return 0;
    mul_mat_vec3(dw, b.mat, dl);
    scl3(n, dw, 1.0 / dd);
  } else {
    int kmin = 0;
    num pen = b.size[0] - std::fabs(loc[0]);
    for (int k = 1; k < 3; k++) {
      num pk = b.size[k] - std::fabs(loc[k]);
      if (pk < pen) { pen = pk; kmin = k; }
    }
    num nl[3] = {0, 0, 0};
    nl[kmin] = loc[kmin] >= 0 ? -1.0 : 1.0;
    mul_mat_vec3(n, b.mat, nl);
    dist = -pen - r;
  }
  num pos[3];
  for (int k = 0; k < 3; k++) pos[k] = p[k] + n[k] * (r + dist / 2);
  set_contact(c, dist, pos, n);
  return 1;
}

/* Signed distance of the box-frame point c + t u to the box of half-sizes s (< 0 inside). */
static num seg_box_f(const num* c, const num* u, const num* s, num t) {
  num out = 0, mx = -1e300;
  for (int k = 0; k < 3; k++) {
    num q = std::fabs(c[k] + t * u[k]) - s[k];
    num qp = q > 0 ? q : 0;
    out += qp * qp;
    mx = q > mx ? q : mx;
  }
  return std::sqrt(out) + (mx < 0 ? mx : 0);
}

/* Exact minimiser of the (convex, piecewise) signed distance along the segment t in [-h, h]:
 * the minimum lies at an end, at a breakpoint where a coordinate crosses a slab boundary or
 * zero, at the stationary point of an outside piece (2 or 3 coordinates outside, fixed signs),
 * or where two inside pieces |q_i| - s_i = |q_j| - s_j cross.  Every candidate is evaluated;
 * ties go to the smallest t.  (Round 1 ran a 40-step golden-section search.) */
static num seg_box_argmin(const num* c, const num* u, const num* s, num h, num* fmin) {
  num best_t = -h, best_f = seg_box_f(c, u, s, -h);
  auto cand = [&](num t) {
    if (!(t > -h)) t = -h;
    if (t > h) t = h;
    num f = seg_box_f(c, u, s, t);
    if (f < best_f || (f == best_f && t < best_t)) { best_f = f; best_t = t; }
  };
  cand(h);
  for (int j = 0; j < 3; j++)
    if (std::fabs(u[j]) > 1e-12) {
      cand((s[j] - c[j]) / u[j]);
      cand((-s[j] - c[j]) / u[j]);
      cand(-c[j] / u[j]);
    }
  /* outside pieces: coordinate j outside with sign sg_j (code 1: +, 2: -), 0: not outside */
  for (int code = 0; code < 27; code++) {
    int cd[3] = {code % 3, (code / 3) % 3, code / 9};
    int nout = (cd[0] != 0) + (cd[1] != 0) + (cd[2] != 0);
    if (nout < 2) continue;
    num num_ = 0, den = 0;
    for (int j = 0; j < 3; j++)
      if (cd[j]) {
        num sg = cd[j] == 1 ? 1.0 : -1.0;
        num_ += (s[j] * sg - c[j]) * u[j];
        den += u[j] * u[j];
      }
    if (den > 1e-24) cand(num_ / den);
  }
  /* inside crossings */
  for (int i = 0; i < 3; i++)
    for (int j = i + 1; j < 3; j++)
      for (int sc = 0; sc < 4; sc++) {
        num si = (sc & 1) ? -1.0 : 1.0, sj = (sc & 2) ? -1.0 : 1.0;
        num den = si * u[i] - sj * u[j];
        if (std::fabs(den) > 1e-12) cand((s[i] - s[j] - si * c[i] + sj * c[j]) / den);
      }
  *fmin = best_f;
  return best_t;
}

/* capsule (geom1) vs box (geom2), restating mjc_CapsuleBox's construction: the capsule is the
 * segment inflated by its radius, so contacts are sphere-box contacts at chosen segment points.
 * 1. t* = the segment point closest to (deepest in) the box (seg_box_argmin, box frame).
 * 2. Closest box feature at t*: two or three coordinates outside their slabs -> an edge or a
 *    corner -> one contact.  Otherwise a face k (the outside coordinate, or the face of least
 *    penetration when inside).
 * 3. Face: the part of the segment over face k (clipped to the face's other two slabs) is
 *    [lo, hi].  If t* is interior to it and an end is as close (parallel capsule), t* moves to
 *    that end; the second point is the other end.  Both become sphere-box contacts within the
 *    margin: a capsule flat on a face gets two contacts at the clipped ends with the exact
 *    depth, a capsule across an edge one. */
static int capsule_box(const GeomView& g1, const GeomView& g2, num margin, Contact* c) {
  num ax[3], dif[3], cl[3], u[3];
  axis_of(ax, g1.mat, 2);
  const num h = g1.size[1], r = g1.size[0];
  const num* sz = g2.size;
  sub3(dif, g1.pos, g2.pos);
  mul_matT_vec3(cl, g2.mat, dif);
  mul_matT_vec3(u, g2.mat, ax);
  num fmin;
  num ts = seg_box_argmin(cl, u, sz, h, &fmin);
  int nout = 0, kout = 0, kin = 0;
  num pen = 1e300;
  for (int k = 0; k < 3; k++) {
    num q = std::fabs(cl[k] + ts * u[k]);
    if (q > sz[k]) { nout++; kout = k; }
    if (sz[k] - q < pen) { pen = sz[k] - q; kin = k; }
  }
  num t2 = ts;
  bool second = false;
  if (nout <= 1) {
    const int fk = nout == 1 ? kout : kin;
    num lo = -h, hi = h;
    for (int j = 0; j < 3; j++) {
      if (j == fk) continue;
      if (std::fabs(u[j]) > 1e-12) {
        num a = (-sz[j] - cl[j]) / u[j], b = (sz[j] - cl[j]) / u[j];
        if (a > b) std::swap(a, b);
        lo = std::max(lo, a);
        hi = std::min(hi, b);
      } else if (std::fabs(cl[j]) > sz[j]) {
        hi = lo - 1;   /* never over the face */
      }
    }
    if (hi > lo) {
      const num tol = 1e-6 * (h + r);
      num near_end = (ts - lo <= hi - ts) ? lo : hi, far_end = near_end == lo ? hi : lo;
      if (near_end != ts && seg_box_f(cl, u, sz, near_end) <= fmin + tol) ts = near_end;
      t2 = far_end;
      second = std::fabs(t2 - ts) > 1e-6 * h;
    }
  }
  num p[3];
  for (int k = 0; k < 3; k++) p[k] = g1.pos[k] + ax[k] * ts;
  int n = sphere_box_pt(p, r, g2, margin, c);
  if (second) {
    for (int k = 0; k < 3; k++) p[k] = g1.pos[k] + ax[k] * t2;
    n += sphere_box_pt(p, r, g2, margin, c + n);
  }
  return n;
}

static int sphere_box(const GeomView& g1, const GeomView& g2, num margin, Contact* c) {
  return sphere_box_pt(g1.pos, g1.size[0], g2, margin, c);
}

/* box-box: SAT over 15 axes; face contact -> candidate points in fixed order
 * (incident-face corners inside the reference rectangle, reference corners projected onto
 * the incident face, incident-edge x reference-edge crossings), keep depth <= margin, at most
 * MAXPAIRCON; edge-edge -> one contact at the closest points of the two edges. */
static int box_box(const GeomView& A, const GeomView& B, num margin, Contact* c) {
  num a[3][3], b[3][3], t[3];
  for (int k = 0; k < 3; k++) { axis_of(a[k], A.mat, k); axis_of(b[k], B.mat, k); }
  sub3(t, B.pos, A.pos);
  const num* sa = A.size;
  const num* sb = B.size;
  num best = -1e300;
  int bestk = -1;
  num bestn[3] = {0, 0, 0};
  for (int k = 0; k < 15; k++) {
    num L[3];
    if (k < 3) copy3(L, a[k]);
    else if (k < 6) copy3(L, b[k - 3]);
    else {
      cross3(L, a[(k - 6) / 3], b[(k - 6) % 3]);
      num ln = norm3(L);
      if (ln < 1e-6) continue;
      scl3(L, L, 1.0 / ln);
    }
    num ra = sa[0] * std::fabs(dot3(L, a[0])) + sa[1] * std::fabs(dot3(L, a[1])) + sa[2] * std::fabs(dot3(L, a[2]));
    num rb = sb[0] * std::fabs(dot3(L, b[0])) + sb[1] * std::fabs(dot3(L, b[1])) + sb[2] * std::fabs(dot3(L, b[2]));
    num tl = dot3(t, L);
    num sep = std::fabs(tl) - ra - rb;
    if (sep > margin) return 0;
    num bias = k < 6 ? 0 : 1e-6;   /* prefer face axes */
    if (sep > best + bias) {
      best = sep; bestk = k;
      copy3(bestn, L);
      if (tl < 0) scl3(bestn, bestn, -1);
    }
  }
  if (bestk < 0) return 0;
  if (bestk < 6) {
    bool refA = bestk < 3;
    const GeomView& R = refA ? A : B;
    const GeomView& I = refA ? B : A;
    num (*ra)[3] = refA ? a : b;
    num (*ia)[3] = refA ? b : a;
    int fk = refA ? bestk : bestk - 3;
    num nr[3];
    copy3(nr, bestn);
    if (!refA) scl3(nr, nr, -1);        /* reference face normal, toward the incident box */
    num sg = dot3(nr, ra[fk]) > 0 ? 1 : -1;
    int ru = (fk + 1) % 3, rv = (fk + 2) % 3;
    num hu = R.size[ru], hv = R.size[rv];
    num fc[3];
    for (int k = 0; k < 3; k++) fc[k] = R.pos[k] + ra[fk][k] * sg * R.size[fk];
    int ik = 0;
    num imin = 1e300, isg = 1;
    for (int k = 0; k < 3; k++) {
      num dd = dot3(ia[k], nr);
      if (dd < imin) { imin = dd; ik = k; isg = 1; }
      if (-dd < imin) { imin = -dd; ik = k; isg = -1; }
    }
    int iu = (ik + 1) % 3, iv = (ik + 2) % 3;
    num inn[3], ic[3];
    scl3(inn, ia[ik], isg);               /* incident face outward normal */
    for (int k = 0; k < 3; k++) ic[k] = I.pos[k] + inn[k] * I.size[ik];
    num su = I.size[iu], sv = I.size[iv];
    /* incident corners in order around the face */
    num P[4][3], pu[4], pv[4];
    const num cs[4][2] = {{1, 1}, {-1, 1}, {-1, -1}, {1, -1}};
    for (int q = 0; q < 4; q++) {
      for (int k = 0; k < 3; k++) P[q][k] = ic[k] + ia[iu][k] * cs[q][0] * su + ia[iv][k] * cs[q][1] * sv;
      num dv[3];
      sub3(dv, P[q], fc);
      pu[q] = dot3(dv, ra[ru]);
      pv[q] = dot3(dv, ra[rv]);
    }
    int cnt = 0;
    num normal[3];
    copy3(normal, bestn);
    auto emit = [&](const num* p) {
      if (cnt >= MAXPAIRCON) return;
      num dv[3];
      sub3(dv, p, fc);
      num dist = dot3(dv, nr);
      if (dist > margin) return;
      num pos[3];
      for (int k = 0; k < 3; k++) pos[k] = p[k] - nr[k] * dist / 2;
      set_contact(c + cnt++, dist, pos, normal);
    };
    /* (1) incident corners inside the reference rectangle */
    for (int q = 0; q < 4; q++)
      if (std::fabs(pu[q]) <= hu && std::fabs(pv[q]) <= hv) emit(P[q]);
    /* (2) reference corners inside the incident face (projected along nr) */
    num den = dot3(nr, inn);
    if (std::fabs(den) > 1e-12) {
      for (int q = 0; q < 4; q++) {
        num Q[3], dq[3];
        for (int k = 0; k < 3; k++) Q[k] = fc[k] + ra[ru][k] * cs[q][0] * hu + ra[rv][k] * cs[q][1] * hv;
        sub3(dq, ic, Q);
        num tt = dot3(dq, inn) / den;
        num Qp[3];
        for (int k = 0; k < 3; k++) Qp[k] = Q[k] + nr[k] * tt;
        sub3(dq, Qp, ic);
        if (std::fabs(dot3(dq, ia[iu])) <= su && std::fabs(dot3(dq, ia[iv])) <= sv) emit(Qp);
      }
    }
    /* (3) incident edges crossing the reference rectangle's edge lines */
    for (int q = 0; q < 4; q++) {
      int q2 = (q + 1) & 3;
      num du = pu[q2] - pu[q], dv = pv[q2] - pv[q];
      for (int side = 0; side < 4; side++) {
        num tt;
        if (side < 2) {
          num U = side == 0 ? hu : -hu;
          if (std::fabs(du) < 1e-12) continue;
          tt = (U - pu[q]) / du;
          if (!(tt > 0 && tt < 1)) continue;
          num vv = pv[q] + tt * dv;
          if (std::fabs(vv) > hv) continue;
        } else {
          num V = side == 2 ? hv : -hv;
          if (std::fabs(dv) < 1e-12) continue;
          tt = (V - pv[q]) / dv;
          if (!(tt > 0 && tt < 1)) continue;
          num uu = pu[q] + tt * du;
          if (std::fabs(uu) > hu) continue;
        }
        num X[3];
        for (int k = 0; k < 3; k++) X[k] = P[q][k] + (P[q2][k] - P[q][k]) * tt;
        emit(X);
      }
    }
    return cnt;
  }
  /* edge-edge */
  int ea = (bestk - 6) / 3, eb = (bestk - 6) % 3;
  num pa[3], pb[3];
  copy3(pa, A.pos);
  copy3(pb, B.pos);
  for (int k = 0; k < 3; k++) {
    if (k != ea) {
      num s = dot3(a[k], bestn) > 0 ? 1 : -1;
      for (int q = 0; q < 3; q++) pa[q] += a[k][q] * s * sa[k];
    }
    if (k != eb) {
      num s = dot3(b[k], bestn) > 0 ? -1 : 1;
      for (int q = 0; q < 3; q++) pb[q] += b[k][q] * s * sb[k];
    }
  }
  num s1[3], d1[3], s2[3], d2[3], c1[3], c2[3];
  for (int q = 0; q < 3; q++) {
    s1[q] = pa[q] - a[ea][q] * sa[ea]; d1[q] = 2 * a[ea][q] * sa[ea];
    s2[q] = pb[q] - b[eb][q] * sb[eb]; d2[q] = 2 * b[eb][q] * sb[eb];
  }
  segment_segment(s1, d1, s2, d2, c1, c2);
  num pos[3];
  for (int q = 0; q < 3; q++) pos[q] = 0.5 * (c1[q] + c2[q]);
  set_contact(c, best, pos, bestn);
  return 1;
}

/* ------------------------------------------------------------------------------------- */
/* MPR (libccd ccdMPRPenetration restated), supports inflated by margin/2 as mjccd_support */
namespace mpr {
static const num EPS = DBL_EPSILON;
static inline bool is_zero(num x) { return std::fabs(x) < EPS; }
static inline bool eq(num a, num b) {
  num ab = std::fabs(a - b);
  if (ab < EPS) return true;
  num fa = std::fabs(a), fb = std::fabs(b);
  return fb > fa ? ab < EPS * fb : ab < EPS * fa;
}
static inline bool veq(const num* a, const num* b) { return eq(a[0], b[0]) && eq(a[1], b[1]) && eq(a[2], b[2]); }
static inline void vnormalize(num* v) {
  num k = 1.0 / std::sqrt(dot3(v, v));
  scl3(v, v, k);
}
static inline num sign(num x) { return x < 0 ? -1 : (x > 0 ? 1 : 0); }

struct Sup { num v[3], v1[3], v2[3]; };

static void geom_support(num* res, const GeomView& g, const num* dir, num margin) {
  num ld[3], r[3];
  mul_matT_vec3(ld, g.mat, dir);
  const num* s = g.size;
  switch (g.type) {
    case GEOM_SPHERE: scl3(r, ld, s[0]); break;
    case GEOM_CAPSULE: scl3(r, ld, s[0]); r[2] += sign(ld[2]) * s[1]; break;
    case GEOM_CYLINDER: {
      num tmp = std::sqrt(ld[0] * ld[0] + ld[1] * ld[1]);
      if (tmp > MINVAL) { r[0] = ld[0] / tmp * s[0]; r[1] = ld[1] / tmp * s[0]; }
      else { r[0] = r[1] = 0; }
      r[2] = sign(ld[2]) * s[1];
      break;
    }
    case GEOM_BOX: for (int k = 0; k < 3; k++) r[k] = sign(ld[k]) * s[k]; break;
    default: r[0] = r[1] = r[2] = 0;
  }
  for (int k = 0; k < 3; k++) r[k] += ld[k] * margin / 2;
  mul_mat_vec3(res, g.mat, r);
  add3(res, res, g.pos);
}

struct Ctx { const GeomView* g1; const GeomView* g2; num margin, tol; int maxit; };

static void support(const Ctx& c, const num* dir, Sup* s) {
  num nd[3];
  scl3(nd, dir, -1);
  geom_support(s->v1, *c.g1, dir, c.margin);
  geom_support(s->v2, *c.g2, nd, c.margin);
  sub3(s->v, s->v1, s->v2);
}

static void portal_dir(const Sup* p, num* dir) {
  num a[3], b[3];
  sub3(a, p[2].v, p[1].v);
  sub3(b, p[3].v, p[1].v);
  cross3(dir, a, b);
  vnormalize(dir);
}
static bool encapsules_origin(const Sup* p, const num* dir) {
  num d = dot3(dir, p[1].v);
  return is_zero(d) || d > 0;
}
static bool reach_tolerance(const Sup* p, const Sup* v4, const num* dir, num tol) {
  num dv1 = dot3(p[1].v, dir), dv2 = dot3(p[2].v, dir), dv3 = dot3(p[3].v, dir), dv4 = dot3(v4->v, dir);
  num d1 = dv4 - dv1, d2 = dv4 - dv2, d3 = dv4 - dv3;
  d1 = d1 < d2 ? d1 : d2;
  d1 = d1 < d3 ? d1 : d3;
  return eq(d1, tol) || d1 < tol;
}
static bool can_encapsule(const Sup* v4, const num* dir) {
  num d = dot3(v4->v, dir);
  return is_zero(d) || d > 0;
}
static void expand(Sup* p, const Sup* v4) {
  num v4v0[3];
  cross3(v4v0, v4->v, p[0].v);
  num d = dot3(p[1].v, v4v0);
  if (d > 0) {
    d = dot3(p[2].v, v4v0);
    if (d > 0) p[1] = *v4; else p[3] = *v4;
  } else {
    d = dot3(p[3].v, v4v0);
    if (d > 0) p[2] = *v4; else p[1] = *v4;
  }
}

static int discover(const Ctx& c, Sup* p) {
  num dir[3], va[3], vb[3];
  copy3(p[0].v1, c.g1->pos);
  copy3(p[0].v2, c.g2->pos);
  sub3(p[0].v, p[0].v1, p[0].v2);
  num zero[3] = {0, 0, 0};
  if (veq(p[0].v, zero)) p[0].v[0] += EPS * 10;
  scl3(dir, p[0].v, -1);
  vnormalize(dir);
  support(c, dir, &p[1]);
  num d = dot3(p[1].v, dir);
  if (is_zero(d) || d < 0) return -1;
  cross3(dir, p[0].v, p[1].v);
  if (is_zero(dot3(dir, dir))) return veq(p[1].v, zero) ? 1 : 2;
  vnormalize(dir);
  support(c, dir, &p[2]);
  d = dot3(p[2].v, dir);
  if (is_zero(d) || d < 0) return -1;
  sub3(va, p[1].v, p[0].v);
  sub3(vb, p[2].v, p[0].v);
  cross3(dir, va, vb);
  vnormalize(dir);
  if (dot3(dir, p[0].v) > 0) {
    Sup t = p[1]; p[1] = p[2]; p[2] = t;
    scl3(dir, dir, -1);
  }
  for (int it = 0; it < 1000; it++) {
    support(c, dir, &p[3]);
    d = dot3(p[3].v, dir);
    if (is_zero(d) || d < 0) return -1;
    bool cont = false;
    cross3(va, p[1].v, p[3].v);
    d = dot3(va, p[0].v);
    if (d < 0 && !is_zero(d)) { p[2] = p[3]; cont = true; }
    if (!cont) {
      cross3(va, p[3].v, p[2].v);
      d = dot3(va, p[0].v);
      if (d < 0 && !is_zero(d)) { p[1] = p[3]; cont = true; }
    }
    if (cont) {
      sub3(va, p[1].v, p[0].v);
      sub3(vb, p[2].v, p[0].v);
      cross3(dir, va, vb);
      vnormalize(dir);
    } else {
      return 0;
    }
  }
  return -1;
}

static int refine(const Ctx& c, Sup* p) {
  num dir[3];
  Sup v4;
  /* libccd loops without a cap; we cap at mpr_iterations (both oracle and kernel) */
  for (int it = 0; it <= c.maxit; it++) {
    portal_dir(p, dir);
    if (encapsules_origin(p, dir)) return 0;
    support(c, dir, &v4);
    if (!can_encapsule(&v4, dir) || reach_tolerance(p, &v4, dir, c.tol)) return -1;
    expand(p, &v4);
  }
  return -1;
}

static num point_segment_dist2(const num* P, const num* x0, const num* b, num* w) {
  num dd[3], a[3];
  sub3(dd, b, x0);
  sub3(a, x0, P);
  num t = -dot3(a, dd) / dot3(dd, dd);
  if (t < 0 || is_zero(t)) { copy3(w, x0); }
  else if (t > 1 || eq(t, 1)) { copy3(w, b); }
  else { for (int k = 0; k < 3; k++) w[k] = x0[k] + dd[k] * t; }
  num df[3];
  sub3(df, w, P);
  return dot3(df, df);
}

static num point_tri_dist2(const num* P, const num* x0, const num* B, const num* C, num* w) {
  num d1[3], d2[3], a[3];
  sub3(d1, B, x0);
  sub3(d2, C, x0);
  sub3(a, x0, P);
  num u = dot3(a, a), v = dot3(d1, d1), ww = dot3(d2, d2), p = dot3(a, d1), q = dot3(a, d2), r = dot3(d1, d2);
  (void)u;
  num dd = ww * v - r * r, s, t;
  if (is_zero(dd)) { s = t = -1; }
  else { s = (q * r - ww * p) / dd; t = (-s * r - q) / ww; }
  if ((is_zero(s) || s > 0) && (eq(s, 1) || s < 1) && (is_zero(t) || t > 0) && (eq(t, 1) || t < 1) &&
      (eq(t + s, 1) || t + s < 1)) {
    for (int k = 0; k < 3; k++) w[k] = x0[k] + d1[k] * s + d2[k] * t;
    num df[3];
    sub3(df, w, P);
    return dot3(df, df);
  }
  num w2[3];
  num dist = point_segment_dist2(P, x0, B, w);
  num d2s = point_segment_dist2(P, x0, C, w2);
  if (d2s < dist) { dist = d2s; copy3(w, w2); }
  d2s = point_segment_dist2(P, B, C, w2);
  if (d2s < dist) { dist = d2s; copy3(w, w2); }
  return dist;
}

static void find_pos(const Sup* p, num* pos) {
  num dir[3], vec[3], b[4];
  portal_dir(p, dir);
  cross3(vec, p[1].v, p[2].v); b[0] = dot3(vec, p[3].v);
  cross3(vec, p[3].v, p[2].v); b[1] = dot3(vec, p[0].v);
  cross3(vec, p[0].v, p[1].v); b[2] = dot3(vec, p[3].v);
  cross3(vec, p[2].v, p[1].v); b[3] = dot3(vec, p[0].v);
  num sum = b[0] + b[1] + b[2] + b[3];
  if (is_zero(sum) || sum < 0) {
    b[0] = 0;
    cross3(vec, p[2].v, p[3].v); b[1] = dot3(vec, dir);
    cross3(vec, p[3].v, p[1].v); b[2] = dot3(vec, dir);
    cross3(vec, p[1].v, p[2].v); b[3] = dot3(vec, dir);
    sum = b[1] + b[2] + b[3];
  }
  num inv = 1.0 / sum, p1[3] = {0, 0, 0}, p2[3] = {0, 0, 0};
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 3; k++) { p1[k] += p[i].v1[k] * b[i]; p2[k] += p[i].v2[k] * b[i]; }
  for (int k = 0; k < 3; k++) pos[k] = 0.5 * (p1[k] + p2[k]) * inv;
}

/* returns 0 on contact with depth/dir/pos, -1 otherwise */
static int penetration(const Ctx& c, num* depth, num* dir, num* pos) {
  Sup p[4];
  int res = discover(c, p);
  if (res < 0) return -1;
  if (res == 1) {
    *depth = 0;
    dir[0] = dir[1] = dir[2] = 0;
    for (int k = 0; k < 3; k++) pos[k] = 0.5 * (p[1].v1[k] + p[1].v2[k]);
    return 0;
  }
  if (res == 2) {
    for (int k = 0; k < 3; k++) pos[k] = 0.5 * (p[1].v1[k] + p[1].v2[k]);
    copy3(dir, p[1].v);
    *depth = std::sqrt(dot3(dir, dir));
    vnormalize(dir);
    return 0;
  }
  if (refine(c, p) < 0) return -1;
  Sup v4;
  num pd[3];
  for (int it = 0;; it++) {
    portal_dir(p, pd);
    support(c, pd, &v4);
    if (reach_tolerance(p, &v4, pd, c.tol) || it > c.maxit) {
      num zero[3] = {0, 0, 0};
      *depth = std::sqrt(point_tri_dist2(zero, p[1].v, p[2].v, p[3].v, dir));
      if (is_zero(*depth)) dir[0] = dir[1] = dir[2] = 0;
      else vnormalize(dir);
      find_pos(p, pos);
      return 0;
    }
    expand(p, &v4);
  }
}
}  // namespace mpr

static int convex(const Model* m, const GeomView& g1, const GeomView& g2, num margin, Contact* c) {
  mpr::Ctx ctx{&g1, &g2, margin, m->mpr_tolerance, m->mpr_iterations};
  num depth, dir[3], pos[3];
  if (mpr::penetration(ctx, &depth, dir, pos) != 0) return 0;
  if (dir[0] == 0 && dir[1] == 0 && dir[2] == 0) return 0;
  num dist = margin - depth;
  if (dist > margin) return 0;
  set_contact(c, dist, pos, dir);
  return 1;
}

/* ------------------------------------------------------------------------------------- */
static int collide_views(const Model* m, GeomView a, GeomView b, num margin, Contact* out);

int collide_geoms(const Model* m, const Data* d, int g1, int g2, num margin, Contact* out, int maxout) {
  (void)maxout;
  GeomView a{&d->geom_xpos[3 * g1], &d->geom_xmat[9 * g1], &d->geom_size[3 * g1], m->geom_type[g1]};
  GeomView b{&d->geom_xpos[3 * g2], &d->geom_xmat[9 * g2], &d->geom_size[3 * g2], m->geom_type[g2]};
  if (a.type > b.type) { GeomView t = a; a = b; b = t; }
  if (a.type != GEOM_PLANE && b.type != GEOM_PLANE) {
    num dif[3];
    sub3(dif, a.pos, b.pos);
    int ga = m->geom_type[g1] <= m->geom_type[g2] ? g1 : g2;
    int gb = ga == g1 ? g2 : g1;
    if (norm3(dif) > m->geom_rbound[ga] + m->geom_rbound[gb] + margin) return 0;
  }
  return collide_views(m, a, b, margin, out);
}

/* narrowphase of two primitives given by pose / size (test hook: exact-geometry collider tests) */
int collide_raw(const Model* m, int t1, const num* p1, const num* m1, const num* s1, int t2, const num* p2,
                const num* m2, const num* s2, num margin, Contact* out) {
  GeomView a{p1, m1, s1, t1}, b{p2, m2, s2, t2};
  if (a.type > b.type) { GeomView t = a; a = b; b = t; }
  return collide_views(m, a, b, margin, out);
}

static int collide_views(const Model* m, GeomView a, GeomView b, num margin, Contact* out) {
  switch (a.type) {
    case GEOM_PLANE:
      switch (b.type) {
        case GEOM_SPHERE: return plane_sphere(a.pos, a.mat, b.pos, b.size[0], margin, out);
        case GEOM_CAPSULE: return plane_capsule(a, b, margin, out);
        case GEOM_CYLINDER: return plane_cylinder(a, b, margin, out);
        case GEOM_BOX: return plane_box(a, b, margin, out);
      }
      return 0;
    case GEOM_SPHERE:
      switch (b.type) {
        case GEOM_SPHERE: return sphere_sphere(a.pos, a.size[0], b.pos, b.size[0], margin, out);
        case GEOM_CAPSULE: return sphere_capsule(a, b, margin, out);
        case GEOM_CYLINDER: return convex(m, a, b, margin, out);
        case GEOM_BOX: return sphere_box(a, b, margin, out);
      }
      return 0;
    case GEOM_CAPSULE:
      switch (b.type) {
        case GEOM_CAPSULE: return capsule_capsule(a, b, margin, out);
        case GEOM_CYLINDER: return convex(m, a, b, margin, out);
        case GEOM_BOX: return capsule_box(a, b, margin, out);
      }
      return 0;
    case GEOM_CYLINDER:
      return convex(m, a, b, margin, out);
    case GEOM_BOX:
      if (b.type == GEOM_BOX) return box_box(a, b, margin, out);
      return 0;
  }
  return 0;
}

static void finish_contacts(Data* d, int start, int g1, int g2, int condim, const num* fr5,
                            const num* solref, const num* solimp, num margin, num gap) {
  for (int i = start; i < d->ncon; i++) {
    Contact* c = &d->contact[i];
    c->geom1 = g1; c->geom2 = g2;
    c->dim = condim;
    for (int k = 0; k < 5; k++) c->friction[k] = fr5[k];
    c->solref[0] = solref[0]; c->solref[1] = solref[1];
    for (int k = 0; k < 5; k++) c->solimp[k] = solimp[k];
    c->includemargin = margin - gap;
    c->efc_address = -1;
    make_frame(c->frame);
  }
}

static num nudge(const Model* m, int g1, int g2) {
  return (g1 == m->nudge_g1 && g2 == m->nudge_g2) || (g1 == m->nudge_g2 && g2 == m->nudge_g1) ? m->nudge_delta : 0;
}

void collision(const Model* m, Data* d) {
  d->ncon = 0;
  if (m->disableflags & (DSBL_CONSTRAINT | DSBL_CONTACT)) return;
  Contact buf[16];
  /* explicit pairs */
  for (int p = 0; p < m->npair; p++) {
    int g1 = m->pair_geom1[p], g2 = m->pair_geom2[p];
    num margin = m->pair_margin[p] + nudge(m, g1, g2);
    int n = collide_geoms(m, d, g1, g2, margin, buf, 16);
    int start = d->ncon;
    for (int k = 0; k < n; k++) {
      if (d->ncon >= m->max_con) { d->status |= ST_CON_OVERFLOW; break; }
      d->contact[d->ncon++] = buf[k];
    }
    finish_contacts(d, start, g1, g2, m->pair_condim[p], &m->pair_friction[5 * p],
                    &m->pair_solref[2 * p], &m->pair_solimp[5 * p], margin, m->pair_gap[p]);
  }
  /* dynamic candidates */
  for (int c = 0; c < m->ncand; c++) {
    int g1 = m->cand_geom1[c], g2 = m->cand_geom2[c];
    num margin = std::fmax(m->geom_margin[g1], m->geom_margin[g2]) + nudge(m, g1, g2);
    num gap = std::fmax(m->geom_gap[g1], m->geom_gap[g2]);
    int n = collide_geoms(m, d, g1, g2, margin, buf, 16);
    if (!n) continue;
    int start = d->ncon;
    for (int k = 0; k < n; k++) {
      if (d->ncon >= m->max_con) { d->status |= ST_CON_OVERFLOW; break; }
      d->contact[d->ncon++] = buf[k];
    }
    /* mj_contactParam: equal priority -> max condim/friction, solmix-weighted ref/imp */
    int condim = m->geom_condim[g1] > m->geom_condim[g2] ? m->geom_condim[g1] : m->geom_condim[g2];
    num s1 = m->geom_solmix[g1], s2 = m->geom_solmix[g2], mix;
    if (s1 >= MINVAL && s2 >= MINVAL) mix = s1 / (s1 + s2);
    else if (s1 < MINVAL && s2 < MINVAL) mix = 0.5;
    else mix = s1 < MINVAL ? 0.0 : 1.0;
    num solref[2], solimp[5], fr[5];
    for (int k = 0; k < 2; k++) solref[k] = mix * m->geom_solref[2 * g1 + k] + (1 - mix) * m->geom_solref[2 * g2 + k];
    for (int k = 0; k < 5; k++) solimp[k] = mix * m->geom_solimp[5 * g1 + k] + (1 - mix) * m->geom_solimp[5 * g2 + k];
    num f0 = std::fmax(m->geom_friction[3 * g1], m->geom_friction[3 * g2]);
    num f1 = std::fmax(m->geom_friction[3 * g1 + 1], m->geom_friction[3 * g2 + 1]);
    num f2 = std::fmax(m->geom_friction[3 * g1 + 2], m->geom_friction[3 * g2 + 2]);
    fr[0] = fr[1] = f0; fr[2] = f1; fr[3] = fr[4] = f2;
    finish_contacts(d, start, g1, g2, condim, fr, solref, solimp, margin, gap);
  }
}

/* ------------------------------------------------------------------------------------- */
/* mju_rayGeom for the site shapes (sphere, capsule, cylinder, box): distance along the
 * (unit) ray to the first surface crossing at t >= 0, or -1. */
num ray_geom(const num* pos, const num* mat, const num* size, const num* pnt, const num* vec, int type) {
  num dif[3], lp[3], lv[3];
  sub3(dif, pnt, pos);
  mul_matT_vec3(lp, mat, dif);
  mul_matT_vec3(lv, mat, vec);
  num best = -1;
  auto consider = [&](num t) { if (t >= 0 && (best < 0 || t < best)) best = t; };
  auto sphere = [&](const num* c, num r) {
    num o[3] = {lp[0] - c[0], lp[1] - c[1], lp[2] - c[2]};
    num a = dot3(lv, lv), b = dot3(o, lv), cc = dot3(o, o) - r * r;
    num disc = b * b - a * cc;
    if (disc < 0 || a < MINVAL) return;
    num sq = std::sqrt(disc);
    consider((-b - sq) / a);
    consider((-b + sq) / a);
  };
  switch (type) {
    case GEOM_SPHERE: { num c[3] = {0, 0, 0}; sphere(c, size[0]); break; }
    case GEOM_BOX:
      for (int k = 0; k < 3; k++) {
        if (std::fabs(lv[k]) < MINVAL) continue;
        for (int s = -1; s <= 1; s += 2) {
          num t = (s * size[k] - lp[k]) / lv[k];
          int u = (k + 1) % 3, v = (k + 2) % 3;
          num pu = lp[u] + t * lv[u], pv = lp[v] + t * lv[v];
          if (std::fabs(pu) <= size[u] && std::fabs(pv) <= size[v]) consider(t);
        }
      }
      break;
    case GEOM_CYLINDER:
    case GEOM_CAPSULE: {
      num r = size[0], h = size[1];
      num a = lv[0] * lv[0] + lv[1] * lv[1];
      num b = lp[0] * lv[0] + lp[1] * lv[1];
      num cc = lp[0] * lp[0] + lp[1] * lp[1] - r * r;
      num disc = b * b - a * cc;
      if (a > MINVAL && disc >= 0) {
        num sq = std::sqrt(disc);
        for (int s = -1; s <= 1; s += 2) {
          num t = (-b + s * sq) / a;
          if (std::fabs(lp[2] + t * lv[2]) <= h) consider(t);
        }
      }
      if (type == GEOM_CYLINDER) {
        if (std::fabs(lv[2]) > MINVAL)
          for (int s = -1; s <= 1; s += 2) {
            num t = (s * h - lp[2]) / lv[2];
            num px = lp[0] + t * lv[0], py = lp[1] + t * lv[1];
            if (px * px + py * py <= r * r) consider(t);
          }
      } else {
        num c1[3] = {0, 0, h}, c2[3] = {0, 0, -h};
        sphere(c1, r);
        sphere(c2, r);
      }
      break;
    }
  }
  return best;
}

}  // namespace orc
