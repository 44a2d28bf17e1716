// aw_solver.h -- constraint assembly, Newton solver, noslip, touch sensor, Euler (fp32).
//
// Restates MuJoCo 2.1 mj_makeConstraint / mj_makeImpedance / mj_solNewton / mj_solNoSlip /
// mj_Euler (fp64 statement: oracle/solver.cc, oracle/mjstep.cc).  Layout on the wave:
//   * rows [0, nsparse): frictionloss / joint-limit / tendon-limit rows with <= 2 nonzeros,
//     kept as (index, value) pairs; rows [nsparse, nefc): contact rows, dense J in LDS.
//   * Newton: lane i holds row i of H = M + J'DJ in VGPRs; the dense part J_d'DJ_d is formed on
//     the matrix cores (v_mfma_f32_16x16x4_f32), H is factored as U D U' in registers (column
//     broadcast through LDS), the factor is written once to LDS for the backward substitution.
//   * rows are evaluated lane-per-row (three rows per lane, nefc <= 192); the exact line search
//     and the cost are wave reductions.
//   * noslip: projected Gauss-Seidel in row space -- lane k owns noslip row k (dof frictionloss
//     rows, then pyramid-edge pairs) and holds its row of A = B inv(M) B' in VGPRs, so a row's
//     update is fma -> med3 -> readlane -> fma on the serial chain.
#pragma once
#include "aw_common.h"
#include "aw_tree.h"

namespace aw {

// ---------------------------------------------------------------------------------------
// dense factorisation of a lane-distributed SPD matrix (lane i holds row i; lower part used).
// LDL': H = U D U' with U unit lower triangular, right-looking in panels of P = 4 columns.  Column
// j: pivot D_j = H'_jj (clamped at MINVAL like mju_cholFactor's diagonal), U_ij = H'_ij / D_j; the
// update H'_ik -= H'_ij U_kj takes the lane's own unscaled entry and the scaled column.  Inside a
// panel the columns reach the panel's later rows by readlane; the panel's four columns are then
// published through LDS ONCE (lane k writes U_k,j0..j0+3 as one 16-byte row) and every lane applies
// them to its trailing entries with one 16-byte broadcast read per k.  Each entry still receives its
// updates one column at a time in column order, so the factor is bitwise the column-at-a-time one
// (r04n A/B against column-at-a-time with 2-column look-ahead: -0.2 % random, -0.3 % DAPG; 8-wide
// panels +0.1 % / +0.5 %).  Every entry on or above a lane's diagonal ends as exactly 0 (U's unit
// diagonal is implicit, 1 / D_j is kept in lane j's invd), so the substitutions below run unmasked;
// entries above the diagonal (and rows of lanes >= NV) take garbage updates that are never read.
template <int NV>
AW_DEV void chol_factor(float (&row)[NV], int lane_in, float& invd, Env& s) {
  const int lane = opaque(lane_in);   // lane compares are made here, not hoisted out of the caller's loop
  constexpr int P = CHOL_P;
  static_assert(sizeof(s.colbuf) >= (size_t)MAXV * P * 4, "panel buffer");
  float4* pan = s.colbuf;
#pragma unroll
  for (int j0 = 0; j0 < NV; j0 += P) {
    float a[P], u[P];
#pragma unroll
    for (int t = 0; t < P; t++) {
      const int j = j0 + t;
      a[t] = u[t] = 0.f;
      if (j < NV) {
        const float dj = __builtin_amdgcn_fmed3f(rlane(row[j], j), MINVAL, 3.402823466e38f);
        const float inv = __builtin_amdgcn_rcpf(dj);
        a[t] = row[j];
        if (lane == j) invd = inv;
        u[t] = lane > j ? a[t] * inv : 0.f;
        row[j] = u[t];
#pragma unroll
        for (int t2 = t + 1; t2 < P; t2++)
          if (j0 + t2 < NV) row[j0 + t2] = fmaf(-a[t], rlane(u[t], j0 + t2), row[j0 + t2]);
      }
    }
    if (j0 + P < NV) {
      if (lane < NV) pan[lane] = make_float4(u[0], u[1], u[2], u[3]);
      wsync();
#pragma unroll
      for (int k = j0 + P; k < NV; k++) {
        const float4 c = pan[k];
        row[k] = fmaf(-a[0], c.x, row[k]);
        row[k] = fmaf(-a[1], c.y, row[k]);
        row[k] = fmaf(-a[2], c.z, row[k]);
        row[k] = fmaf(-a[3], c.w, row[k]);
      }
      wsync();
    }
  }
}
// packed rows of U into s.L (row padding included: the factor-reuse path reloads whole 4-blocks)
template <int NV>
AW_DEV void chol_store(const float (&row)[NV], int lane_in, Env& s) {
  const int lane = opaque(lane_in);
  if (lane < NV) {
    // whole 4-blocks up to the lane's own: 16-byte stores (the padding past NV in the last block is
    // written as 0 -- inside the row's padded length, never read as a factor entry); against one
    // 4-byte store per entry: -1.2 % random, -0.9 % DAPG (r04q)
#pragma unroll
    for (int q = 0; q < (NV + 3) / 4; q++)
      if (4 * q <= lane)
        *reinterpret_cast<float4*>(&s.L[tri(lane) + 4 * q]) =
            make_float4(row[4 * q], 4 * q + 1 < NV ? row[4 * q + 1 < NV ? 4 * q + 1 : 0] : 0.f,
                        4 * q + 2 < NV ? row[4 * q + 2 < NV ? 4 * q + 2 : 0] : 0.f,
                        4 * q + 3 < NV ? row[4 * q + 3 < NV ? 4 * q + 3 : 0] : 0.f);
  }
}
// x = inv(U D U') b, b lane-distributed; U rows in registers (forward) and packed in LDS (backward)
template <int NV>
AW_DEV float chol_solve(const float (&row)[NV], float invd, float b, int lane_in, const Env& s) {
  const int lane = opaque(lane_in);
#pragma unroll
  for (int j = 0; j < NV; j++) b = fmaf(-row[j], rlane(b, j), b);
  b *= invd;
  const int lc = lane < NV ? lane : 0;
#pragma unroll
  for (int j = NV - 1; j > 0; j--) {
    const float c = s.L[tri(j) + lc];
    b = fmaf(lane < j ? -c : 0.f, rlane(b, j), b);
  }
  return lane < NV ? b : 0.f;
}
// y = M x with M lane-distributed rows and x in LDS (broadcast reads)
template <int NV>
AW_DEV float matvec_lds(const float (&row)[NV], const float* x) {
  float acc = 0.f;
#pragma unroll
  for (int q = 0; q < (NV + 3) / 4; q++) {
    const float4 v = *reinterpret_cast<const float4*>(x + 4 * q);
    const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int t = 0; t < 4; t++)
      if (4 * q + t < NV) acc = fmaf(row[4 * q + t], vv[t], acc);
  }
  return acc;
}
// y = M x with M lane-distributed rows and x lane-distributed
template <int NV>
AW_DEV float matvec(const float (&row)[NV], float x) {
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < NV; k++) acc = fmaf(row[k], rlane(x, k), acc);
  return acc;
}

// ---------------------------------------------------------------------------------------
AW_DEV float getimpedance(gp_t<const float> solimp, float pm) {
  float d0 = clampf(solimp[0], 0.0001f, 0.9999f), dmax = clampf(solimp[1], 0.0001f, 0.9999f);
  if (d0 == dmax || solimp[2] <= MINVAL) return 0.5f * (d0 + dmax);
  float x = fabsf(pm / solimp[2]);
  if (x >= 1 || x <= 0) return x >= 1 ? dmax : d0;
  float y, mid = solimp[3], p = solimp[4];
  if (p == 1) y = x;
  else if (p == 2) y = x <= mid ? x * x / mid : 1 - (1 - x) * (1 - x) / (1 - mid);   // default solimp power
  else if (x <= mid) y = powf(x, p) / powf(mid, p - 1);
  else y = 1 - powf(1 - x, p) / powf(1 - mid, p - 1);
  return d0 + y * (dmax - d0);
}

// ---------------------------------------------------------------------------------------
// Dense J storage: rows [0, JL) in LDS (s.J), rows [JL, ndense) in this env's global spill
// block.  Spill rows are written and read with VECTOR memory instructions only: every read
// below uses a lane-dependent address (a row per lane, or the row's entry per lane followed by
// a readlane broadcast), so no uniform (scalar-cache) load can see a previous substep's row.
AW_DEV gp_t<float> jspill_row(const DModel& m, const Env& s, int d) {
  return gmp(m.jspill) + (size_t)s.slot * JSPILL + (size_t)(d - JL) * VS;
}
AW_DEV void jput(const DModel& m, Env& s, int d, int k, float v) {
  if (d < JL) s.J[d][k] = v;
  else jspill_row(m, s, d)[k] = v;
}
// the wave's spill-row stores complete before any lane reads them back
AW_DEV void jspill_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// J_r . x  (x in LDS); r is per lane
template <int NV>
AW_DEV float row_dot(const DModel& m, const Env& s, int r, const float* x) {
  if (r < s.nsparse) {
    const int i1 = s.efc_i1[r];
    const float x1 = x[i1 >= 0 ? i1 : 0], v1 = s.efc_v1[r];   // loaded unconditionally, then selected
    return s.efc_v0[r] * x[s.efc_i0[r]] + (i1 >= 0 ? v1 * x1 : 0.f);
  }
  const int d = r - s.nsparse;
  float acc = 0.f;
  if (d < JL) {
    const float* J = s.J[d];
#pragma unroll
    for (int k = 0; k < NV; k++) acc = fmaf(J[k], x[k], acc);
  } else {
    gp_t<const float> J = jspill_row(m, s, d);
#pragma unroll
    for (int k = 0; k < NV; k++) acc = fmaf(J[k], x[k], acc);
  }
  return acc;
}

// (J_r . x, J_r . y) for two vectors in LDS: one pass over the row's entries
template <int NV>
AW_DEV void row_dot2(const DModel& m, const Env& s, int r, const float* x, const float* y, float& dx, float& dy) {
  if (r < s.nsparse) {
    const int i0 = s.efc_i0[r], i1 = s.efc_i1[r];
    const float v0 = s.efc_v0[r], v1 = s.efc_v1[r];
    const int j1 = i1 >= 0 ? i1 : 0;   // loaded unconditionally, then selected
    const float x1 = x[j1], y1 = y[j1];
    dx = v0 * x[i0] + (i1 >= 0 ? v1 * x1 : 0.f);
    dy = v0 * y[i0] + (i1 >= 0 ? v1 * y1 : 0.f);
    return;
  }
  const int d = r - s.nsparse;
  float ax = 0.f, ay = 0.f;
  if (d < JL) {
    const float* J = s.J[d];
#pragma unroll
    for (int k = 0; k < NV; k++) { ax = fmaf(J[k], x[k], ax); ay = fmaf(J[k], y[k], ay); }
  } else {
    gp_t<const float> J = jspill_row(m, s, d);
#pragma unroll
    for (int k = 0; k < NV; k++) { const float j = J[k]; ax = fmaf(j, x[k], ax); ay = fmaf(j, y[k], ay); }
  }
  dx = ax;
  dy = ay;
}

// out_k = (J' f)_k for k = lane; f given per row in s.rowbuf (must be written + synced)
// ABS: *absum = the lane's sum of the magnitudes of its terms (|sparse part| + sum_d |J_dk f_d|),
// the scale of the result's fp32 rounding noise
template <int NV, bool ABS = false>
AW_DEV float jt_mul(const DModel& m, Env& s, int lane, float* absum = nullptr) {
  if (lane < NV) s.vec2[lane] = 0.f;
  wsync();
  for (int r = lane; r < s.nsparse; r += 64) {
    float f = s.rowbuf[r];
    if (f != 0.f) {
      atomicAdd(&s.vec2[s.efc_i0[r]], s.efc_v0[r] * f);
      int i1 = s.efc_i1[r];
      if (i1 >= 0) atomicAdd(&s.vec2[i1], s.efc_v1[r] * f);
    }
  }
  wsync();
  const int li = lane < NV ? lane : NV - 1;
  float out = s.vec2[li];
  float oa = fabsf(out);
  const int nd = s.ndense, ndl = nd < JL ? nd : JL;
  // unrolled by 4: the loads of four rows are issued before their fmas (one load latency per
  // four rows, not per row; the spill rows are global loads)
#ifndef AW_JT_UNROLL
#define AW_JT_UNROLL 4
#endif
#pragma unroll AW_JT_UNROLL
  for (int d = 0; d < ndl; d++) {
    const float j = s.J[d][li], f = s.rowbuf[s.nsparse + d];
    out = fmaf(j, f, out);
    if (ABS) oa = fmaf(fabsf(j), fabsf(f), oa);
  }
  if (nd > JL) {
    gp_t<const float> Jg = jspill_row(m, s, JL);
#pragma unroll AW_JT_UNROLL
    for (int d = JL; d < nd; d++) {
      const float j = Jg[(d - JL) * VS + li], f = s.rowbuf[s.nsparse + d];
      out = fmaf(j, f, out);
      if (ABS) oa = fmaf(fabsf(j), fabsf(f), oa);
    }
  }
  if (ABS) *absum = lane < NV ? oa : 0.f;
  return lane < NV ? out : 0.f;
}

// ---------------------------------------------------------------------------------------
// mj_makeConstraint + mj_makeImpedance + reference acceleration
template <int NV>
AW_DEV void stage_constraints(const DModel& m, Env& s, int lane) {
  if (m.disableflags & DSBL_CONSTRAINT) {
    if (lane == 0) { s.nefc = s.nsparse = s.ndense = 0; }
    wsync();
    return;
  }
  const int nfl = (m.disableflags & DSBL_FRICTIONLOSS) ? 0 : m.nfl;
  // frictionloss rows (dof order)
  if (lane < nfl) {
    int d = MD(fl_dof, lane);
    s.efc_type[lane] = C_FRIC_DOF; s.efc_id[lane] = d;
    s.efc_i0[lane] = d; s.efc_i1[lane] = -1; s.efc_v0[lane] = 1.f; s.efc_v1[lane] = 0.f;
    // (aw_set_fault kind 2, the parity classifier's negative test: one row held in the stick state)
    s.rowbuf[lane] = 0.f; s.efc_floss[lane] = lane == m.fault_flrow ? 1e6f : MD(dof_frictionloss, d);
    s.efc_force[lane] = MD(dof_invweight0, d);
  }
  // joint limits: lower then upper per joint, joints in order.  MuJoCo activates a side when
  // dist = side * (range - q) < margin, in fp64.  That test is evaluated here in fp64 too, on the
  // fp32 state with the model's fp64 range / margin (jnt_range64): a joint resting on a range
  // edge equal to its margin (hammer's nail: range edge 0.01 = margin, q ~ 1e-22) is then decided
  // exactly as the reference decides it -- in fp32, range - q rounds the other way.  dlo / dhi
  // are dist - margin.
  const bool lim = !(m.disableflags & DSBL_LIMIT);
  int lo = 0, hi = 0;
  float dlo = 0, dhi = 0;
  if (lim && lane < m.njnt && MD(jnt_limited, lane)) {
    const double q = qpos64(s, lane), mgd = MD(jnt_margin64, lane);
    const double d0 = __dsub_rn(q, MD(jnt_range64, 2 * lane));
    const double d1 = __dsub_rn(MD(jnt_range64, 2 * lane + 1), q);
    lo = d0 < mgd; hi = d1 < mgd;
    dlo = (float)(d0 - mgd); dhi = (float)(d1 - mgd);
  }
  int njl;
  int off = nfl + wave_excl_scan<2>(lo + hi, lane, &njl);
  if (lo || hi) {
    for (int side = 0; side < 2; side++) {
      if (!(side ? hi : lo)) continue;
      int r = off++;
      if (r >= EFC_CAP) { atomicOr(&s.status, (unsigned)ST_EFC_OVERFLOW); continue; }
      s.efc_type[r] = C_LIM_JNT; s.efc_id[r] = lane;
      s.efc_i0[r] = lane; s.efc_i1[r] = -1; s.efc_v0[r] = side ? -1.f : 1.f; s.efc_v1[r] = 0.f;
      s.rowbuf[r] = side ? dhi : dlo; s.efc_floss[r] = 0.f; s.efc_force[r] = MD(dof_invweight0, lane);
    }
  }
  // tendon limits
  lo = hi = 0;
  if (lim && lane < m.ntendon && MD(ten_limited, lane)) {
    const int d1 = MD(ten_d1, lane);
    // fixed tendon length in fp64 with the reference's operation order (no contraction)
    const double len = __dadd_rn(__dmul_rn(MD(ten_c0_64, lane), qpos64(s, MD(ten_d0, lane))),
                                 d1 >= 0 ? __dmul_rn(MD(ten_c1_64, lane), qpos64(s, d1)) : 0.0);
    const double mgd = MD(ten_margin64, lane);
    const double e0 = __dsub_rn(len, MD(ten_range64, 2 * lane));
    const double e1 = __dsub_rn(MD(ten_range64, 2 * lane + 1), len);
    lo = e0 < mgd; hi = e1 < mgd;
    dlo = (float)(e0 - mgd); dhi = (float)(e1 - mgd);
  }
  int ntl;
  off = nfl + njl + wave_excl_scan<2>(lo + hi, lane, &ntl);
  if (lo || hi) {
    for (int side = 0; side < 2; side++) {
      if (!(side ? hi : lo)) continue;
      int r = off++;
      if (r >= EFC_CAP) { atomicOr(&s.status, (unsigned)ST_EFC_OVERFLOW); continue; }
      float sg = side ? -1.f : 1.f;
      s.efc_type[r] = C_LIM_TEN; s.efc_id[r] = lane;
      s.efc_i0[r] = MD(ten_d0, lane); s.efc_i1[r] = MD(ten_d1, lane);
      s.efc_v0[r] = sg * MD(ten_c0, lane); s.efc_v1[r] = sg * MD(ten_c1, lane);
      s.rowbuf[r] = side ? dhi : dlo; s.efc_floss[r] = 0.f; s.efc_force[r] = MD(ten_invweight0, lane);
    }
  }
  int nsparse = nfl + njl + ntl;
  if (nsparse > EFC_CAP) nsparse = EFC_CAP;
  // contacts: dense rows, lane = contact in chunks of 64 (one chunk in the fast tier).  A contact
  // is kept only if its rows fit: the row offsets are prefix sums, so the kept contacts are a
  // prefix of the list (mj_makeConstraint stops at the first one that does not fit).
  const int ncon = s.ncon;
  int nd = 0, dbase = 0;
  int c_dim[NCH], c_pair[NCH], c_r0[NCH];
  static_assert(2 * (6 - 1) < 16, "rows per contact (condim <= 6) fit the scan's 4 bits");
#pragma unroll
  for (int h = 0; h < NCH; h++) {
    const int c = lane + 64 * h;
    int dim = 0, nr = 0, pair = 0;
    if (c < ncon) {
      pair = s.con_pair[c];
      dim = MD(cp_condim, pair);
      nr = dim == 1 ? 1 : 2 * (dim - 1);
    }
    int ntot;
    const int doff = dbase + wave_excl_scan<4>(nr, lane, &ntot);
    dbase += ntot;
    const bool inc = c < ncon && doff + nr <= MAXDENSE && nsparse + doff + nr <= EFC_CAP;
    {
      const int cand = inc ? doff + nr : 0;
      const int ndh = (int)wave_max((float)cand);
      nd = h == 0 ? ndh : (ndh > nd ? ndh : nd);
    }
    if (c < ncon && !inc) atomicOr(&s.status, (unsigned)ST_EFC_OVERFLOW);
    if (c < ncon) s.con_efc[c] = inc ? nsparse + doff : -1;
    if (inc) {
      const float tran = MD(cp_tran, pair), rot = MD(cp_rot, pair);
      float pm = s.con_dist[c] - (MD(cp_margin, pair) - MD(cp_gap, pair));
      int r = nsparse + doff;
      if (dim == 1) {
        s.efc_type[r] = C_CON_FRICTIONLESS; s.efc_id[r] = c; s.rowbuf[r] = pm; s.efc_floss[r] = 0.f;
        s.efc_force[r] = tran; s.efc_i0[r] = 0; s.efc_i1[r] = 0;
      } else {
        for (int k = 1; k < dim; k++) {
          float fri = MD(cp_friction, 5 * pair + k - 1);
          float dA = tran + fri * fri * (k < 3 ? tran : rot);
          for (int sd = 0; sd < 2; sd++) {
            s.efc_type[r] = C_CON_PYRAMIDAL; s.efc_id[r] = c; s.rowbuf[r] = pm; s.efc_floss[r] = 0.f;
            s.efc_force[r] = dA; s.efc_i0[r] = k; s.efc_i1[r] = sd ? -1 : 1;
            r++;
          }
        }
      }
    }
    c_dim[h] = dim; c_pair[h] = pair; c_r0[h] = inc ? nsparse + doff : -1;
  }
  if (lane == 0) { s.nsparse = nsparse; s.ndense = nd; s.nefc = nsparse + nd; }
  wsync();
  AW_PROF(s, PR_CS_SPARSE);
  // dense J rows, one contact chunk at a time.  The chunk's per-contact model data is gathered
  // first with lane = contact (one round of loads).
#pragma unroll
  for (int h = 0; h < NCH; h++) {
    const int cb = 64 * h;
    unsigned long long c_m1 = 0ull, c_m2 = 0ull;
    int c_root1 = 0, c_root2 = 0;
    float c_f0 = 0.f, c_f1 = 0.f;
    if (lane + cb < ncon) {
      const int pair = c_pair[h];
      c_m1 = MD(cp_mask1, pair); c_m2 = MD(cp_mask2, pair);
      c_root1 = MD(cp_root1, pair); c_root2 = MD(cp_root2, pair);
      c_f0 = MD(cp_friction, 5 * pair); c_f1 = MD(cp_friction, 5 * pair + 1);
    }
    // (contact, dof) work items flattened over the wave: ceil(ncon NV / 64) passes instead of one
    // per contact (hammer: 33 of 64 lanes busy per contact before); each lane takes its contact's
    // data from the contact's lane by a bpermute.  Same arithmetic per entry (r04w A/B: -1.5 %
    // DAPG, -0.3 % random)
    const int nlead = __popcll(__ballot(c_r0[h] >= 0));   // the chunk's kept contacts (a prefix)
    const int total = nlead * NV;
    for (int base = 0; base < total; base += 64) {
      const int w = base + lane;
      const bool act = w < total;
      const int cl = act ? w / NV : 0;
      const int k = act ? w - cl * NV : 0;
      const int c = cb + cl;
      const int r0 = __shfl(c_r0[h], cl, 64);
      const int pr = __shfl(c_pair[h], cl, 64);
      const int cdim = __shfl(c_dim[h], cl, 64);
      const unsigned long long m1 = ((unsigned long long)(unsigned)__shfl((int)(c_m1 >> 32), cl, 64) << 32) |
                                    (unsigned)__shfl((int)c_m1, cl, 64);
      const unsigned long long m2 = ((unsigned long long)(unsigned)__shfl((int)(c_m2 >> 32), cl, 64) << 32) |
                                    (unsigned)__shfl((int)c_m2, cl, 64);
      const int root1 = __shfl(c_root1, cl, 64), root2 = __shfl(c_root2, cl, 64);
      const float f0 = __shfl(c_f0, cl, 64), f1 = __shfl(c_f1, cl, 64);
      if (act) {
        const float* pos = s.con_pos[c];
        float fr[9];
        for (int q = 0; q < 3; q++) { fr[q] = s.con_nrm[c][q]; fr[3 + q] = 0.f; }
        make_frame(fr);
        const float* cd = s.cdof[k];
        float jp[3] = {0, 0, 0}, jr[3] = {0, 0, 0};
        if ((m2 >> k) & 1ull) {
          float off3[3], t[3];
          sub3(off3, pos, s.subcom[root2]);
          cross3(t, cd, off3);
          for (int q = 0; q < 3; q++) { jr[q] += cd[q]; jp[q] += cd[3 + q] + t[q]; }
        }
        if ((m1 >> k) & 1ull) {
          float off3[3], t[3];
          sub3(off3, pos, s.subcom[root1]);
          cross3(t, cd, off3);
          for (int q = 0; q < 3; q++) { jr[q] -= cd[q]; jp[q] -= cd[3 + q] + t[q]; }
        }
        float B[6];
        for (int q = 0; q < 3; q++) { B[q] = dot3(fr + 3 * q, jp); B[3 + q] = dot3(fr + 3 * q, jr); }
        int d = r0 - nsparse;
        if (cdim == 1) {
          jput(m, s, d, k, B[0]);
        } else {
          for (int kk = 1; kk < cdim; kk++) {
            const float fri = kk == 1 ? f0 : (kk == 2 ? f1 : MD(cp_friction, 5 * pr + kk - 1));
            jput(m, s, d, k, B[0] + fri * B[kk]);
            jput(m, s, d + 1, k, B[0] - fri * B[kk]);
            d += 2;
          }
        }
      }
    }
  }
  if (nd > JL) jspill_fence();
  wsync();
  AW_PROF(s, PR_CS_J);
  // impedance, regularisation, reference acceleration
  for (int r = lane; r < s.nefc; r += 64) {
    int t = s.efc_type[r], id = s.efc_id[r];
    gp_t<const float> solref, solimp;
    if (t == C_FRIC_DOF) { solref = MDP(dof_solref, 2 * id); solimp = MDP(dof_solimp, 5 * id); }
    else if (t == C_LIM_JNT) { solref = MDP(jnt_solref, 2 * id); solimp = MDP(jnt_solimp, 5 * id); }
    else if (t == C_LIM_TEN) { solref = MDP(ten_solref, 2 * id); solimp = MDP(ten_solimp, 5 * id); }
    else { int pr = s.con_pair[id]; solref = MDP(cp_solref, 2 * pr); solimp = MDP(cp_solimp, 5 * pr); }
    float pm = s.rowbuf[r];          // stashed by the row assembly above
    float imp = getimpedance(solimp, pm);
    float dmax = clampf(solimp[1], 0.0001f, 0.9999f);
    float K, B;
    if (solref[0] > 0) {
      float tc = solref[0], dr = solref[1];
      if (!(m.disableflags & DSBL_REFSAFE)) tc = fmaxf(tc, 2.f * m.timestep);
      K = 1.f / (dmax * dmax * tc * tc * dr * dr);
      B = 2.f / (dmax * tc);
    } else {
      K = -solref[0] / (dmax * dmax);
      B = -solref[1] / dmax;
    }
    float R = fmaxf((1.f - imp) * s.efc_force[r] / imp, MINVAL);
    s.efc_D[r] = 1.f / R;
    float vel = row_dot<NV>(m, s, r, s.qvel);
    s.efc_aref[r] = -B * vel - K * imp * pm;
  }
  wsync();
}

// ---------------------------------------------------------------------------------------
// Newton solver
// fp32 termination of the Newton solve, per dof: a gradient component below this fraction of the
// summed magnitudes of its terms (sum_k |M_ik a_k|, |qfrc_smooth_i|, sum_r |J_ri f_r|) is rounding
// noise.  Per dof, not over the norm of all dofs: a light object's dofs (relocate's ball) are not
// masked by the hand's large forces (the norm-wide floor stopped one iteration before the fp64
// reference on relocate's first steps, r04c); and over the terms' magnitudes, not the sums' (with
// |Ma_i| etc. a component whose terms cancel never reached its floor: 20-iteration solves, r04h).
#ifndef AW_NT_NOISE_DOF
#define AW_NT_NOISE_DOF 4e-6f
#endif
constexpr float NT_NOISE_DOF = AW_NT_NOISE_DOF;
// why the Newton solve stopped (s.it_newton = iterations + 1000 * reason, aw_forward_dump)
// NT_EXIT_NOROWS: no constraint rows, no Newton solve (forward's default before the solver runs)
enum { NT_EXIT_MAXITER = 0, NT_EXIT_NOSTEP = 1, NT_EXIT_NOISE = 2, NT_EXIT_IMPROVE = 3, NT_EXIT_GRAD = 4, NT_EXIT_NOROWS = 5 };
struct RowR {
  float D, R, floss, Jaref, Jp, force;   // R = 1 / D (the regularisation), formed once per solve
  int st, fr, valid;
};

// mj_solNewton's row cost, force and state at jar.  Branch-free (AW_ROW_EVAL_SELECT, default): every
// zone's value is formed with the same expressions as the branching form and the row's zone selects
// one -- the branching form compiled to four levels of divergent exec-mask regions per row, on every
// line-search derivative (three rows per lane) and cost evaluation.  Bitwise the same results.
#ifndef AW_ROW_EVAL_SELECT
#define AW_ROW_EVAL_SELECT 1
#endif
AW_DEV float row_eval(const RowR& r, float jar, float* force, int* st) {
#if AW_ROW_EVAL_SELECT
  const float f = r.floss, R = r.R;
  const float fq = -r.D * jar, cq = 0.5f * r.D * jar * jar;          // quadratic zone
  const float cn = -f * jar - 0.5f * R * f * f, cp = f * jar - 0.5f * R * f * f;   // linear zones
  const bool neg = jar <= -R * f, pos = jar >= R * f, quad = jar < 0;
  float fo, c;
  int so;
  if (r.fr) {   // a branch on the row type: a slot whose lanes are all contact rows skips this side
    fo = neg ? f : (pos ? -f : fq);
    c = neg ? cn : (pos ? cp : cq);
    so = neg ? S_LNEG : (pos ? S_LPOS : S_QUAD);
  } else {
    fo = quad ? fq : 0.f;
    c = quad ? cq : 0.f;
    so = quad ? S_QUAD : S_SAT;
  }
  *force = r.valid ? fo : 0.f;
  *st = r.valid ? so : S_SAT;
  return r.valid ? c : 0.f;
#else
  if (!r.valid) { *force = 0.f; *st = S_SAT; return 0.f; }
  if (r.fr) {
    float f = r.floss, R = r.R;
    if (jar <= -R * f) { *force = f; *st = S_LNEG; return -f * jar - 0.5f * R * f * f; }
    if (jar >= R * f) { *force = -f; *st = S_LPOS; return f * jar - 0.5f * R * f * f; }
    *force = -r.D * jar; *st = S_QUAD; return 0.5f * r.D * jar * jar;
  }
  if (jar < 0) { *force = -r.D * jar; *st = S_QUAD; return 0.5f * r.D * jar * jar; }
  *force = 0.f; *st = S_SAT; return 0.f;
#endif
}

// J_d' diag(w) J_d over the dense rows (weights w_d in s.rowbuf[nsparse + d], 0 for rows outside
// the quadratic zone) on the matrix cores, written into the packed lower triangle s.L (the
// rank-1 VALU updates per row are in git history, r03p).  v_mfma_f32_16x16x4_f32 takes four rows per
// K-step: lane l supplies A[i = l&15][k = l>>4] = w_d J[d][16 ti + i] and B[k][j = l&15] =
// J[d][16 tj + j] with d = d0 + (l>>4); accumulator register r of lane l is entry
// (16 ti + 4 (l>>4) + r, 16 tj + (l&15)).  Tiles (0,0), (1,0), (1,1) cover rows < 32 and, for
// NV > 32 (hammer 33, relocate 36), (2,0), (2,1), (2,2) the rows from 32.  An MFMA is a k-ordered
// fp32 fma chain, so the dense part is bitwise the per-row rank-1 updates.  The operands of the
// K-step two ahead are loaded before this step's MFMAs (LDS rows, or the global spill block past
// JL): the row loop no longer waits on a load per row.
template <int NV>
AW_DEV void hess_dense_mfma(const DModel& m, Env& s, int lane) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  // three row tiles: rows 32.. come from the third tile's b2 = Jr[32 + (col & 3)] (4 columns)
  static_assert(NV <= 36, "hess_dense_mfma covers at most 36 dofs");
  constexpr bool X2 = NV > 32;
  const int nd = s.ndense, ns = s.nsparse;
  const int sub = lane >> 4, col = lane & 15;
  f4 c00 = {0.f, 0.f, 0.f, 0.f}, c10 = c00, c11 = c00, c20 = c00, c21 = c00, c22 = c00;
  auto load = [&](int d0, float& w, float& b0, float& b1, float& b2) {
    const int d = d0 + sub;
    const bool v = d < nd;
    const int dd = v ? d : d0;   // a row of this K-step (d0 < nd): in the same storage as the rest
    // JL is a multiple of 4: a K-step's rows are all in LDS or all in the spill block
    const float* Jr = d0 < JL ? &s.J[dd][0] : (const float*)jspill_row(m, s, dd);
    const float wl = s.rowbuf[ns + dd];   // dd is a row of this K-step: loaded unconditionally, then
    w = v ? wl : 0.f;                     // selected (a conditional load is an exec-mask branch)
    b0 = Jr[col];
    b1 = Jr[16 + col];
    b1 = 16 + col < NV ? b1 : 0.f;
    b2 = X2 ? Jr[32 + (col & 3)] : 0.f;
    b2 = 32 + col < NV ? b2 : 0.f;
  };
  float w = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f;
  if (nd > 0) load(0, w, b0, b1, b2);
  // two K-steps of look-ahead: a K-step's loads (LDS, or L2 for the spill block) get two steps of
  // MFMAs to land (r05u: -0.3 % random, -0.1 % DAPG against one step)
  float w2 = 0.f, b02 = 0.f, b12 = 0.f, b22 = 0.f;
  if (nd > 4) load(4, w2, b02, b12, b22);
  for (int d0 = 0; d0 < nd; d0 += 4) {
    float wn = 0.f, b0n = 0.f, b1n = 0.f, b2n = 0.f;
    if (d0 + 8 < nd) load(d0 + 8, wn, b0n, b1n, b2n);
    const float a0 = w * b0, a1 = w * b1;
    c00 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, c00, 0, 0, 0);
    c10 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, c10, 0, 0, 0);
    c11 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, c11, 0, 0, 0);
    if (X2) {
      const float a2 = w * b2;
      c20 = __builtin_amdgcn_mfma_f32_16x16x4f32(a2, b0, c20, 0, 0, 0);
      c21 = __builtin_amdgcn_mfma_f32_16x16x4f32(a2, b1, c21, 0, 0, 0);
      c22 = __builtin_amdgcn_mfma_f32_16x16x4f32(a2, b2, c22, 0, 0, 0);
    }
    w = w2; b0 = b02; b1 = b12; b2 = b22;
    w2 = wn; b02 = b0n; b12 = b1n; b22 = b2n;
  }
  // lower triangle + row padding (entries j <= (i | 3)) of every row, each written once
  auto put = [&](const f4& c, int ti, int tj) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int i = 16 * ti + 4 * sub + r, j = 16 * tj + col;
      if (i < NV && j <= (i | 3)) s.L[tri(i) + j] = c[r];
    }
  };
  put(c00, 0, 0);
  put(c10, 1, 0);
  put(c11, 1, 1);
  if (X2) {
    put(c20, 2, 0);
    put(c21, 2, 1);
    put(c22, 2, 2);
  }
}

template <int NV, bool ROWST = false>
AW_DEV void solve_newton(const DModel& m, Env& s, int lane_nt, const float (&Mrow)[NV], float& a, float qfrc_smooth,
                         float qacc_smooth, float* rowst = nullptr) {
  const int lane = lane_nt;
  const int nefc = s.nefc;
  const float fs = lane < NV ? qfrc_smooth : 0.f;
  const float a0 = lane < NV ? qacc_smooth : 0.f;
  RowR rr[NRL];
#pragma unroll
  for (int h = 0; h < NRL; h++) {
    int r = lane + 64 * h;
    rr[h].valid = r < nefc;
    int rc = rr[h].valid ? r : 0;
    rr[h].D = s.efc_D[rc];
    rr[h].R = 1.f / rr[h].D;
    rr[h].floss = s.efc_floss[rc];
    int t = s.efc_type[rc];
    rr[h].fr = (t == C_FRIC_DOF || t == C_FRIC_TEN);
    rr[h].Jaref = rr[h].Jp = rr[h].force = 0.f;
    rr[h].st = S_SAT;
  }
  const float scale = 1.f / (m.meaninertia * (float)(NV > 1 ? NV : 1));
  float Ma;
  // both starting points (qacc_smooth, warmstart) in one pass over M and the rows, then the
  // cheaper one is kept (mj_solNewton: the warmstart when its cost is strictly lower); r04h A/B
  // against two set-point passes: -0.6 % random, -1.0 % DAPG
  float cost;
  {
    const bool ws = !(m.disableflags & DSBL_WARMSTART);
    const float aw = ws && lane < NV ? s.warm[lane] : 0.f;
    if (lane < NV) { s.vec[lane] = a0; s.vec2[lane] = aw; }
    wsync();
    const float Ma0 = matvec_lds<NV>(Mrow, s.vec);
    const float Maw = matvec_lds<NV>(Mrow, s.vec2);
    float j0[NRL], jw[NRL];
#pragma unroll
    for (int h = 0; h < NRL; h++) {
      const int r = lane + 64 * h;
      j0[h] = jw[h] = 0.f;
      if (r < nefc) {
        row_dot2<NV>(m, s, r, s.vec, s.vec2, j0[h], jw[h]);
        const float ar = s.efc_aref[r];
        j0[h] -= ar;
        jw[h] -= ar;
      }
    }
    wsync();
    float c0 = 0.f, cwl = 0.f, fw[NRL];
    int sw[NRL];
#pragma unroll
    for (int h = 0; h < NRL; h++) {
      c0 += row_eval(rr[h], j0[h], &rr[h].force, &rr[h].st);
      cwl += row_eval(rr[h], jw[h], &fw[h], &sw[h]);
    }
    cost = wave_sum(c0);   // the Gauss term is 0 at qacc_smooth
    const float cw = ws ? 0.5f * wave_sum(lane < NV ? (Maw - fs) * (aw - a0) : 0.f) + wave_sum(cwl) : cost;
    const bool take_w = ws && cw < cost;
    cost = take_w ? cw : cost;
    a = take_w ? aw : (lane < NV ? a0 : 0.f);
    Ma = take_w ? Maw : Ma0;
#pragma unroll
    for (int h = 0; h < NRL; h++) {
      rr[h].Jaref = take_w ? jw[h] : j0[h];
      rr[h].force = take_w ? fw[h] : rr[h].force;
      rr[h].st = take_w ? sw[h] : rr[h].st;
    }
  }
  // fp32 noise scale of each gradient component Ma_i - fs_i - (J'f)_i: the magnitudes of all of
  // its terms, sum_k |M_ik a_k| + |fs_i| + sum_r |J_ri f_r| (the magnitude of a sum would miss the
  // cancellation inside it)
  float gnoise = 0.f;
  auto gradient = [&]() {
#pragma unroll
    for (int h = 0; h < NRL; h++) { int r = lane + 64 * h; if (r < nefc) s.rowbuf[r] = rr[h].force; }
    if (lane < NV) s.hdiag[lane] = fabsf(a);
    wsync();
    float jfa;
    float jf = jt_mul<NV, true>(m, s, lane, &jfa);
    float maa = 0.f;
#pragma unroll
    for (int q = 0; q < (NV + 3) / 4; q++) {
      const float4 v = *reinterpret_cast<const float4*>(s.hdiag + 4 * q);
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int t = 0; t < 4; t++)
        if (4 * q + t < NV) maa = fmaf(fabsf(Mrow[4 * q + t]), vv[t], maa);
    }
    gnoise = lane < NV ? maa + fabsf(fs) + jfa : 0.f;
    return lane < NV ? Ma - fs - jf : 0.f;
  };
  float grad = gradient();
  AW_PROF(s, PR_NT_INIT);
  int iter = 0;
  // The Hessian factor persists across iterations in LDS (s.L, packed rows; the backward solve
  // reads it there anyway).  An iteration in which no row changed its quadratic state has the
  // same Hessian as the previous one: its factor is reloaded instead of rebuilt (4 % of k_step on
  // the A/B; rank-1 up / downdates for a few changed rows measured slower than refactoring).
  float invd = 1.f;
  int why = NT_EXIT_MAXITER;   // which test ended the solve (introspection: aw_forward_dump)
  bool inH[NRL];
#pragma unroll
  for (int h = 0; h < NRL; h++) inH[h] = false;
  const int li = lane < NV ? lane : NV - 1;
  for (; iter < m.iterations; iter++) {
    const int lane = opaque(lane_nt);   // per-iteration lane id: its compares stay inside the loop
    float H[NV];
    bool full = iter == 0;
    if (!full) {
      bool chg = false;
#pragma unroll
      for (int h = 0; h < NRL; h++) chg |= rr[h].valid && ((rr[h].st == S_QUAD) != inH[h]);
      full = __ballot(chg) != 0ull;
    }
    if (!full) {
      // this lane's factor row from LDS (16-byte reads; entries above the diagonal are padding)
      const float* Lr = &s.L[tri(li)];
#pragma unroll
      for (int q = 0; q < (NV + 3) / 4; q++) {
        const float4 v = q * 4 <= li ? *reinterpret_cast<const float4*>(Lr + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int t = 0; t < 4; t++)
          if (4 * q + t < NV) H[4 * q + t] = vv[t];
      }
    }
    if (full) {
    // Hessian H = M + J' D_quad J, lower triangle only (the right-looking factorisation never
    // reads a lane's entries above its diagonal).  Sparse rows (<= 2 dofs: frictionloss, joint
    // and tendon limits) are scattered with LDS atomics into the packed lower triangle in the
    // factor's own storage s.L (dead until chol_store), which each lane then adds to its row
    // with 16-byte reads -- a two-dof tendon row's off-diagonal term lands in ONE entry, where
    // adding it in registers took a 2 x NV select chain per row.  Dense rows: rank-1 updates
    // with the row broadcast from LDS.
    // Dense part J_d' D J_d on the matrix cores (hess_dense_mfma above): every lower-triangle
    // entry (and the row padding) of s.L is written by exactly one plain store, then the sparse
    // rows are added with LDS atomics as below.
#pragma unroll
    for (int h = 0; h < NRL; h++) {
      int r = lane + 64 * h;
      if (r < nefc) s.rowbuf[r] = rr[h].st == S_QUAD ? rr[h].D : 0.f;
    }
    wsync();
    hess_dense_mfma<NV>(m, s, lane);
    wsync();
#pragma unroll
    for (int h = 0; h < NRL; h++) {
      int r = lane + 64 * h;
      if (r < nefc) {
        float w = rr[h].st == S_QUAD ? rr[h].D : 0.f;
        if (r < s.nsparse && w != 0.f) {
          int i0 = s.efc_i0[r], i1 = s.efc_i1[r];
          float v0 = s.efc_v0[r], v1 = s.efc_v1[r];
          atomicAdd(&s.L[tri(i0) + i0], w * v0 * v0);
          if (i1 >= 0) {
            atomicAdd(&s.L[tri(i1) + i1], w * v1 * v1);
            const int hi = i0 > i1 ? i0 : i1, lo = i0 > i1 ? i1 : i0;
            atomicAdd(&s.L[tri(hi) + lo], w * v0 * v1);
          }
        }
      }
    }
    wsync();
    AW_PROF(s, PR_NT_HSPARSE);
    {
      const float* Lr = &s.L[tri(li)];
#pragma unroll
      for (int q = 0; q < (NV + 3) / 4; q++) {
        const float4 v = q * 4 <= li ? *reinterpret_cast<const float4*>(Lr + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int t = 0; t < 4; t++)
          if (4 * q + t < NV) H[4 * q + t] = Mrow[4 * q + t] + vv[t];
      }
    }
    AW_PROF(s, PR_NT_HOFFD);
    wsync();
    AW_PROF(s, PR_NT_HESS);
    chol_factor<NV>(H, lane, invd, s);
    chol_store<NV>(H, lane, s);
    wsync();
    }
#pragma unroll
    for (int h = 0; h < NRL; h++) inH[h] = rr[h].valid && rr[h].st == S_QUAD;
    AW_PROF(s, PR_NT_CHOL);
    float p = -chol_solve<NV>(H, invd, grad, lane, s);
    AW_PROF(s, PR_NT_SOLVE);
    // exact line search on the piecewise-quadratic 1-D cost
    if (lane < NV) s.vec[lane] = p;
    wsync();
    float Mp = matvec_lds<NV>(Mrow, s.vec);
    float c0 = wave_sum(lane < NV ? p * (Ma - fs) : 0.f);
    float c1 = wave_sum(lane < NV ? p * Mp : 0.f);
#pragma unroll
    for (int h = 0; h < NRL; h++) {
      int r = lane + 64 * h;
      rr[h].Jp = r < nefc ? row_dot<NV>(m, s, r, s.vec) : 0.f;
    }
    wsync();
    auto deriv = [&](float alpha, float* d1, float* d2) {
      float g1 = 0.f, g2 = 0.f;
#pragma unroll
      for (int h = 0; h < NRL; h++) {
        float jp = rr[h].Jp;
        if (!rr[h].valid || jp == 0.f) continue;
        float f;
        int st;
        row_eval(rr[h], rr[h].Jaref + alpha * jp, &f, &st);
        g1 -= f * jp;
        if (st == S_QUAD) g2 += rr[h].D * jp * jp;
      }
      *d1 = c0 + alpha * c1 + wave_sum(g1);
      *d2 = c1 + wave_sum(g2);
    };
    float d1, d2;
    deriv(0.f, &d1, &d2);
    float alpha = 0.f;
    if (d1 < 0.f) {
      float tol = 1e-6f * fabsf(d1), lo = 0.f, hi = -1.f;
      for (int it = 0; it < 50; it++) {
        float an = alpha - d1 / d2;
        if (hi >= 0.f && (an <= lo || an >= hi)) an = 0.5f * (lo + hi);
        if (an == alpha) break;
        alpha = an;
        deriv(alpha, &d1, &d2);
        if (d1 < 0.f) lo = alpha; else hi = alpha;
        if (fabsf(d1) <= tol) break;
      }
    }
    AW_PROF(s, PR_NT_LS);
    if (alpha == 0.f) { iter++; why = NT_EXIT_NOSTEP; break; }
    // the rows' cost before the step, per lane (the improvement below is formed from per-row
    // differences, not as the difference of two whole costs)
    float rc_old = 0.f;
#pragma unroll
    for (int h = 0; h < NRL; h++) {
      float f;
      int st;
      rc_old += row_eval(rr[h], rr[h].Jaref, &f, &st);
    }
    a += alpha * p;
    Ma += alpha * Mp;
#pragma unroll
    for (int h = 0; h < NRL; h++) rr[h].Jaref += alpha * rr[h].Jp;
    // mj_solNewton's improvement = scale (oldcost - cost) without the fp32 cancellation of two
    // whole costs: the smooth part's change along the line is exactly alpha c0 + alpha^2 c1 / 2
    // (M a0 = qfrc_smooth, so p' M (a - a0) = c0), the rows' change is summed row by row.  (The
    // difference of the two fp32 costs carried their rounding noise, ~1e-7 of the cost: r04f/g
    // A/B, C3 hammer 8 -> 0 misses.)
    float rc_new = 0.f;
#pragma unroll
    for (int h = 0; h < NRL; h++) rc_new += row_eval(rr[h], rr[h].Jaref, &rr[h].force, &rr[h].st);
    const float dcost = -(alpha * c0 + 0.5f * alpha * alpha * c1 + wave_sum(rc_new - rc_old));
    grad = gradient();
    float gn = sqrtf(wave_sum(grad * grad));
    float improvement = scale * dcost, gradnorm = scale * gn;
    // fp32 termination: every gradient component at the rounding floor of its own terms (Ma,
    // qfrc_smooth, J'f) cannot shrink further -- the fp64 reference would already stop on its
    // 1e-8 test here; an extra Newton step in fp32 only re-solves the same active set.  (Without
    // this exit: +8 % k_step, r04g.)
    if (__ballot(lane < NV && fabsf(grad) > NT_NOISE_DOF * gnoise) == 0ull) { iter++; why = NT_EXIT_NOISE; break; }
    AW_PROF(s, PR_NT_UPD);
    if (improvement < m.tolerance) { iter++; why = NT_EXIT_IMPROVE; break; }
    if (gradnorm < m.tolerance) { iter++; why = NT_EXIT_GRAD; break; }
  }
  if (lane == 0) s.it_newton = iter + 1000 * why;
  AW_PROF_ADD(s, PR_NEWTON_IT, iter);
  AW_PROF_ADD(s, PR_NEFC, nefc);
  AW_PROF_ADD(s, PR_NCON, s.ncon);
#pragma unroll
  for (int h = 0; h < NRL; h++) {
    int r = lane + 64 * h;
    if (r < nefc) s.efc_force[r] = rr[h].force;
    if (ROWST && r < nefc) rowst[r] = (float)rr[h].st;
  }
  wsync();
}

// ---------------------------------------------------------------------------------------
// noslip: PGS over frictionloss rows and opposing pyramid-edge pairs, no regularisation
// Row space (default).  mj_solNoSlip is projected Gauss-Seidel over the noslip rows: the
// frictionloss row of every dof (J = e_d) and the opposing pyramid-edge pairs.  A pair's update
// keeps f1 + f2 and moves f1 - f2 (d2 = -d1), so it acts through its difference row
// jd = J_e - J_e+1.  With B stacking those rows, the residuals move through the constant
// A = B inv(M) B'.  Each lane owns one row -- lanes [0, NV) the dof rows, lanes [NV, NV + npl)
// the first npl <= 64 - NV pairs -- and keeps that row of A in VGPRs: dof lane d holds
// inv(M)[d][.] and xd_p[d] = (inv(M) jd_p')[d]; pair lane q holds xd_q[.] and
// G_q[p] = jd_q . xd_p.  The residual vector R (dof lanes: qacc; pair lanes: jd_q . qacc) then
// moves by ONE fma per row step, for dof rows and pairs alike: a step is
// fma -> med3 -> readlane -> fma on the serial chain, and qacc is R's dof lanes at the end.
// Row constants: y = cb - R ca is the unclamped update, d = med3(y, lo, hi) with
// lo = -lim - fa, hi = lim + fb (dof rows: fa = f, fb = -f, lim = frictionloss; pairs: fa = f1,
// fb = f2, lim = 0), and the row's cost change is diag d (d / 2 - y).  Pairs past the lanes
// (npr > npl, rare) rebuild their column of A every sweep.
template <int TASK>
AW_DEV void solve_noslip(const DModel& m, Env& s, int lane_ns, const float (&Mrow)[Tree<TASK>::NV], float& qacc) {
  const int lane = lane_ns;
  constexpr int NV = Tree<TASK>::NV;
  constexpr int NPL = 64 - NV;          // pairs with a lane of their own
  constexpr int XS = (NV + 3) & ~3;     // row stride of the xd transpose buffer (16-byte rows)
  static_assert(NPL * XS * sizeof(float) <= offsetof(Env, qpos), "xd transpose buffer exceeds the phase-K/S union");
  float* Xb = reinterpret_cast<float*>(&s);   // phase-K / phase-S union: dead during noslip
  const int nsparse = s.nsparse, ndense = s.ndense;
  // dof columns of this lane's row of A: inv(M) from the tree factor of M (aw_tree.h)
  float Am[NV];
  {
    float row[NV];
#pragma unroll
    for (int k = 0; k < NV; k++) row[k] = Mrow[k];
    float invd;
    tree_factor<TASK>(row, invd, lane);
    tree_inverse<TASK>(row, invd, lane, Am);
  }
  if (lane >= NV) {
#pragma unroll
    for (int k = 0; k < NV; k++) Am[k] = 0.f;
  }
  const int li = lane < NV ? lane : 0;
  const float lm = lane < NV ? 1.f : 0.f;
  wsync();
  AW_PROF(s, PR_NS_MINV);
  // dof rows: lanes without an active frictionloss row propose exactly zero (ca = cb = 0, no clamp)
  const bool use_fl = !(m.disableflags & DSBL_FRICTIONLOSS);
  const int flrow = lane < NV ? MD(fl_row, lane) : -1;
  const bool has_fl = flrow >= 0 && flrow < nsparse;
  float ca = 0.f, cb = 0.f, lim = 0.f, fa = 0.f, fb = 0.f, diag = 0.f;
  int rowe = 0;   // pair lanes: the pair's first dense row
  {
    float dg = 0.f;   // inv(M)[lane][lane]
#pragma unroll
    for (int k = 0; k < NV; k++) dg = k == lane ? Am[k] : dg;
    if (has_fl) { fa = s.efc_force[flrow]; fb = -fa; }
    if (use_fl && has_fl && dg >= MINVAL) {
      ca = 1.0f / dg;
      cb = s.efc_aref[flrow] * ca;
      lim = s.efc_floss[flrow];
      diag = dg;
    } else if (lane < NV) {
      lim = 3.0e38f;
    }
  }
  float R = lane < NV ? qacc : 0.f;
  // column of A for the pair starting at dense row e: col = A[lane][0..NV) . jd (dof lanes: xd,
  // pair lanes with their dof columns loaded: G_q); jd = J_e - J_e+1 at this lane's dof
  auto jval = [&](int d) { return lm * (d < JL ? s.J[d][li] : jspill_row(m, s, d)[li]); };
  auto pair_col = [&](int e, float& jd, float& col) {
    float a = 0.f;
    if (e + 1 < JL) {
#pragma unroll
      for (int j = 0; j < NV; j++) a = fmaf(Am[j], s.J[e][j] - s.J[e + 1][j], a);
      jd = lm * (s.J[e][li] - s.J[e + 1][li]);
    } else {
      const float dl = jval(e) - jval(e + 1);
#pragma unroll
      for (int j = 0; j < NV; j++) a = fmaf(Am[j], rlane(dl, j), a);
      jd = dl;
    }
    col = a;
  };
  // candidate pairs: first rows e of opposing pyramid-edge pairs, in row order, found by a ballot
  // over the dense rows (no serial scan).  The first NPL get a lane: xd = inv(M) jd' goes to the
  // transpose buffer here, and the pair lane forms its own constants below (K = jd . xd and
  // jd . qacc in-lane, no wave reductions on the scan).  A pair with K < MINVAL keeps its lane but
  // is inert (ca = cb = 0: its update is exactly zero).  Pairs past NPL keep their constants in
  // lane p - NPL.
  unsigned long long cmask[NDCH];
#pragma unroll
  for (int h = 0; h < NDCH; h++) {
    const int e = lane + 64 * h;
    bool c = e + 1 < ndense;
    if (c) c = s.efc_type[nsparse + e] == C_CON_PYRAMIDAL && s.efc_i1[nsparse + e] == 1;
    cmask[h] = __ballot(c);
  }
  int npr = 0;
  // pairs past the lanes: pair NPL + 64 xc + l keeps its constants in lane l of chunk xc
  constexpr int NXCH = (MAXDENSE / 2 - NPL + 63) / 64 > 0 ? (MAXDENSE / 2 - NPL + 63) / 64 : 1;
  int ex_e[NXCH];
  float ex_ca[NXCH], ex_cb[NXCH], ex_K[NXCH], ex_fa[NXCH], ex_fb[NXCH];
#pragma unroll
  for (int xc = 0; xc < NXCH; xc++) { ex_e[xc] = 0; ex_ca[xc] = ex_cb[xc] = ex_K[xc] = ex_fa[xc] = ex_fb[xc] = 0.f; }
  // with >= 4 pair lanes the lane pairs' xd = inv(M) jd' come from one MFMA product below
  // (DAPG +2.7 %, random +-0, r03zg, against per-pair VALU products)
  int npr_all = 0;
#pragma unroll
  for (int h = 0; h < NDCH; h++) npr_all += __popcll(cmask[h]);
  // (hammer; relocate's 36 x 36 inv(M) does not fit the staging area, door / pen have 34 pair lanes)
  // the staging writes NV rows of inv(M) and the product writes rows p < 32 of the buffer
  constexpr bool X_FIT = NPL <= 32 && (NV > 32 ? NV : 32) * XS * sizeof(float) <= offsetof(Env, qpos);
  const bool x_mfma = X_FIT && (npr_all < NPL ? npr_all : NPL) >= 4;
#pragma unroll
  for (int h = 0; h < NDCH; h++) {
    unsigned long long mk = cmask[h];
    while (mk) {
      const int e = 64 * h + __builtin_ctzll(mk);
      mk &= mk - 1ull;
      const int p = npr++;
      if (p < NPL) {
        if (!x_mfma) {
          float jd, xd;
          pair_col(e, jd, xd);
          if (lane < NV) Xb[p * XS + lane] = xd;
        }
        if (lane == NV + p) rowe = e;
      } else {
        float jd, xd;
        pair_col(e, jd, xd);
        const float K = wave_sum(jd * xd);
        const bool ok = K >= MINVAL;
        const float ik = ok ? 1.0f / K : 0.f;
        const float ard = s.efc_aref[nsparse + e] - s.efc_aref[nsparse + e + 1];
        const int x = p - NPL;
#pragma unroll
        for (int xc = 0; xc < NXCH; xc++)
          if (xc == (x >> 6) && lane == (x & 63)) {
            ex_e[xc] = e; ex_ca[xc] = ik; ex_cb[xc] = ard * ik; ex_K[xc] = ok ? K : 0.f;
            ex_fa[xc] = s.efc_force[nsparse + e];
            ex_fb[xc] = s.efc_force[nsparse + e + 1];
          }
      }
    }
  }
  if constexpr (X_FIT) {
    static_assert(32 * XS * sizeof(float) <= offsetof(Env, qpos), "x_mfma output rows exceed the staging area");
    if (x_mfma) {
      // X = inv(M) Jd' (NV x npl, K = NV) on the matrix cores: A rows are inv(M)'s rows (each dof
      // lane stages its row Am in the transpose buffer), B columns the pairs' difference rows
      // jd_p = J_e - J_e+1 (Jacobian rows in LDS / global spill; e by a shuffle from the pair's
      // lane); the product is written over the staging as the transpose buffer rows Xb[p][i].
      typedef float f4 __attribute__((ext_vector_type(4)));
      constexpr int NTI = (NV + 15) / 16;
      const int np = npr < NPL ? npr : NPL;
      if (lane < NV) {
#pragma unroll
        for (int q = 0; q < XS / 4; q++) {
          float4 v;
          v.x = 4 * q + 0 < NV ? Am[4 * q + 0 < NV ? 4 * q + 0 : 0] : 0.f;
          v.y = 4 * q + 1 < NV ? Am[4 * q + 1 < NV ? 4 * q + 1 : 0] : 0.f;
          v.z = 4 * q + 2 < NV ? Am[4 * q + 2 < NV ? 4 * q + 2 : 0] : 0.f;
          v.w = 4 * q + 3 < NV ? Am[4 * q + 3 < NV ? 4 * q + 3 : 0] : 0.f;
          *reinterpret_cast<float4*>(Xb + lane * XS + 4 * q) = v;
        }
      }
      wsync();
      const int sub = lane >> 4, col = lane & 15;
      const bool two = np > 16;
      const float* r0[2];
      const float* r1[2];
      bool pv[2];
#pragma unroll
      for (int t = 0; t < 2; t++) {
        const int q = 16 * t + col;
        pv[t] = q < np;
        const int es = __shfl(rowe, (NV + q) & 63, 64);   // every lane takes part in the shuffle
        const int e = pv[t] ? es : 0;
        r0[t] = e < JL ? &s.J[e][0] : (const float*)jspill_row(m, s, e);
        r1[t] = e + 1 < JL ? &s.J[e + 1][0] : (const float*)jspill_row(m, s, e + 1);
      }
      f4 c[NTI][2];
#pragma unroll
      for (int ti = 0; ti < NTI; ti++) c[ti][0] = c[ti][1] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < XS / 4; ks++) {
        const int k = 4 * ks + sub;
        const bool kv = k < NV;
        const int kk = kv ? k : 0;
        float a[NTI], b[2];
#pragma unroll
        for (int ti = 0; ti < NTI; ti++) {
          const int i = 16 * ti + col;
          const float xv = Xb[(i < NV ? i : 0) * XS + kk];
          a[ti] = (kv && i < NV) ? xv : 0.f;
        }
#pragma unroll
        for (int t = 0; t < 2; t++) {
          const float jv = r0[t][kk] - r1[t][kk];   // valid rows (e = 0 / kk = 0 stand-ins)
          b[t] = (kv && pv[t]) ? jv : 0.f;
        }
#pragma unroll
        for (int ti = 0; ti < NTI; ti++) {
          c[ti][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ti], b[0], c[ti][0], 0, 0, 0);
          if (two) c[ti][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ti], b[1], c[ti][1], 0, 0, 0);
        }
      }
      wsync();
      // every staged inv(M) operand has returned (the MFMAs consumed it): overwrite with Xb[p][i]
#pragma unroll
      for (int ti = 0; ti < NTI; ti++)
#pragma unroll
        for (int t = 0; t < 2; t++) {
          if (t == 1 && !two) continue;
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int i = 16 * ti + 4 * sub + r, p = 16 * t + col;
            if (i < NV) Xb[p * XS + i] = c[ti][t][r];
          }
        }
    }
  }
  const int npl = npr < NPL ? npr : NPL;
  if (lane < NV) s.rowbuf[lane] = R;   // qacc for the pair lanes' jd . qacc (rowbuf is rewritten after noslip)
  wsync();
  const bool pl = lane >= NV && lane < NV + npl;
  // pair lanes: the dof columns of their row, xd_q, from the transpose buffer
  if (pl) {
    const float* xr = Xb + (lane - NV) * XS;
#pragma unroll
    for (int q = 0; q < XS / 4; q++) {
      const float4 v = *reinterpret_cast<const float4*>(xr + 4 * q);
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int t = 0; t < 4; t++)
        if (4 * q + t < NV) Am[4 * q + t] = vv[t];
    }
  }
  // With >= 4 pair lanes (NPL <= 32) the pair-pair block G is formed on the matrix cores below; its
  // diagonal is K = jd_q . xd_q and one extra B column (qacc, at index npl) gives S = jd_q . qacc, so
  // the pair lanes' own difference rows (per-lane Jacobian rows: 8-way LDS bank conflicts) are not read
  // at all (AW_NS_KS_MFMA; the same products in the same k order as the VALU chains below)
#ifndef AW_NS_KS_MFMA
#define AW_NS_KS_MFMA 1
#endif
  const bool g_mfma_ks = AW_NS_KS_MFMA && NPL <= 32 && npl >= 4;
  if (pl) {
    fa = s.efc_force[nsparse + rowe];
    fb = s.efc_force[nsparse + rowe + 1];
  }
  // pair lanes: their difference row jd_q (registers), K = jd_q . xd_q, jd_q . qacc and constants
  float jq[NV];
  if (!g_mfma_ks) {
    const int e = pl ? rowe : 0;
    if (e + 1 < JL) {
#pragma unroll
      for (int d = 0; d < NV; d++) jq[d] = s.J[e][d] - s.J[e + 1][d];
    } else {
      auto jat = [&](int r, int d) { return r < JL ? s.J[r][d] : jspill_row(m, s, r)[d]; };
#pragma unroll
      for (int d = 0; d < NV; d++) jq[d] = jat(e, d) - jat(e + 1, d);
    }
    float K = 0.f, S = 0.f;
#pragma unroll
    for (int q = 0; q < XS / 4; q++) {
      const float4 v = *reinterpret_cast<const float4*>(s.rowbuf + 4 * q);
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int t = 0; t < 4; t++)
        if (4 * q + t < NV) {
          K = fmaf(jq[4 * q + t], Am[4 * q + t], K);
          S = fmaf(jq[4 * q + t], vv[t], S);
        }
    }
    if (pl) {
      const bool ok = K >= MINVAL;
      ca = ok ? 1.0f / K : 0.f;
      cb = (s.efc_aref[nsparse + e] - s.efc_aref[nsparse + e + 1]) * ca;
      diag = ok ? K : 0.f;
      R = S;
    }
  }
  wsync();
  // pair columns of every lane's row: dof lanes read xd_p[lane] back from the transpose buffer;
  // pair lanes form G_q[p] = jd_q . xd_p from their difference row (registers) and xd_p
  // (broadcast reads of the buffer)
  float Ap[NPL];
  {
    // G = Jd Xd' (npl x npl, K = NV) on the matrix cores when there are enough pairs: A rows are
    // the pairs' difference rows jd_q = J_e - J_e+1 read from the Jacobian (LDS rows / global
    // spill rows; the pair's row index e comes from its lane by a shuffle), B rows the xd_p in
    // the transpose buffer.  Dof lanes take their xd_p[lane] first; the buffer is then reused to
    // stage G (row stride 32) and each pair lane reads its row back.
    bool g_mfma = false;
    if constexpr (NPL <= 32) {
      static_assert(32 * 32 * sizeof(float) <= offsetof(Env, qpos), "G staging exceeds the phase-K/S union");
      if (npl >= 4) {
        g_mfma = true;
        typedef float f4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int p = 0; p < NPL; p++) Ap[p] = Xb[p * XS + li];   // entries p >= npl are never read
        const int sub = lane >> 4, col = lane & 15;
        const int ncol = g_mfma_ks ? npl + 1 : npl;   // + the qacc column (S)
        const bool two = ncol > 16;
        const float* r0[2];
        const float* r1[2];
        bool qv[2], pv[2];
#pragma unroll
        for (int t = 0; t < 2; t++) {
          const int q = 16 * t + col;
          qv[t] = q < npl;
          pv[t] = q < npl;
          // every lane takes part in the shuffle (a lane read while inactive returns nothing)
          const int es = __shfl(rowe, (NV + q) & 63, 64);
          const int e = qv[t] ? es : 0;
          r0[t] = e < JL ? &s.J[e][0] : (const float*)jspill_row(m, s, e);
          r1[t] = e + 1 < JL ? &s.J[e + 1][0] : (const float*)jspill_row(m, s, e + 1);
        }
        f4 c00 = {0.f, 0.f, 0.f, 0.f}, c01 = c00, c10 = c00, c11 = c00;
#pragma unroll
        for (int ks = 0; ks < XS / 4; ks++) {
          const int k = 4 * ks + sub;
          const bool kv = k < NV;
          const int kk = kv ? k : 0;
          float a[2], b[2];
#pragma unroll
          for (int t = 0; t < 2; t++) {
            // operands read from valid addresses (stand-in row 0 / column 0), then selected; the
            // compiler still sinks some reads under the lane conditions, which measured faster than
            // forcing them all (r06v: +0.8 % DAPG with the reads pinned)
            const float jv = r0[t][kk] - r1[t][kk], xv = Xb[(16 * t + col) * XS + kk], qa = s.rowbuf[kk];
            a[t] = (kv && qv[t]) ? jv : 0.f;
            b[t] = (kv && pv[t]) ? xv : 0.f;
            if (g_mfma_ks && 16 * t + col == npl) b[t] = kv ? qa : 0.f;   // qacc (rowbuf, above)
          }
          c00 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c00, 0, 0, 0);
          if (two) {
            c01 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[1], c01, 0, 0, 0);
            c10 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[0], c10, 0, 0, 0);
            c11 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c11, 0, 0, 0);
          }
        }
        wsync();
        float* Gb = Xb;   // [32][32]: every operand read above has returned (the MFMAs consumed it)
        auto put = [&](const f4& c, int ti, int tj) {
#pragma unroll
          for (int r = 0; r < 4; r++) Gb[(16 * ti + 4 * sub + r) * 32 + 16 * tj + col] = c[r];
        };
        put(c00, 0, 0);
        if (two) {
          put(c01, 0, 1);
          put(c10, 1, 0);
          put(c11, 1, 1);
        }
        wsync();
        if (pl) {
          const float* gr = Gb + (lane - NV) * 32;
#pragma unroll
          for (int q = 0; q < (NPL + 3) / 4; q++) {
            const float4 v = *reinterpret_cast<const float4*>(gr + 4 * q);
            const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int t = 0; t < 4; t++)
              if (4 * q + t < NPL) Ap[4 * q + t] = vv[t];
          }
          if (g_mfma_ks) {
            const float K = gr[lane - NV], S = gr[npl];
            const bool ok = K >= MINVAL;
            ca = ok ? 1.0f / K : 0.f;
            cb = (s.efc_aref[nsparse + rowe] - s.efc_aref[nsparse + rowe + 1]) * ca;
            diag = ok ? K : 0.f;
            R = S;
          }
        }
        wsync();
      }
    }
#pragma unroll
    for (int p = 0; p < NPL; p++) {
      if (p < npl && !g_mfma) {
        const float* xr = Xb + p * XS;
        float g = 0.f;
#pragma unroll
        for (int q = 0; q < XS / 4; q++) {
          const float4 v = *reinterpret_cast<const float4*>(xr + 4 * q);
          const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int t = 0; t < 4; t++)
            if (4 * q + t < NV) g = fmaf(jq[4 * q + t], vv[t], g);
        }
        Ap[p] = lane < NV ? xr[li] : g;
      }
    }
  }
  AW_PROF(s, PR_NS_SETUP);
  if (lane == 0) s.it_noslip = 0;
  const float scale = 1.f / (m.meaninertia * (float)(NV > 1 ? NV : 1));
  for (int it = 0; it < m.noslip_iterations; it++) {
    const int lane = opaque(lane_ns);   // per-sweep lane id: the row compares stay in the sweep
    AW_PROF_ADD(s, PR_NOSLIP_IT, 1);
    if (lane == 0) s.it_noslip = it + 1;
    const float lo = -lim - fa, hi = lim + fb;
    float ysv = 0.f;   // this lane's unclamped update at its own step (its bounds hold all sweep)
    auto step = [&](float a_c, int c) {
      const float y = fmaf(-R, ca, cb);
      const float d = rlane(__builtin_amdgcn_fmed3f(y, lo, hi), c);
      ysv = lane == c ? y : ysv;
      R = fmaf(a_c, d, R);
    };
#pragma unroll
    for (int c = 0; c < NV; c++) step(Am[c], c);
#pragma unroll
    for (int p = 0; p < NPL; p++)
      if (p < npl) step(Ap[p], NV + p);
    const float d = __builtin_amdgcn_fmed3f(ysv, lo, hi);
    float imp = diag * d * (0.5f * d - ysv);
    fa += d;
    fb -= d;
    // pairs past the lanes: their column of A rebuilt, the residual by a wave reduction
#pragma unroll
    for (int xc = 0; xc < NXCH; xc++) {
      const int nx = npr - NPL - 64 * xc;
      for (int x = 0; x < (nx < 64 ? nx : 64); x++) {
        const int e = rlane_i(ex_e[xc], x);
        float jd, col;
        pair_col(e, jd, col);
        const float y = fmaf(-wave_sum(jd * R), rlane(ex_ca[xc], x), rlane(ex_cb[xc], x));
        const float d1 = __builtin_amdgcn_fmed3f(y, -rlane(ex_fa[xc], x), rlane(ex_fb[xc], x));
        R = fmaf(col, d1, R);
        if (lane == x) {
          imp += ex_K[xc] * d1 * (0.5f * d1 - y);
          ex_fa[xc] += d1;
          ex_fb[xc] -= d1;
        }
      }
    }
    if (-wave_sum(imp) * scale < m.noslip_tolerance) break;
  }
  AW_PROF(s, PR_NS_ITER);
  qacc = lane < NV ? R : 0.f;
  if (has_fl) s.efc_force[flrow] = fa;
  if (lane >= NV && lane < NV + npl) {
    s.efc_force[nsparse + rowe] = fa;
    s.efc_force[nsparse + rowe + 1] = fb;
  }
#pragma unroll
  for (int xc = 0; xc < NXCH; xc++)
    if (lane + 64 * xc < npr - NPL) {
      s.efc_force[nsparse + ex_e[xc]] = ex_fa[xc];
      s.efc_force[nsparse + ex_e[xc] + 1] = ex_fb[xc];
    }
  wsync();
}

// ---------------------------------------------------------------------------------------
// mju_rayGeom for site shapes: distance to the first crossing at t >= 0, or -1
AW_DEV float ray_geom(const float* pos, const float* mat, const float* size, const float* pnt,
                          const float* vec, int type) {
  float dif[3], lp[3], lv[3];
  sub3(dif, pnt, pos);
  mulmtv3(lp, mat, dif);
  mulmtv3(lv, mat, vec);
  float best = -1.f;
  auto consider = [&](float t) { if (t >= 0 && (best < 0 || t < best)) best = t; };
  auto sphere = [&](float cz, float r) {
    float o[3] = {lp[0], lp[1], lp[2] - cz};
    float a = dot3(lv, lv), b = dot3(o, lv), cc = dot3(o, o) - r * r;
    float disc = b * b - a * cc;
    if (disc < 0 || a < MINVAL) return;
    float sq = sqrtf(disc);
    consider((-b - sq) / a);
    consider((-b + sq) / a);
  };
  if (type == GEOM_SPHERE) sphere(0.f, size[0]);
  else if (type == GEOM_BOX) {
    for (int k = 0; k < 3; k++) {
      if (fabsf(lv[k]) < MINVAL) continue;
      for (int sd = -1; sd <= 1; sd += 2) {
        float t = (sd * size[k] - lp[k]) / lv[k];
        int u = (k + 1) % 3, v = (k + 2) % 3;
        if (fabsf(lp[u] + t * lv[u]) <= size[u] && fabsf(lp[v] + t * lv[v]) <= size[v]) consider(t);
      }
    }
  } else if (type == GEOM_CYLINDER || type == GEOM_CAPSULE) {
    float r = size[0], h = size[1];
    float a = lv[0] * lv[0] + lv[1] * lv[1];
    float b = lp[0] * lv[0] + lp[1] * lv[1];
    float cc = lp[0] * lp[0] + lp[1] * lp[1] - r * r;
    float disc = b * b - a * cc;
    if (a > MINVAL && disc >= 0) {
      float sq = sqrtf(disc);
      for (int sd = -1; sd <= 1; sd += 2) {
        float t = (-b + sd * sq) / a;
        if (fabsf(lp[2] + t * lv[2]) <= h) consider(t);
      }
    }
    if (type == GEOM_CYLINDER) {
      if (fabsf(lv[2]) > MINVAL)
        for (int sd = -1; sd <= 1; sd += 2) {
          float t = (sd * h - lp[2]) / lv[2];
          float px = lp[0] + t * lv[0], py = lp[1] + t * lv[1];
          if (px * px + py * py <= r * r) consider(t);
        }
    } else {
      sphere(h, r);
      sphere(-h, r);
    }
  }
  return best;
}

// touch sensors of the task (mj_sensorAcc, mjSENS_TOUCH)
AW_DEV void stage_touch(const DModel& m, Env& s, int lane) {
  for (int t = 0; t < m.ntouch; t++) {
    int site = MD(touch_site, t), bid = MD(site_bodyid, site);
    float val = 0.f;
#pragma unroll
    for (int h = 0; h < NCH; h++) {
      const int c = lane + 64 * h;
      if (c < s.ncon && s.con_efc[c] >= 0 && !(m.disableflags & DSBL_SENSOR)) {
        int pr = s.con_pair[c];
        int b1 = MD(geom_bodyid, MD(cp_g1, pr)), b2 = MD(geom_bodyid, MD(cp_g2, pr));
        if (bid == b1 || bid == b2) {
          int adr = s.con_efc[c], dim = MD(cp_condim, pr);
          float fn = 0.f;
          if (dim == 1) fn = s.efc_force[adr];
          else for (int j = 0; j < 2 * (dim - 1); j++) fn += s.efc_force[adr + j];
          if (fn > 0.f) {
            float ray[3];
            copy3(ray, s.con_nrm[c]);
            normalize3(ray);
            if (bid == b2) scl3(ray, ray, -1.f);
            float tsz[3] = {MD(touch_size, 3 * t), MD(touch_size, 3 * t + 1), MD(touch_size, 3 * t + 2)};
            if (ray_geom(s.sxpos[site], s.txmat[t], tsz, s.con_pos[c], ray, MD(touch_type, t)) >= 0.f)
              val += fn;
          }
        }
      }
    }
    float tot = wave_sum(val);
    if (lane == 0) s.touch[t] = tot;
  }
  wsync();
}

}  // namespace aw
