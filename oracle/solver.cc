/* solver.cc -- fp64 restatement of MuJoCo 2.1 constraint assembly and the Newton solver.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Physics parity with real MuJoCo is unpinned.
 *
 * mj_makeConstraint order: dof frictionloss, tendon frictionloss, joint limits (lower then
 * upper side), tendon limits, contacts (frictionless: 1 row; pyramidal: 2(dim-1) edges
 * J_n +- mu_k J_k).  Impedance (getimpedance), regularisation R = (1-imp)/imp * diagApprox
 * (mj_diagApprox from body/dof/tendon invweight0), reference aref = -B v - K imp (pos-margin)
 * with timeconst >= 2*timestep (refsafe).
 *
 * mj_solNewton restated: primal soft-constraint cost
 *     f(a) = 1/2 (a - a0)' M (a - a0) + sum_i s_i(J_i a - aref_i)
 * (s_i quadratic one-sided for limits/contacts, Huber for frictionloss), start from the
 * better of qacc_warmstart / qacc_smooth, Newton direction from a dense Cholesky of
 * H = M + J' D_active J, exact (safeguarded-Newton) line search, stop when the scaled
 * improvement or gradient falls below opt.tolerance or after opt.iterations.
 * Then mj_solNoSlip restated: PGS over frictionloss rows (box-clamped) and over each pair of
 * opposing pyramid edges (normal sum held), without regularisation.
 */
#include <cmath>
#include <cstring>

#include "oracle.h"

namespace orc {

static const num MINVAL = 1e-15;

static void getimpedance(const num* solimp, num pos, num margin, num* imp) {
  num d0 = solimp[0], dmax = solimp[1];
  d0 = d0 < 0.0001 ? 0.0001 : (d0 > 0.9999 ? 0.9999 : d0);
  dmax = dmax < 0.0001 ? 0.0001 : (dmax > 0.9999 ? 0.9999 : dmax);
  if (d0 == dmax || solimp[2] <= MINVAL) { *imp = 0.5 * (d0 + dmax); return; }
  num x = (pos - margin) / solimp[2];
  if (x < 0) x = -x;
  if (x >= 1 || x <= 0) { *imp = x >= 1 ? dmax : d0; return; }
  num y, mid = solimp[3], p = solimp[4];
  if (p == 1) y = x;
  else if (x <= mid) y = std::pow(x, p) / std::pow(mid, p - 1);
  else y = 1 - std::pow(1 - x, p) / std::pow(1 - mid, p - 1);
  *imp = d0 + y * (dmax - d0);
}

/* mj_jac at a point of body b: jacp (3 x nv) and jacr (3 x nv), row-major */
static void jac_point(const Model* m, const Data* d, int body, const num* point, num* jacp, num* jacr) {
  int nv = m->nv;
  memset(jacp, 0, sizeof(num) * 3 * nv);
  memset(jacr, 0, sizeof(num) * 3 * nv);
  num off[3];
  sub3(off, point, &d->subtree_com[3 * m->body_rootid[body]]);
  while (body && !m->body_dofnum[body]) body = m->body_parentid[body];
  if (!body) return;
  int da = m->body_dofadr[body] + m->body_dofnum[body] - 1;
  while (da >= 0) {
    const num* cd = &d->cdof[6 * da];
    num t[3];
    cross3(t, cd, off);
    for (int k = 0; k < 3; k++) {
      jacr[k * nv + da] = cd[k];
      jacp[k * nv + da] = cd[3 + k] + t[k];
    }
    da = m->dof_parentid[da];
  }
}

static int add_row(const Model* m, Data* d, int type, int id, num pos, num margin, num floss,
                   num diagApprox) {
  if (d->nefc >= m->max_efc) { d->status |= ST_EFC_OVERFLOW; return -1; }
  int i = d->nefc++;
  d->efc_type[i] = type; d->efc_id[i] = id;
  d->efc_pos[i] = pos; d->efc_margin[i] = margin; d->efc_frictionloss[i] = floss;
  d->efc_diagApprox[i] = diagApprox;
  memset(&d->efc_J[(size_t)i * m->nv], 0, sizeof(num) * m->nv);
  return i;
}

void make_constraint(const Model* m, Data* d) {
  int nv = m->nv;
  d->nefc = 0;
  if (m->disableflags & DSBL_CONSTRAINT) return;
  /* frictionloss */
  if (!(m->disableflags & DSBL_FRICTIONLOSS)) {
    for (int j = 0; j < nv; j++) {
      if (m->dof_frictionloss[j] <= 0) continue;
      int i = add_row(m, d, CNSTR_FRICTION_DOF, j, 0, 0, m->dof_frictionloss[j], m->dof_invweight0[j]);
      if (i < 0) return;
      d->efc_J[(size_t)i * nv + j] = 1;
    }
    for (int t = 0; t < m->ntendon; t++) {
      if (m->tendon_frictionloss[t] <= 0) continue;
      int i = add_row(m, d, CNSTR_FRICTION_TENDON, t, 0, 0, m->tendon_frictionloss[t], m->tendon_invweight0[t]);
      if (i < 0) return;
      memcpy(&d->efc_J[(size_t)i * nv], &d->ten_J[(size_t)t * nv], sizeof(num) * nv);
    }
  }
  /* limits */
  if (!(m->disableflags & DSBL_LIMIT)) {
    for (int j = 0; j < m->njnt; j++) {
      if (!m->jnt_limited[j]) continue;
      num q = d->qpos[m->jnt_qposadr[j]];
      for (int side = -1; side <= 1; side += 2) {
        num dist = side * (m->jnt_range[2 * j + (side + 1) / 2] - q);
        if (dist < m->jnt_margin[j]) {
          int da = m->jnt_dofadr[j];
          int i = add_row(m, d, CNSTR_LIMIT_JOINT, j, dist, m->jnt_margin[j], 0, m->dof_invweight0[da]);
          if (i < 0) return;
          d->efc_J[(size_t)i * nv + da] = -side;
        }
      }
    }
    for (int t = 0; t < m->ntendon; t++) {
      if (!m->tendon_limited[t]) continue;
      num len = d->ten_length[t];
      for (int side = -1; side <= 1; side += 2) {
        num dist = side * (m->tendon_range[2 * t + (side + 1) / 2] - len);
        if (dist < m->tendon_margin[t]) {
          int i = add_row(m, d, CNSTR_LIMIT_TENDON, t, dist, m->tendon_margin[t], 0, m->tendon_invweight0[t]);
          if (i < 0) return;
          for (int k = 0; k < nv; k++) d->efc_J[(size_t)i * nv + k] = -side * d->ten_J[(size_t)t * nv + k];
        }
      }
    }
  }
  /* contacts */
  std::vector<num> j1p(3 * nv), j1r(3 * nv), j2p(3 * nv), j2r(3 * nv), jc(6 * nv);
  for (int c = 0; c < d->ncon; c++) {
    Contact* con = &d->contact[c];
    int b1 = m->geom_bodyid[con->geom1], b2 = m->geom_bodyid[con->geom2];
    jac_point(m, d, b1, con->pos, j1p.data(), j1r.data());
    jac_point(m, d, b2, con->pos, j2p.data(), j2r.data());
    /* project the Jacobian difference on the contact frame: rows 0-2 translational (normal,
     * tangent1, tangent2), rows 3-5 rotational (normal, tangent1, tangent2) */
    for (int r = 0; r < 3; r++)
      for (int k = 0; k < nv; k++) {
        num sp = 0, sr = 0;
        for (int q = 0; q < 3; q++) {
          sp += con->frame[3 * r + q] * (j2p[q * nv + k] - j1p[q * nv + k]);
          sr += con->frame[3 * r + q] * (j2r[q * nv + k] - j1r[q * nv + k]);
        }
        jc[r * nv + k] = sp;
        jc[(3 + r) * nv + k] = sr;
      }
    num tran = m->body_invweight0[2 * b1] + m->body_invweight0[2 * b2];
    num rot = m->body_invweight0[2 * b1 + 1] + m->body_invweight0[2 * b2 + 1];
    int dim = con->dim;
    if (dim == 1) {
      int i = add_row(m, d, CNSTR_CONTACT_FRICTIONLESS, c, con->dist, con->includemargin, 0, tran);
      if (i < 0) return;
      con->efc_address = i;
      memcpy(&d->efc_J[(size_t)i * nv], &jc[0], sizeof(num) * nv);
    } else {
      if (d->nefc + 2 * (dim - 1) > m->max_efc) { d->status |= ST_EFC_OVERFLOW; return; }
      con->efc_address = d->nefc;
      for (int k = 1; k < dim; k++) {
        num fri = con->friction[k - 1];
        num dA = tran + fri * fri * (k < 3 ? tran : rot);
        for (int s = 1; s >= -1; s -= 2) {
          int i = add_row(m, d, CNSTR_CONTACT_PYRAMIDAL, c, con->dist, con->includemargin, 0, dA);
          for (int q = 0; q < nv; q++) d->efc_J[(size_t)i * nv + q] = jc[q] + s * fri * jc[k * nv + q];
        }
      }
    }
  }
}

/* mj_makeImpedance + mj_referenceConstraint (needs qvel) */
static void make_impedance(const Model* m, Data* d) {
  int nv = m->nv;
  for (int i = 0; i < d->nefc; i++) {
    const num *solref, *solimp;
    int id = d->efc_id[i];
    switch (d->efc_type[i]) {
      case CNSTR_FRICTION_DOF: solref = &m->dof_solref[2 * id]; solimp = &m->dof_solimp[5 * id]; break;
      case CNSTR_FRICTION_TENDON: solref = &m->tendon_solref[2 * id]; solimp = &m->tendon_solimp[5 * id]; break;
      case CNSTR_LIMIT_JOINT: solref = &m->jnt_solref[2 * id]; solimp = &m->jnt_solimp[5 * id]; break;
      case CNSTR_LIMIT_TENDON: solref = &m->tendon_solref[2 * id]; solimp = &m->tendon_solimp[5 * id]; break;
      default: solref = d->contact[id].solref; solimp = d->contact[id].solimp; break;
    }
    num imp;
    getimpedance(solimp, d->efc_pos[i], d->efc_margin[i], &imp);
    num dmax = solimp[1];
    dmax = dmax < 0.0001 ? 0.0001 : (dmax > 0.9999 ? 0.9999 : dmax);
    num K, B;
    if (solref[0] > 0) {
      num tc = solref[0], dr = solref[1];
      if (!(m->disableflags & DSBL_REFSAFE)) tc = std::fmax(tc, 2 * m->timestep);
      K = 1.0 / (dmax * dmax * tc * tc * dr * dr);
      B = 2.0 / (dmax * tc);
    } else {
      K = -solref[0] / (dmax * dmax);
      B = -solref[1] / dmax;
    }
    num R = (1 - imp) * d->efc_diagApprox[i] / imp;
    d->efc_R[i] = R < MINVAL ? MINVAL : R;
    d->efc_D[i] = 1.0 / d->efc_R[i];
    num vel = 0;
    const num* J = &d->efc_J[(size_t)i * nv];
    for (int k = 0; k < nv; k++) vel += J[k] * d->qvel[k];
    d->efc_vel[i] = vel;
    d->efc_aref[i] = -B * vel - K * imp * (d->efc_pos[i] - d->efc_margin[i]);
  }
}

/* row cost, force, state at constraint-space residual jar */
static inline num row_eval(const Data* d, int i, num jar, num* force, int* state) {
  num D = d->efc_D[i], R = d->efc_R[i];
  int t = d->efc_type[i];
  if (t == CNSTR_FRICTION_DOF || t == CNSTR_FRICTION_TENDON) {
    num f = d->efc_frictionloss[i];
    if (jar <= -R * f) { *force = f; *state = CSTATE_LINEARNEG; return -f * jar - 0.5 * R * f * f; }
    if (jar >= R * f) { *force = -f; *state = CSTATE_LINEARPOS; return f * jar - 0.5 * R * f * f; }
    *force = -D * jar; *state = CSTATE_QUADRATIC; return 0.5 * D * jar * jar;
  }
  if (jar < 0) { *force = -D * jar; *state = CSTATE_QUADRATIC; return 0.5 * D * jar * jar; }
  *force = 0; *state = CSTATE_SATISFIED; return 0;
}

namespace {
struct NewtonWS {
  std::vector<num> a, Ma, Jaref, grad, p, Mp, Jp, H, tmp, force;
  std::vector<int> state;
};
}

static num eval_point(const Model* m, const Data* d, NewtonWS& w) {
  int nv = m->nv;
  num gauss = 0;
  for (int k = 0; k < nv; k++) gauss += (w.Ma[k] - d->qfrc_smooth[k]) * (w.a[k] - d->qacc_smooth[k]);
  num cost = 0.5 * gauss;
  for (int i = 0; i < d->nefc; i++) cost += row_eval(d, i, w.Jaref[i], &w.force[i], &w.state[i]);
  return cost;
}

static void set_point(const Model* m, const Data* d, NewtonWS& w, const num* a) {
  int nv = m->nv;
  for (int k = 0; k < nv; k++) w.a[k] = a[k];
  mul_M(m, d, w.a.data(), w.Ma.data());
  for (int i = 0; i < d->nefc; i++) {
    const num* J = &d->efc_J[(size_t)i * nv];
    num s = 0;
    for (int k = 0; k < nv; k++) s += J[k] * w.a[k];
    w.Jaref[i] = s - d->efc_aref[i];
  }
}

/* dense Cholesky H = L L' in place (lower); returns 0 on success */
static int cholesky(num* H, int n) {
  for (int j = 0; j < n; j++) {
    num s = H[j * n + j];
    for (int k = 0; k < j; k++) s -= H[j * n + k] * H[j * n + k];
    if (s < MINVAL) s = MINVAL;
    num l = std::sqrt(s);
    H[j * n + j] = l;
    for (int i = j + 1; i < n; i++) {
      num t = H[i * n + j];
      for (int k = 0; k < j; k++) t -= H[i * n + k] * H[j * n + k];
      H[i * n + j] = t / l;
    }
  }
  return 0;
}
static void chol_solve(const num* L, int n, num* x) {
  for (int i = 0; i < n; i++) {
    num s = x[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * x[k];
    x[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    num s = x[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * x[k];
    x[i] = s / L[i * n + i];
  }
}

/* derivative of the 1-D cost along p at step alpha */
static void ls_deriv(const Data* d, const NewtonWS& w, num c0, num c1, num alpha, num* d1, num* d2) {
  num g1 = c0 + alpha * c1, g2 = c1;
  for (int i = 0; i < d->nefc; i++) {
    num jp = w.Jp[i];
    if (jp == 0) continue;
    num f;
    int st;
    row_eval(d, i, w.Jaref[i] + alpha * jp, &f, &st);
    g1 -= f * jp;
    if (st == CSTATE_QUADRATIC) g2 += d->efc_D[i] * jp * jp;
  }
  *d1 = g1;
  *d2 = g2;
}

static num line_search(const Model* m, Data* d, NewtonWS& w) {
  int nv = m->nv;
  mul_M(m, d, w.p.data(), w.Mp.data());
  num c0 = 0, c1 = 0;
  for (int k = 0; k < nv; k++) { c0 += w.p[k] * (w.Ma[k] - d->qfrc_smooth[k]); c1 += w.p[k] * w.Mp[k]; }
  for (int i = 0; i < d->nefc; i++) {
    const num* J = &d->efc_J[(size_t)i * nv];
    num s = 0;
    for (int k = 0; k < nv; k++) s += J[k] * w.p[k];
    w.Jp[i] = s;
  }
  num d1, d2;
  ls_deriv(d, w, c0, c1, 0, &d1, &d2);
  d->ls_iter++;
  if (d1 >= 0) return 0;
  num tol = 1e-10 * std::fabs(d1);
  num alpha = 0, lo = 0, hi = -1;
  for (int it = 0; it < 50; it++) {
    num an = alpha - d1 / d2;
    if (hi >= 0 && (an <= lo || an >= hi)) an = 0.5 * (lo + hi);
    if (an == alpha) break;
    alpha = an;
    ls_deriv(d, w, c0, c1, alpha, &d1, &d2);
    d->ls_iter++;
    if (d1 < 0) lo = alpha; else hi = alpha;
    if (std::fabs(d1) <= tol) break;
  }
  return alpha;
}

static void noslip(const Model* m, Data* d);

void contact_force(const Model* m, const Data* d, int c, num* r) {
  (void)m;
  const Contact* con = &d->contact[c];
  for (int k = 0; k < 6; k++) r[k] = 0;
  int adr = con->efc_address;
  if (adr < 0) return;
  if (con->dim == 1) { r[0] = d->efc_force[adr]; return; }
  for (int j = 0; j < 2 * (con->dim - 1); j++) r[0] += d->efc_force[adr + j];
  for (int k = 1; k < con->dim; k++)
    r[k] = (d->efc_force[adr + 2 * k - 2] - d->efc_force[adr + 2 * k - 1]) * con->friction[k - 1];
}

void fwd_constraint(const Model* m, Data* d) {
  int nv = m->nv, nefc = d->nefc;
  d->solver_iter = d->noslip_iter = d->ls_iter = 0;
  if (!nefc) {
    d->qacc = d->qacc_smooth;
    std::fill(d->qfrc_constraint.begin(), d->qfrc_constraint.end(), 0.0);
    return;
  }
  make_impedance(m, d);
  NewtonWS w;
  w.a.resize(nv); w.Ma.resize(nv); w.grad.resize(nv); w.p.resize(nv); w.Mp.resize(nv);
  w.tmp.resize(nv); w.H.resize((size_t)nv * nv);
  w.Jaref.resize(nefc); w.Jp.resize(nefc); w.force.resize(nefc); w.state.resize(nefc);
  num scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));

  /* initial point: better of warmstart and qacc_smooth */
  set_point(m, d, w, d->qacc_smooth.data());
  num cost = eval_point(m, d, w);
  if (!(m->disableflags & DSBL_WARMSTART)) {
    std::vector<num> a0 = w.a, Ma0 = w.Ma, J0 = w.Jaref;
    set_point(m, d, w, d->qacc_warmstart.data());
    num cw = eval_point(m, d, w);
    if (cw < cost) cost = cw;
    else { w.a = a0; w.Ma = Ma0; w.Jaref = J0; cost = eval_point(m, d, w); }
  }
  auto gradient = [&]() {
    for (int k = 0; k < nv; k++) w.grad[k] = w.Ma[k] - d->qfrc_smooth[k];
    for (int i = 0; i < nefc; i++) {
      if (w.force[i] == 0) continue;
      const num* J = &d->efc_J[(size_t)i * nv];
      for (int k = 0; k < nv; k++) w.grad[k] -= J[k] * w.force[i];
    }
  };
  gradient();
  for (int iter = 0; iter < m->iterations; iter++) {
    /* Hessian and Newton direction */
    for (size_t k = 0; k < (size_t)nv * nv; k++) w.H[k] = d->qM[k];
    for (int i = 0; i < nefc; i++) {
      if (w.state[i] != CSTATE_QUADRATIC) continue;
      const num* J = &d->efc_J[(size_t)i * nv];
      num D = d->efc_D[i];
      for (int r = 0; r < nv; r++) {
        if (J[r] == 0) continue;
        num jr = D * J[r];
        for (int c = 0; c <= r; c++) w.H[r * nv + c] += jr * J[c];
      }
    }
    cholesky(w.H.data(), nv);
    for (int k = 0; k < nv; k++) w.p[k] = -w.grad[k];
    chol_solve(w.H.data(), nv, w.p.data());
    num alpha = line_search(m, d, w);
    d->solver_iter = iter + 1;
    if (alpha == 0) break;
    for (int k = 0; k < nv; k++) { w.a[k] += alpha * w.p[k]; w.Ma[k] += alpha * w.Mp[k]; }
    for (int i = 0; i < nefc; i++) w.Jaref[i] += alpha * w.Jp[i];
    num oldcost = cost;
    cost = eval_point(m, d, w);
    gradient();
    num gn = 0;
    for (int k = 0; k < nv; k++) gn += w.grad[k] * w.grad[k];
    num improvement = scale * (oldcost - cost), gradnorm = scale * std::sqrt(gn);
    if (improvement < m->tolerance || gradnorm < m->tolerance) break;
  }
  for (int i = 0; i < nefc; i++) { d->efc_force[i] = w.force[i]; d->efc_state[i] = w.state[i]; }
  d->qacc = w.a;
  for (int k = 0; k < nv; k++) d->qfrc_constraint[k] = 0;
  for (int i = 0; i < nefc; i++) {
    const num* J = &d->efc_J[(size_t)i * nv];
    for (int k = 0; k < nv; k++) d->qfrc_constraint[k] += J[k] * d->efc_force[i];
  }
  if (m->noslip_iterations > 0 && !(m->disableflags & DSBL_NOSLIP)) noslip(m, d);
}

static void noslip(const Model* m, Data* d) {
  int nv = m->nv, nefc = d->nefc;
  std::vector<int> F;
  for (int i = 0; i < nefc; i++) {
    int t = d->efc_type[i];
    if (t == CNSTR_FRICTION_DOF || t == CNSTR_FRICTION_TENDON || t == CNSTR_CONTACT_PYRAMIDAL) F.push_back(i);
  }
  int nf = (int)F.size();
  if (!nf) return;
  /* A_FF = J_F M^-1 J_F' ; r_F = J_F qacc - aref_F */
  std::vector<num> MinvJ((size_t)nf * nv), A((size_t)nf * nf), r(nf);
  std::vector<int> pos_in_F(nefc, -1);
  for (int a = 0; a < nf; a++) {
    pos_in_F[F[a]] = a;
    num* x = &MinvJ[(size_t)a * nv];
    memcpy(x, &d->efc_J[(size_t)F[a] * nv], sizeof(num) * nv);
    solve_ld(m, d->qLD.data(), d->qLDiagInv.data(), x);
  }
  for (int a = 0; a < nf; a++) {
    const num* Ja = &d->efc_J[(size_t)F[a] * nv];
    for (int b = 0; b < nf; b++) {
      const num* x = &MinvJ[(size_t)b * nv];
      num s = 0;
      for (int k = 0; k < nv; k++) s += Ja[k] * x[k];
      A[(size_t)a * nf + b] = s;
    }
    num s = 0;
    for (int k = 0; k < nv; k++) s += Ja[k] * d->qacc[k];
    r[a] = s - d->efc_aref[F[a]];
  }
  num scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
  auto upd = [&](int a, num delta) {
    for (int b = 0; b < nf; b++) r[b] += A[(size_t)b * nf + a] * delta;
    d->efc_force[F[a]] += delta;
  };
  for (int it = 0; it < m->noslip_iterations; it++) {
    num improvement = 0;
    /* dry friction rows */
    for (int a = 0; a < nf; a++) {
      int i = F[a], t = d->efc_type[i];
      if (t != CNSTR_FRICTION_DOF && t != CNSTR_FRICTION_TENDON) continue;
      num Aii = A[(size_t)a * nf + a];
      if (Aii < MINVAL) continue;
      num f = d->efc_force[i], fl = d->efc_frictionloss[i];
      num x = f - r[a] / Aii;
      x = x < -fl ? -fl : (x > fl ? fl : x);
      num delta = x - f;
      if (delta == 0) continue;
      improvement -= r[a] * delta + 0.5 * Aii * delta * delta;
      upd(a, delta);
    }
    /* pyramidal contacts: opposing edge pairs */
    for (int c = 0; c < d->ncon; c++) {
      const Contact* con = &d->contact[c];
      if (con->dim == 1 || con->efc_address < 0) continue;
      for (int k = 0; k < con->dim - 1; k++) {
        int i1 = con->efc_address + 2 * k, i2 = i1 + 1;
        int a1 = pos_in_F[i1], a2 = pos_in_F[i2];
        num A11 = A[(size_t)a1 * nf + a1], A22 = A[(size_t)a2 * nf + a2], A12 = A[(size_t)a1 * nf + a2];
        num K = A11 + A22 - 2 * A12;
        if (K < MINVAL) continue;
        num f1 = d->efc_force[i1], f2 = d->efc_force[i2];
        num s = f1 + f2, x = f1 - f2;
        num xn = x - 2 * (r[a1] - r[a2]) / K;
        xn = xn < -s ? -s : (xn > s ? s : xn);
        num d1 = 0.5 * (s + xn) - f1, d2 = 0.5 * (s - xn) - f2;
        if (d1 == 0 && d2 == 0) continue;
        improvement -= r[a1] * d1 + r[a2] * d2 + 0.5 * (A11 * d1 * d1 + 2 * A12 * d1 * d2 + A22 * d2 * d2);
        upd(a1, d1);
        upd(a2, d2);
      }
    }
    d->noslip_iter = it + 1;
    if (improvement * scale < m->noslip_tolerance) break;
  }
  for (int k = 0; k < nv; k++) d->qfrc_constraint[k] = 0;
  for (int i = 0; i < nefc; i++) {
    const num* J = &d->efc_J[(size_t)i * nv];
    for (int k = 0; k < nv; k++) d->qfrc_constraint[k] += J[k] * d->efc_force[i];
  }
  for (int k = 0; k < nv; k++) d->qacc[k] = d->qfrc_constraint[k];
  solve_ld(m, d->qLD.data(), d->qLDiagInv.data(), d->qacc.data());
  for (int k = 0; k < nv; k++) d->qacc[k] += d->qacc_smooth[k];
}

}  // namespace orc
