/* mjstep.cc -- fp64 restatement of MuJoCo 2.1 mj_step (Euler) for the Adroit models.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Physics parity with real MuJoCo is unpinned.
 *
 * Stage order follows mj_forward: fwdPosition (kinematics, comPos, tendon, crb, factorM,
 * collision, makeConstraint, transmission) -> fwdVelocity (comVel, passive, rne) ->
 * fwdActuation -> fwdAcceleration -> fwdConstraint -> sensors; then mj_Euler with implicit
 * joint damping.  Called by the reference through mjrl do_simulation
 * (hand_manipulation_suite/hammer_v0.py:60) -> mujoco-py MjSim.step.
 */
#include <cmath>
#include <cstring>

#include "oracle.h"

namespace orc {

static const num MINVAL = 1e-15;
static const num MAXVAL = 1e10;

num norm3(const num* a) { return std::sqrt(dot3(a, a)); }
num normalize3(num* a) {
  num n = norm3(a);
  if (n < MINVAL) { a[0] = 1; a[1] = 0; a[2] = 0; return n; }
  a[0] /= n; a[1] /= n; a[2] /= n;
  return n;
}
void mul_mat_vec3(num* r, const num* m, const num* v) {
  num t0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  num t1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  num t2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
void mul_matT_vec3(num* r, const num* m, const num* v) {
  num t0 = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  num t1 = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  num t2 = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
void mul_quat(num* r, const num* a, const num* b) {
  num t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  num t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  num t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  num t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
void rot_vec_quat(num* r, const num* v, const num* q) {
  /* r = v + 2 w (u x v) + 2 u x (u x v),  u = q[1:4] */
  num u[3] = {q[1], q[2], q[3]}, t[3], t2[3];
  cross3(t, u, v);
  scl3(t, t, 2.0);
  cross3(t2, u, t);
  r[0] = v[0] + q[0] * t[0] + t2[0];
  r[1] = v[1] + q[0] * t[1] + t2[1];
  r[2] = v[2] + q[0] * t[2] + t2[2];
}
void quat2mat(num* m, const num* q) {
  num w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = 1 - 2 * (x * x + y * y);
}
void axis_angle2quat(num* q, const num* axis, num angle) {
  num s = std::sin(angle * 0.5);
  q[0] = std::cos(angle * 0.5); q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}
void normalize4(num* q) {
  num n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  for (int i = 0; i < 4; i++) q[i] /= n;
}
void mul_mat_mat3(num* r, const num* a, const num* b) {
  num t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      t[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
  memcpy(r, t, sizeof(t));
}

/* mju_makeFrame: complete an orthonormal frame from its first row (the contact normal). */
void make_frame(num* f) {
  normalize3(f);
  if (norm3(f + 3) < 0.5) {
    if (std::fabs(f[1]) < 0.5) { f[3] = 0; f[4] = 1; f[5] = 0; }
    else { f[3] = 0; f[4] = 0; f[5] = 1; }
  }
  num d = dot3(f, f + 3);
  f[3] -= d * f[0]; f[4] -= d * f[1]; f[5] -= d * f[2];
  normalize3(f + 3);
  cross3(f + 6, f, f + 3);
}

/* ------------------------------------------------------------------------------------- */
/* spatial algebra (MuJoCo layout: motion = [ang; lin], cinert = [Ixx Iyy Izz Ixy Ixz Iyz mc(3) m]) */
static void mul_inert_vec(num* r, const num* i, const num* v) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
static void cross_motion(num* r, const num* v, const num* u) {
  num t[6];
  t[0] = -v[2] * u[1] + v[1] * u[2];
  t[1] = v[2] * u[0] - v[0] * u[2];
  t[2] = -v[1] * u[0] + v[0] * u[1];
  t[3] = -v[2] * u[4] + v[1] * u[5] - v[5] * u[1] + v[4] * u[2];
  t[4] = v[2] * u[3] - v[0] * u[5] + v[5] * u[0] - v[3] * u[2];
  t[5] = -v[1] * u[3] + v[0] * u[4] - v[4] * u[0] + v[3] * u[1];
  memcpy(r, t, sizeof(t));
}
static void cross_force(num* r, const num* v, const num* f) {
  num t[6];
  t[0] = -v[2] * f[1] + v[1] * f[2] - v[5] * f[4] + v[4] * f[5];
  t[1] = v[2] * f[0] - v[0] * f[2] + v[5] * f[3] - v[3] * f[5];
  t[2] = -v[1] * f[0] + v[0] * f[1] - v[4] * f[3] + v[3] * f[4];
  t[3] = -v[2] * f[4] + v[1] * f[5];
  t[4] = v[2] * f[3] - v[0] * f[5];
  t[5] = -v[1] * f[3] + v[0] * f[4];
  memcpy(r, t, sizeof(t));
}
static num dot6(const num* a, const num* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

/* ------------------------------------------------------------------------------------- */
/* mj_kinematics */
void kinematics(const Model* m, Data* d) {
  d->xpos[0] = d->xpos[1] = d->xpos[2] = 0;
  d->xquat[0] = 1; d->xquat[1] = d->xquat[2] = d->xquat[3] = 0;
  quat2mat(&d->xmat[0], &d->xquat[0]);
  for (int i = 1; i < m->nbody; i++) {
    int p = m->body_parentid[i];
    num xpos[3], xquat[4];
    mul_mat_vec3(xpos, &d->xmat[9 * p], &d->body_pos[3 * i]);
    add3(xpos, xpos, &d->xpos[3 * p]);
    mul_quat(xquat, &d->xquat[4 * p], &d->body_quat[4 * i]);
    for (int k = 0; k < m->body_jntnum[i]; k++) {
      int j = m->body_jntadr[i] + k, qa = m->jnt_qposadr[j];
      num xaxis[3], xanchor[3];
      rot_vec_quat(xaxis, &m->jnt_axis[3 * j], xquat);
      rot_vec_quat(xanchor, &m->jnt_pos[3 * j], xquat);
      add3(xanchor, xanchor, xpos);
      num q = d->qpos[qa] - m->qpos0[qa];
      if (m->jnt_type[j] == JNT_SLIDE) {
        xpos[0] += xaxis[0] * q; xpos[1] += xaxis[1] * q; xpos[2] += xaxis[2] * q;
      } else {
        num qloc[4], v[3];
        axis_angle2quat(qloc, &m->jnt_axis[3 * j], q);
        mul_quat(xquat, xquat, qloc);
        rot_vec_quat(v, &m->jnt_pos[3 * j], xquat);
        sub3(xpos, xanchor, v);
      }
      copy3(&d->xanchor[3 * j], xanchor);
      copy3(&d->xaxis[3 * j], xaxis);
    }
    normalize4(xquat);
    memcpy(&d->xquat[4 * i], xquat, sizeof(xquat));
    copy3(&d->xpos[3 * i], xpos);
    quat2mat(&d->xmat[9 * i], xquat);
  }
  /* mj_local2Global for inertial frames, geoms, sites */
  for (int i = 0; i < m->nbody; i++) {
    num q[4];
    mul_mat_vec3(&d->xipos[3 * i], &d->xmat[9 * i], &m->body_ipos[3 * i]);
    add3(&d->xipos[3 * i], &d->xipos[3 * i], &d->xpos[3 * i]);
    mul_quat(q, &d->xquat[4 * i], &m->body_iquat[4 * i]);
    quat2mat(&d->ximat[9 * i], q);
  }
  for (int g = 0; g < m->ngeom; g++) {
    int b = m->geom_bodyid[g];
    num q[4];
    mul_mat_vec3(&d->geom_xpos[3 * g], &d->xmat[9 * b], &d->geom_pos[3 * g]);
    add3(&d->geom_xpos[3 * g], &d->geom_xpos[3 * g], &d->xpos[3 * b]);
    mul_quat(q, &d->xquat[4 * b], &m->geom_quat[4 * g]);
    quat2mat(&d->geom_xmat[9 * g], q);
  }
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_bodyid[s];
    num q[4];
    mul_mat_vec3(&d->site_xpos[3 * s], &d->xmat[9 * b], &d->site_pos[3 * s]);
    add3(&d->site_xpos[3 * s], &d->site_xpos[3 * s], &d->xpos[3 * b]);
    mul_quat(q, &d->xquat[4 * b], &m->site_quat[4 * s]);
    quat2mat(&d->site_xmat[9 * s], q);
  }
}

/* mj_comPos: subtree com (divided by the compile-time subtree mass), cinert, cdof */
void com_pos(const Model* m, Data* d) {
  int nb = m->nbody;
  for (int i = 0; i < nb; i++) scl3(&d->subtree_com[3 * i], &d->xipos[3 * i], d->body_mass[i]);
  for (int i = nb - 1; i > 0; i--)
    add3(&d->subtree_com[3 * m->body_parentid[i]], &d->subtree_com[3 * m->body_parentid[i]],
         &d->subtree_com[3 * i]);
  for (int i = 0; i < nb; i++) {
    if (m->body_subtreemass[i] < MINVAL) copy3(&d->subtree_com[3 * i], &d->xipos[3 * i]);
    else scl3(&d->subtree_com[3 * i], &d->subtree_com[3 * i], 1.0 / m->body_subtreemass[i]);
  }
  for (int i = 0; i < 10; i++) d->cinert[i] = 0;
  for (int i = 1; i < nb; i++) {
    const num* R = &d->ximat[9 * i];
    const num* I = &m->body_inertia[3 * i];
    num mass = d->body_mass[i], dif[3], *c = &d->cinert[10 * i];
    sub3(dif, &d->xipos[3 * i], &d->subtree_com[3 * m->body_rootid[i]]);
    /* R diag(I) R' */
    num T[9];
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++)
        T[3 * a + b] = R[3 * a] * I[0] * R[3 * b] + R[3 * a + 1] * I[1] * R[3 * b + 1] +
                       R[3 * a + 2] * I[2] * R[3 * b + 2];
    c[0] = T[0] + mass * (dif[1] * dif[1] + dif[2] * dif[2]);
    c[1] = T[4] + mass * (dif[0] * dif[0] + dif[2] * dif[2]);
    c[2] = T[8] + mass * (dif[0] * dif[0] + dif[1] * dif[1]);
    c[3] = T[1] - mass * dif[0] * dif[1];
    c[4] = T[2] - mass * dif[0] * dif[2];
    c[5] = T[5] - mass * dif[1] * dif[2];
    c[6] = mass * dif[0]; c[7] = mass * dif[1]; c[8] = mass * dif[2];
    c[9] = mass;
  }
  for (int j = 0; j < m->njnt; j++) {
    int b = m->jnt_bodyid[j], da = m->jnt_dofadr[j];
    num* cd = &d->cdof[6 * da];
    const num* axis = &d->xaxis[3 * j];
    if (m->jnt_type[j] == JNT_SLIDE) {
      cd[0] = cd[1] = cd[2] = 0;
      copy3(cd + 3, axis);
    } else {
      num off[3];
      sub3(off, &d->subtree_com[3 * m->body_rootid[b]], &d->xanchor[3 * j]);
      copy3(cd, axis);
      cross3(cd + 3, axis, off);
    }
  }
}

/* mj_tendon: fixed tendons, length = sum coef * q, J = coef */
void tendon(const Model* m, Data* d) {
  int nv = m->nv;
  for (int t = 0; t < m->ntendon; t++) {
    num len = 0;
    num* J = &d->ten_J[(size_t)t * nv];
    for (int k = 0; k < nv; k++) J[k] = 0;
    for (int w = m->tendon_adr[t]; w < m->tendon_adr[t] + m->tendon_num[t]; w++) {
      int j = m->wrap_jnt[w];
      len += m->wrap_coef[w] * d->qpos[m->jnt_qposadr[j]];
      J[m->jnt_dofadr[j]] += m->wrap_coef[w];
    }
    d->ten_length[t] = len;
  }
}

/* mj_crb: composite rigid body inertia -> qM (tree-sparse, stored dense symmetric) */
void crb(const Model* m, Data* d) {
  int nv = m->nv;
  d->crb = d->cinert;
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    if (p > 0)
      for (int k = 0; k < 10; k++) d->crb[10 * p + k] += d->crb[10 * i + k];
  }
  std::fill(d->qM.begin(), d->qM.end(), 0.0);
  for (int i = 0; i < nv; i++) {
    num buf[6];
    mul_inert_vec(buf, &d->crb[10 * m->dof_bodyid[i]], &d->cdof[6 * i]);
    int j = i;
    while (j >= 0) {
      num v = dot6(&d->cdof[6 * j], buf);
      d->qM[(size_t)i * nv + j] += v;
      if (j != i) d->qM[(size_t)j * nv + i] += v;
      j = m->dof_parentid[j];
    }
  }
  for (int i = 0; i < nv; i++) d->qM[(size_t)i * nv + i] += m->dof_armature[i];
}

/* mj_factorI: M = L' D L, L unit lower (tree-sparse, no fill-in), eliminated leaves-first.
 * LD holds L below the diagonal and D on it (dense storage, ancestors only). */
void factor_lower(const Model* m, const num* M, num* LD, num* diaginv) {
  int nv = m->nv;
  for (size_t k = 0; k < (size_t)nv * nv; k++) LD[k] = M[k];
  for (int k = nv - 1; k >= 0; k--) {
    num* rowk = LD + (size_t)k * nv;
    if (rowk[k] < MINVAL) rowk[k] = MINVAL;
    num invD = 1.0 / rowk[k];
    for (int i = m->dof_parentid[k]; i >= 0; i = m->dof_parentid[i]) {
      num t = rowk[i] * invD;
      num* rowi = LD + (size_t)i * nv;
      for (int j = i; j >= 0; j = m->dof_parentid[j]) rowi[j] -= t * rowk[j];
      rowk[i] = t;
    }
  }
  for (int i = 0; i < nv; i++) diaginv[i] = 1.0 / LD[(size_t)i * nv + i];
}

/* mj_solveLD: x <- inv(L' D L) x */
void solve_ld(const Model* m, const num* LD, const num* diaginv, num* x) {
  int nv = m->nv;
  for (int i = nv - 1; i >= 0; i--) {
    num xi = x[i];
    if (xi == 0) continue;
    for (int j = m->dof_parentid[i]; j >= 0; j = m->dof_parentid[j]) x[j] -= LD[(size_t)i * nv + j] * xi;
  }
  for (int i = 0; i < nv; i++) x[i] *= diaginv[i];
  for (int i = 0; i < nv; i++)
    for (int j = m->dof_parentid[i]; j >= 0; j = m->dof_parentid[j]) x[i] -= LD[(size_t)i * nv + j] * x[j];
}

void mul_M(const Model* m, const Data* d, const num* x, num* y) {
  int nv = m->nv;
  for (int i = 0; i < nv; i++) {
    num s = 0;
    for (int j = 0; j < nv; j++) s += d->qM[(size_t)i * nv + j] * x[j];
    y[i] = s;
  }
}

/* mj_comVel */
void com_vel(const Model* m, Data* d) {
  for (int k = 0; k < 6; k++) d->cvel[k] = 0;
  for (int i = 1; i < m->nbody; i++) {
    num cvel[6];
    memcpy(cvel, &d->cvel[6 * m->body_parentid[i]], sizeof(cvel));
    int da = m->body_dofadr[i];
    for (int k = 0; k < m->body_dofnum[i]; k++) {
      int j = da + k;
      cross_motion(&d->cdof_dot[6 * j], cvel, &d->cdof[6 * j]);
      for (int c = 0; c < 6; c++) cvel[c] += d->cdof[6 * j + c] * d->qvel[j];
    }
    memcpy(&d->cvel[6 * i], cvel, sizeof(cvel));
  }
}

/* mj_rne with flg_acc = 0: qfrc_bias = C(q, qdot) qdot + g(q) */
void rne(const Model* m, Data* d) {
  int nb = m->nbody;
  std::vector<num> cacc(6 * nb, 0.0), cfrc(6 * nb, 0.0);
  if (!(m->disableflags & DSBL_GRAVITY)) {
    cacc[3] = -m->gravity[0]; cacc[4] = -m->gravity[1]; cacc[5] = -m->gravity[2];
  }
  for (int i = 1; i < nb; i++) {
    int p = m->body_parentid[i], da = m->body_dofadr[i];
    for (int c = 0; c < 6; c++) cacc[6 * i + c] = cacc[6 * p + c];
    for (int k = 0; k < m->body_dofnum[i]; k++)
      for (int c = 0; c < 6; c++) cacc[6 * i + c] += d->cdof_dot[6 * (da + k) + c] * d->qvel[da + k];
    num t1[6], t2[6];
    mul_inert_vec(&cfrc[6 * i], &d->cinert[10 * i], &cacc[6 * i]);
    mul_inert_vec(t1, &d->cinert[10 * i], &d->cvel[6 * i]);
    cross_force(t2, &d->cvel[6 * i], t1);
    for (int c = 0; c < 6; c++) cfrc[6 * i + c] += t2[c];
  }
  for (int i = nb - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    if (p > 0)
      for (int c = 0; c < 6; c++) cfrc[6 * p + c] += cfrc[6 * i + c];
  }
  for (int j = 0; j < m->nv; j++) d->qfrc_bias[j] = dot6(&d->cdof[6 * j], &cfrc[6 * m->dof_bodyid[j]]);
}

/* mj_passive: joint damping only (the Adroit model has no springs, tendon damping is 0) */
void passive(const Model* m, Data* d) {
  for (int j = 0; j < m->nv; j++)
    d->qfrc_passive[j] = (m->disableflags & DSBL_PASSIVE) ? 0 : -m->dof_damping[j] * d->qvel[j];
}

/* mj_transmission + mj_fwdActuation: general actuator, fixed gain, affine bias, joint trn */
void actuation(const Model* m, Data* d) {
  for (int j = 0; j < m->nv; j++) d->qfrc_actuator[j] = 0;
  for (int i = 0; i < m->nu; i++) {
    int jnt = m->actuator_trnid[i];
    num gear = m->actuator_gear[i];
    d->actuator_length[i] = gear * d->qpos[m->jnt_qposadr[jnt]];
    d->actuator_velocity[i] = gear * d->qvel[m->jnt_dofadr[jnt]];
    if (m->disableflags & DSBL_ACTUATION) { d->actuator_force[i] = 0; continue; }
    num ctrl = d->ctrl[i];
    if (m->actuator_ctrllimited[i] && !(m->disableflags & DSBL_CLAMPCTRL)) {
      num lo = m->actuator_ctrlrange[2 * i], hi = m->actuator_ctrlrange[2 * i + 1];
      ctrl = ctrl < lo ? lo : (ctrl > hi ? hi : ctrl);
    }
    const num* g = &m->actuator_gainprm[3 * i];
    const num* b = &m->actuator_biasprm[3 * i];
    num f = g[0] * ctrl + b[0] + b[1] * d->actuator_length[i] + b[2] * d->actuator_velocity[i];
    if (m->actuator_forcelimited[i]) {
      num lo = m->actuator_forcerange[2 * i], hi = m->actuator_forcerange[2 * i + 1];
      f = f < lo ? lo : (f > hi ? hi : f);
    }
    d->actuator_force[i] = f;
    d->qfrc_actuator[m->jnt_dofadr[jnt]] += gear * f;
  }
}

/* mj_sensor: the three sensor types in the Adroit models (only S_nail feeds an obs) */
void sensors(const Model* m, Data* d) {
  if (m->disableflags & DSBL_SENSOR) return;
  for (int s = 0; s < m->nsensor; s++) {
    int adr = m->sensor_adr[s], obj = m->sensor_objid[s];
    switch (m->sensor_type[s]) {
      case 1: d->sensordata[adr] = d->qpos[m->jnt_qposadr[obj]]; break;
      case 2: d->sensordata[adr] = d->actuator_force[obj]; break;
      case 0: {
        /* touch: sum of normal forces of contacts on the site's body whose normal ray from
         * the contact point intersects the site volume (mj_sensorAcc, mjSENS_TOUCH) */
        int bid = m->site_bodyid[obj];
        num sum = 0;
        for (int c = 0; c < d->ncon; c++) {
          const Contact* con = &d->contact[c];
          int b1 = m->geom_bodyid[con->geom1], b2 = m->geom_bodyid[con->geom2];
          if (con->efc_address < 0 || (bid != b1 && bid != b2)) continue;
          num f6[6];
          contact_force(m, d, c, f6);
          if (f6[0] <= 0) continue;
          num ray[3];
          scl3(ray, con->frame, f6[0]);
          normalize3(ray);
          if (bid == b2) scl3(ray, ray, -1);
          if (ray_geom(&d->site_xpos[3 * obj], &d->site_xmat[9 * obj], &m->site_size[3 * obj],
                       con->pos, ray, m->site_type[obj]) >= 0)
            sum += f6[0];
        }
        d->sensordata[adr] = sum;
        break;
      }
    }
  }
}

/* mj_forward */
void forward(const Model* m, Data* d) {
  kinematics(m, d);
  com_pos(m, d);
  tendon(m, d);
  crb(m, d);
  factor_lower(m, d->qM.data(), d->qLD.data(), d->qLDiagInv.data());
  collision(m, d);
  make_constraint(m, d);
  com_vel(m, d);
  passive(m, d);
  rne(m, d);
  actuation(m, d);
  for (int j = 0; j < m->nv; j++) {
    d->qfrc_smooth[j] = d->qfrc_passive[j] - d->qfrc_bias[j] + d->qfrc_actuator[j];
    d->qacc_smooth[j] = d->qfrc_smooth[j];
  }
  solve_ld(m, d->qLD.data(), d->qLDiagInv.data(), d->qacc_smooth.data());
  fwd_constraint(m, d);
  sensors(m, d);
}

/* mj_Euler: implicit joint damping, semi-implicit position update, warmstart <- qacc */
void euler(const Model* m, Data* d) {
  int nv = m->nv;
  num h = m->timestep;
  bool dmp = false;
  if (!(m->disableflags & DSBL_EULERDAMP) && !(m->disableflags & DSBL_PASSIVE))
    for (int j = 0; j < nv; j++)
      if (m->dof_damping[j] > 0) { dmp = true; break; }
  std::vector<num> acc(nv);
  if (!dmp) {
    acc = d->qacc;
  } else {
    d->qH = d->qM;
    for (int j = 0; j < nv; j++) d->qH[(size_t)j * nv + j] += h * m->dof_damping[j];
    factor_lower(m, d->qH.data(), d->qH.data(), d->qHDiagInv.data());
    for (int j = 0; j < nv; j++) acc[j] = d->qfrc_smooth[j] + d->qfrc_constraint[j];
    solve_ld(m, d->qH.data(), d->qHDiagInv.data(), acc.data());
  }
  for (int j = 0; j < nv; j++) d->qvel[j] += h * acc[j];
  for (int j = 0; j < nv; j++) d->qpos[j] += h * d->qvel[j];   /* hinge/slide only */
  d->time += h;
  d->qacc_warmstart = d->qacc;
}

void reset_data(const Model* m, Data* d) {
  for (int i = 0; i < m->nq; i++) d->qpos[i] = m->qpos0[i];
  std::fill(d->qvel.begin(), d->qvel.end(), 0.0);
  std::fill(d->qacc_warmstart.begin(), d->qacc_warmstart.end(), 0.0);
  std::fill(d->ctrl.begin(), d->ctrl.end(), 0.0);
  d->time = 0;
}

static bool bad(const std::vector<num>& v) {
  for (num x : v)
    if (std::isnan(x) || std::fabs(x) > MAXVAL) return true;
  return false;
}

/* mj_step: checkPos / checkVel / forward / checkAcc / Euler.  MuJoCo resets the data on a
 * bad state (with a warning); the batched env additionally records a status flag. */
void step(const Model* m, Data* d) {
  if (bad(d->qpos)) { d->status |= ST_BADQPOS; reset_data(m, d); }
  if (bad(d->qvel)) { d->status |= ST_BADQVEL; reset_data(m, d); }
  forward(m, d);
  if (bad(d->qacc)) {
    d->status |= ST_BADQACC;
    reset_data(m, d);
    forward(m, d);
  }
  euler(m, d);
}

}  // namespace orc
