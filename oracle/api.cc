/* api.cc -- ctypes entry points of the CPU oracle (TEST INFRASTRUCTURE ONLY, see oracle.h).
 *
 * Batched env semantics restate the reference env methods:
 *   or_reset : mjrl MujocoEnv.reset -> sim.reset() + reset_model (hammer_v0.py:106-132,
 *              door_v0.py:103-119, pen_v0.py:115-132, relocate_v0.py:85-103)
 *   or_step  : *EnvV0.step (hammer_v0.py:54-90 ...): clip, scale (act_mid/act_rng),
 *              do_simulation(ctrl, frame_skip), obs, reward, done, goal_achieved
 */
#include <cstring>
#include <string>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "oracle.h"

using namespace orc;

namespace {
struct Handle {
  Model m;
  Data d1;  /* single-env introspection data */
};

void load_state(const Model* m, Data* d, const double* qpos, const double* qvel, const double* warm) {
  for (int i = 0; i < m->nq; i++) d->qpos[i] = qpos[i];
  for (int i = 0; i < m->nv; i++) d->qvel[i] = qvel[i];
  for (int i = 0; i < m->nv; i++) d->qacc_warmstart[i] = warm ? warm[i] : 0.0;
}
void store_state(const Model* m, const Data* d, double* qpos, double* qvel, double* warm) {
  for (int i = 0; i < m->nq; i++) qpos[i] = d->qpos[i];
  for (int i = 0; i < m->nv; i++) qvel[i] = d->qvel[i];
  if (warm)
    for (int i = 0; i < m->nv; i++) warm[i] = d->qacc_warmstart[i];
}
void env_step(const Model* m, Data* d, const double* action) {
  for (int i = 0; i < m->nu; i++) {
    double a = action[i];
    a = a < -1.0 ? -1.0 : (a > 1.0 ? 1.0 : a);
    d->ctrl[i] = m->task_act_mid[i] + a * m->task_act_rng[i];
  }
  for (int k = 0; k < m->task_frame_skip; k++) step(m, d);
}
}  // namespace

extern "C" {

void* or_create(const void* blob, size_t nbytes) {
  Handle* h = new Handle();
  if (load_model(&h->m, blob, nbytes) != 0) { delete h; return nullptr; }
  init_data(&h->m, &h->d1);
  return h;
}

void or_destroy(void* p) { delete (Handle*)p; }

/* negative arguments keep the current value */
void or_set_option(void* p, int disableflags, int max_con, int max_efc, int iterations, int noslip_iterations) {
  Handle* h = (Handle*)p;
  if (disableflags >= 0) h->m.disableflags = disableflags;
  if (max_con > 0) h->m.max_con = max_con;
  if (max_efc > 0) h->m.max_efc = max_efc;
  if (iterations >= 0) h->m.iterations = iterations;
  if (noslip_iterations >= 0) h->m.noslip_iterations = noslip_iterations;
  init_data(&h->m, &h->d1);
}

/* test hook: shift the margin of one geom pair (model geom ids, either order; g1 < 0 clears) */
void or_set_margin_nudge(void* p, int g1, int g2, double delta) {
  Handle* h = (Handle*)p;
  h->m.nudge_g1 = g1; h->m.nudge_g2 = g2; h->m.nudge_delta = g1 < 0 ? 0.0 : delta;
}

int or_dims(void* p, int* out) {
  const Model& m = ((Handle*)p)->m;
  int v[] = {m.nq, m.nv, m.nu, m.nbody, m.ngeom, m.nsite, m.task_obs_dim, m.task_nparam,
             m.task_frame_skip, m.task_horizon, m.nsensor, m.ntendon, m.max_con, m.max_efc};
  memcpy(out, v, sizeof(v));
  return (int)(sizeof(v) / sizeof(int));
}

int or_reset(void* p, int n, const double* params, double* qpos, double* qvel, double* warm,
             double* obs, int nthreads) {
  const Model* m = &((Handle*)p)->m;
  int P = m->task_nparam, O = m->task_obs_dim;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
  {
    Data d;
    init_data(m, &d);
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
    for (int e = 0; e < n; e++) {
      reset_data(m, &d);
      apply_params(m, &d, params ? params + (size_t)e * P : nullptr);
      forward(m, &d);
      store_state(m, &d, qpos + (size_t)e * m->nq, qvel + (size_t)e * m->nv, warm ? warm + (size_t)e * m->nv : nullptr);
      if (obs) task_obs(m, &d, obs + (size_t)e * O);
    }
  }
  return 0;
}

int or_step(void* p, int n, const double* params, const double* action, double* qpos, double* qvel,
            double* warm, double* obs, double* reward, uint8_t* done, uint8_t* goal, uint32_t* status,
            int nthreads) {
  const Model* m = &((Handle*)p)->m;
  int P = m->task_nparam, O = m->task_obs_dim;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
  {
    Data d;
    init_data(m, &d);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
    for (int e = 0; e < n; e++) {
      apply_params(m, &d, params ? params + (size_t)e * P : nullptr);
      load_state(m, &d, qpos + (size_t)e * m->nq, qvel + (size_t)e * m->nv, warm ? warm + (size_t)e * m->nv : nullptr);
      d.status = 0;
      env_step(m, &d, action + (size_t)e * m->nu);
      store_state(m, &d, qpos + (size_t)e * m->nq, qvel + (size_t)e * m->nv, warm ? warm + (size_t)e * m->nv : nullptr);
      if (obs) task_obs(m, &d, obs + (size_t)e * O);
      double r;
      uint8_t dn, gl;
      task_reward(m, &d, &r, &dn, &gl, 0);
      if (reward) reward[e] = r;
      if (done) done[e] = dn;
      if (goal) goal[e] = gl;
      if (status) status[e] = d.status;
    }
  }
  return 0;
}

/* or_step + per-env work counts of the env-step (test / profiling hook, tools/work_counts.py):
 * stats[e][12] = max ncon, max nefc, max dense (contact) rows over the frame_skip substeps, summed
 * Newton iterations, line-search derivative evaluations and noslip sweeps, substeps, status, summed
 * ncon, nefc and dense rows, substeps with a box-box contact */
int or_step_stats(void* p, int n, const double* params, const double* action, double* qpos, double* qvel,
                  double* warm, double* obs, double* reward, uint8_t* done, uint8_t* goal, int32_t* stats,
                  int nthreads) {
  const Model* m = &((Handle*)p)->m;
  int P = m->task_nparam, O = m->task_obs_dim;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
  {
    Data d;
    init_data(m, &d);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
    for (int e = 0; e < n; e++) {
      apply_params(m, &d, params ? params + (size_t)e * P : nullptr);
      load_state(m, &d, qpos + (size_t)e * m->nq, qvel + (size_t)e * m->nv, warm ? warm + (size_t)e * m->nv : nullptr);
      d.status = 0;
      const double* a = action + (size_t)e * m->nu;
      for (int i = 0; i < m->nu; i++) {
        double x = a[i] < -1.0 ? -1.0 : (a[i] > 1.0 ? 1.0 : a[i]);
        d.ctrl[i] = m->task_act_mid[i] + x * m->task_act_rng[i];
      }
      int32_t* st = stats + (size_t)e * 12;
      for (int k = 0; k < 12; k++) st[k] = 0;
      for (int k = 0; k < m->task_frame_skip; k++) {
        step(m, &d);
        int nd = 0;
        for (int i = 0; i < d.nefc; i++) nd += d.efc_type[i] >= CNSTR_CONTACT_FRICTIONLESS;
        st[0] = d.ncon > st[0] ? d.ncon : st[0];
        st[1] = d.nefc > st[1] ? d.nefc : st[1];
        st[2] = nd > st[2] ? nd : st[2];
        st[3] += d.solver_iter; st[4] += d.ls_iter; st[5] += d.noslip_iter; st[6] += 1;
        st[8] += d.ncon; st[9] += d.nefc; st[10] += nd;
        int bb = 0;
        for (int c = 0; c < d.ncon; c++)
          bb |= m->geom_type[d.contact[c].geom1] == GEOM_BOX && m->geom_type[d.contact[c].geom2] == GEOM_BOX;
        st[11] += bb;
      }
      st[7] = (int32_t)d.status;
      store_state(m, &d, qpos + (size_t)e * m->nq, qvel + (size_t)e * m->nv, warm ? warm + (size_t)e * m->nv : nullptr);
      if (obs) task_obs(m, &d, obs + (size_t)e * O);
      double r;
      uint8_t dn, gl;
      task_reward(m, &d, &r, &dn, &gl, 0);
      if (reward) reward[e] = r;
      if (done) done[e] = dn;
      if (goal) goal[e] = gl;
    }
  }
  return 0;
}

/* ---- single-env introspection --------------------------------------------------------- */
int or_forward1(void* p, const double* params, const double* qpos, const double* qvel,
                const double* warm, const double* ctrl) {
  Handle* h = (Handle*)p;
  Data* d = &h->d1;
  apply_params(&h->m, d, params);
  load_state(&h->m, d, qpos, qvel, warm);
  for (int i = 0; i < h->m.nu; i++) d->ctrl[i] = ctrl ? ctrl[i] : 0.0;
  d->status = 0;
  forward(&h->m, d);
  return 0;
}

int or_mjstep1(void* p, const double* params, double* qpos, double* qvel, double* warm, const double* ctrl, int nstep) {
  Handle* h = (Handle*)p;
  Data* d = &h->d1;
  apply_params(&h->m, d, params);
  load_state(&h->m, d, qpos, qvel, warm);
  for (int i = 0; i < h->m.nu; i++) d->ctrl[i] = ctrl ? ctrl[i] : 0.0;
  d->status = 0;
  for (int k = 0; k < nstep; k++) step(&h->m, d);
  store_state(&h->m, d, qpos, qvel, warm);
  return (int)d->status;
}

/* copy a named array of the introspection data; returns the element count */
int or_get1(void* p, const char* name, double* out, int cap) {
  Handle* h = (Handle*)p;
  const Data* d = &h->d1;
  const Model* m = &h->m;
  std::string s(name);
  const std::vector<double>* v = nullptr;
  size_t cnt = 0;
#define F(x, n) if (s == #x) { v = &d->x; cnt = (n); }
  F(xpos, 3 * m->nbody) F(xquat, 4 * m->nbody) F(xmat, 9 * m->nbody) F(xipos, 3 * m->nbody)
  F(geom_xpos, 3 * m->ngeom) F(geom_xmat, 9 * m->ngeom) F(site_xpos, 3 * m->nsite)
  F(site_xmat, 9 * m->nsite) F(subtree_com, 3 * m->nbody) F(cinert, 10 * m->nbody)
  F(cdof, 6 * m->nv) F(qM, (size_t)m->nv * m->nv) F(qLD, (size_t)m->nv * m->nv)
  F(qLDiagInv, m->nv) F(ten_length, m->ntendon) F(cvel, 6 * m->nbody) F(cdof_dot, 6 * m->nv)
  F(qfrc_bias, m->nv) F(qfrc_passive, m->nv) F(qfrc_actuator, m->nv) F(qfrc_smooth, m->nv)
  F(qacc_smooth, m->nv) F(qfrc_constraint, m->nv) F(qacc, m->nv) F(sensordata, m->nsensor)
  F(actuator_force, m->nu) F(qpos, m->nq) F(qvel, m->nv) F(qacc_warmstart, m->nv)
  F(efc_J, (size_t)d->nefc * m->nv) F(efc_pos, d->nefc) F(efc_margin, d->nefc)
  F(efc_D, d->nefc) F(efc_R, d->nefc) F(efc_aref, d->nefc) F(efc_force, d->nefc)
  F(efc_vel, d->nefc) F(efc_diagApprox, d->nefc) F(efc_frictionloss, d->nefc)
#undef F
  if (v) {
    if (out)
      for (size_t i = 0; i < cnt && (int)i < cap; i++) out[i] = (*v)[i];
    return (int)cnt;
  }
  std::vector<double> tmp;
  if (s == "scalars") {
    tmp = {(double)d->ncon, (double)d->nefc, (double)d->solver_iter, (double)d->noslip_iter, (double)d->status,
           (double)d->ls_iter};
  } else if (s == "efc_type") {
    for (int i = 0; i < d->nefc; i++) tmp.push_back(d->efc_type[i]);
  } else if (s == "efc_id") {
    for (int i = 0; i < d->nefc; i++) tmp.push_back(d->efc_id[i]);
  } else if (s == "efc_state") {
    for (int i = 0; i < d->nefc; i++) tmp.push_back(d->efc_state[i]);
  } else if (s == "contact") {
    /* per contact: dist, pos(3), frame(9), geom1, geom2, dim, efc_address, includemargin, friction(5) */
    for (int c = 0; c < d->ncon; c++) {
      const Contact& k = d->contact[c];
      tmp.push_back(k.dist);
      for (int q = 0; q < 3; q++) tmp.push_back(k.pos[q]);
      for (int q = 0; q < 9; q++) tmp.push_back(k.frame[q]);
      tmp.push_back(k.geom1); tmp.push_back(k.geom2); tmp.push_back(k.dim);
      tmp.push_back(k.efc_address); tmp.push_back(k.includemargin);
      for (int q = 0; q < 5; q++) tmp.push_back(k.friction[q]);
    }
  } else if (s == "obs") {
    tmp.resize(m->task_obs_dim);
    task_obs(m, d, tmp.data());
  } else if (s == "reward") {
    double r;
    uint8_t dn, gl;
    task_reward(m, d, &r, &dn, &gl, 0);
    tmp = {r, (double)dn, (double)gl};
  } else {
    return -1;
  }
  if (out)
    for (size_t i = 0; i < tmp.size() && (int)i < cap; i++) out[i] = tmp[i];
  return (int)tmp.size();
}

/* Test hook: narrowphase of two primitives (types, world positions, row-major rotation
 * matrices, sizes) with the handle's MPR options.  out: up to 16 contacts x (dist, pos[3],
 * normal[3]) pointing from the first-listed (lower type) geom to the other; returns the count. */
int or_collide(void* p, int t1, const double* p1, const double* m1, const double* s1, int t2, const double* p2,
               const double* m2, const double* s2, double margin, double* out) {
  Handle* h = (Handle*)p;
  Contact buf[16];
  int n = collide_raw(&h->m, t1, p1, m1, s1, t2, p2, m2, s2, margin, buf);
  for (int i = 0; i < n; i++) {
    out[7 * i] = buf[i].dist;
    for (int k = 0; k < 3; k++) { out[7 * i + 1 + k] = buf[i].pos[k]; out[7 * i + 4 + k] = buf[i].frame[k]; }
  }
  return n;
}

/* exposed for the golden-vector test of the task layer: quat2euler (quatmath.py:136) */
void or_quat2euler(const double* q, double* e) { quat2euler(q, e); }

/* task layer on caller-provided kinematics: sets qpos/qvel/xpos/xquat/site_xpos/sensordata */
int or_task_eval(void* p, const double* qpos, const double* qvel, const double* xpos,
                 const double* xquat, const double* site_xpos, const double* sensordata,
                 double* obs, double* rdg) {
  Handle* h = (Handle*)p;
  Data* d = &h->d1;
  const Model* m = &h->m;
  memcpy(d->qpos.data(), qpos, sizeof(double) * m->nq);
  memcpy(d->qvel.data(), qvel, sizeof(double) * m->nv);
  memcpy(d->xpos.data(), xpos, sizeof(double) * 3 * m->nbody);
  memcpy(d->xquat.data(), xquat, sizeof(double) * 4 * m->nbody);
  memcpy(d->site_xpos.data(), site_xpos, sizeof(double) * 3 * m->nsite);
  memcpy(d->sensordata.data(), sensordata, sizeof(double) * m->nsensor);
  task_obs(m, d, obs);
  double r;
  uint8_t dn, gl;
  task_reward(m, d, &r, &dn, &gl, 0);
  rdg[0] = r; rdg[1] = dn; rdg[2] = gl;
  return 0;
}

}  // extern "C"
