/* model.cc -- oracle model loading from the flat table (TEST INFRASTRUCTURE ONLY, see oracle.h). */
#include <cmath>
#include <cstring>

#include "../include/aw_blob.h"
#include "oracle.h"

namespace orc {

namespace {
struct Reader {
  const void* blob;
  size_t n;
  bool ok = true;
  void f(const char* name, std::vector<num>& out, bool required = true) {
    aw_blob_entry e;
    if (!aw_blob_find(blob, n, name, &e)) {
      if (required) ok = false;
      out.clear();
      return;
    }
    size_t cnt = (size_t)e.rows * e.cols;
    out.resize(cnt);
    const char* p = (const char*)e.data;
    for (size_t i = 0; i < cnt; i++) {
      if (e.kind == 0) {
        double v; memcpy(&v, p + 8 * i, 8); out[i] = v;
      } else {
        int32_t v; memcpy(&v, p + 4 * i, 4); out[i] = v;
      }
    }
  }
  void i(const char* name, std::vector<int>& out, bool required = true) {
    aw_blob_entry e;
    if (!aw_blob_find(blob, n, name, &e)) {
      if (required) ok = false;
      out.clear();
      return;
    }
    size_t cnt = (size_t)e.rows * e.cols;
    out.resize(cnt);
    const char* p = (const char*)e.data;
    for (size_t k = 0; k < cnt; k++) {
      if (e.kind == 1) {
        int32_t v; memcpy(&v, p + 4 * k, 4); out[k] = v;
      } else {
        double v; memcpy(&v, p + 8 * k, 8); out[k] = (int)v;
      }
    }
  }
};
}  // namespace

int load_model(Model* m, const void* blob, size_t nbytes) {
  Reader r{blob, nbytes};
#define DIM(x) m->x = aw_blob_dim(blob, nbytes, #x, -1); if (m->x < 0) return -1;
  DIM(nq) DIM(nv) DIM(nu) DIM(nbody) DIM(njnt) DIM(ngeom) DIM(nsite) DIM(ntendon) DIM(nwrap)
  DIM(nsensor) DIM(npair) DIM(ncand)
#undef DIM
  m->timestep = aw_blob_opt(blob, nbytes, "timestep", 0.002);
  m->gravity[0] = aw_blob_opt(blob, nbytes, "gravity_x", 0);
  m->gravity[1] = aw_blob_opt(blob, nbytes, "gravity_y", 0);
  m->gravity[2] = aw_blob_opt(blob, nbytes, "gravity_z", -9.81);
  m->iterations = (int)aw_blob_opt(blob, nbytes, "iterations", 100);
  m->tolerance = aw_blob_opt(blob, nbytes, "tolerance", 1e-8);
  m->noslip_iterations = (int)aw_blob_opt(blob, nbytes, "noslip_iterations", 0);
  m->noslip_tolerance = aw_blob_opt(blob, nbytes, "noslip_tolerance", 1e-6);
  m->impratio = aw_blob_opt(blob, nbytes, "impratio", 1);
  m->mpr_tolerance = aw_blob_opt(blob, nbytes, "mpr_tolerance", 1e-6);
  m->mpr_iterations = (int)aw_blob_opt(blob, nbytes, "mpr_iterations", 50);
  m->meaninertia = aw_blob_opt(blob, nbytes, "meaninertia", 1);
  m->disableflags = 0;
  m->max_con = 100;   // MuJoCo's nconmax / njmax of the reference model (DAPG_assets.xml:4)
  m->max_efc = 500;

  r.i("body_parentid", m->body_parentid); r.i("body_rootid", m->body_rootid);
  r.i("body_weldid", m->body_weldid); r.i("body_jntnum", m->body_jntnum);
  r.i("body_jntadr", m->body_jntadr); r.i("body_dofnum", m->body_dofnum);
  r.i("body_dofadr", m->body_dofadr); r.i("body_mocap", m->body_mocap);
  r.f("body_pos", m->body_pos); r.f("body_quat", m->body_quat); r.f("body_ipos", m->body_ipos);
  r.f("body_iquat", m->body_iquat); r.f("body_mass", m->body_mass);
  r.f("body_inertia", m->body_inertia); r.f("body_invweight0", m->body_invweight0);
  r.f("body_subtreemass", m->body_subtreemass);
  r.i("jnt_type", m->jnt_type); r.i("jnt_bodyid", m->jnt_bodyid);
  r.i("jnt_qposadr", m->jnt_qposadr); r.i("jnt_dofadr", m->jnt_dofadr);
  r.i("jnt_limited", m->jnt_limited); r.f("jnt_pos", m->jnt_pos); r.f("jnt_axis", m->jnt_axis);
  r.f("jnt_range", m->jnt_range); r.f("jnt_margin", m->jnt_margin);
  r.f("jnt_solref", m->jnt_solref); r.f("jnt_solimp", m->jnt_solimp);
  r.i("dof_bodyid", m->dof_bodyid); r.i("dof_jntid", m->dof_jntid);
  r.i("dof_parentid", m->dof_parentid); r.f("dof_armature", m->dof_armature);
  r.f("dof_damping", m->dof_damping); r.f("dof_frictionloss", m->dof_frictionloss);
  r.f("dof_solref", m->dof_solref); r.f("dof_solimp", m->dof_solimp);
  r.f("dof_invweight0", m->dof_invweight0);
  r.i("geom_type", m->geom_type); r.i("geom_bodyid", m->geom_bodyid);
  r.i("geom_contype", m->geom_contype); r.i("geom_conaffinity", m->geom_conaffinity);
  r.i("geom_condim", m->geom_condim); r.i("geom_priority", m->geom_priority);
  r.f("geom_size", m->geom_size); r.f("geom_pos", m->geom_pos); r.f("geom_quat", m->geom_quat);
  r.f("geom_friction", m->geom_friction); r.f("geom_solmix", m->geom_solmix);
  r.f("geom_solref", m->geom_solref); r.f("geom_solimp", m->geom_solimp);
  r.f("geom_margin", m->geom_margin); r.f("geom_gap", m->geom_gap);
  r.f("geom_rbound", m->geom_rbound);
  r.i("site_type", m->site_type); r.i("site_bodyid", m->site_bodyid);
  r.f("site_size", m->site_size); r.f("site_pos", m->site_pos); r.f("site_quat", m->site_quat);
  r.i("tendon_adr", m->tendon_adr); r.i("tendon_num", m->tendon_num);
  r.i("tendon_limited", m->tendon_limited); r.i("wrap_jnt", m->wrap_jnt);
  r.f("tendon_range", m->tendon_range); r.f("tendon_margin", m->tendon_margin);
  r.f("tendon_solref", m->tendon_solref); r.f("tendon_solimp", m->tendon_solimp);
  r.f("tendon_frictionloss", m->tendon_frictionloss);
  r.f("tendon_invweight0", m->tendon_invweight0); r.f("wrap_coef", m->wrap_coef);
  r.i("actuator_trnid", m->actuator_trnid); r.i("actuator_ctrllimited", m->actuator_ctrllimited);
  r.i("actuator_forcelimited", m->actuator_forcelimited); r.f("actuator_gear", m->actuator_gear);
  r.f("actuator_gainprm", m->actuator_gainprm); r.f("actuator_biasprm", m->actuator_biasprm);
  r.f("actuator_ctrlrange", m->actuator_ctrlrange);
  r.f("actuator_forcerange", m->actuator_forcerange);
  r.i("sensor_type", m->sensor_type); r.i("sensor_objid", m->sensor_objid);
  r.i("sensor_adr", m->sensor_adr);
  r.i("pair_geom1", m->pair_geom1); r.i("pair_geom2", m->pair_geom2);
  r.i("pair_condim", m->pair_condim); r.f("pair_friction", m->pair_friction);
  r.f("pair_solref", m->pair_solref); r.f("pair_solimp", m->pair_solimp);
  r.f("pair_margin", m->pair_margin); r.f("pair_gap", m->pair_gap);
  r.i("cand_geom1", m->cand_geom1); r.i("cand_geom2", m->cand_geom2);
  r.f("qpos0", m->qpos0);
  if (!r.ok) return -2;

  m->task_kind = aw_blob_dim(blob, nbytes, "task_kind", -1);
  m->task_frame_skip = aw_blob_dim(blob, nbytes, "task_frame_skip", 1);
  m->task_horizon = aw_blob_dim(blob, nbytes, "task_horizon", 0);
  m->task_obs_dim = aw_blob_dim(blob, nbytes, "task_obs_dim", 0);
  m->task_nparam = aw_blob_dim(blob, nbytes, "task_nparam", 0);
  r.i("task_idx", m->task_idx, false);
  r.i("task_param_field", m->task_param_field, false);
  r.i("task_param_obj", m->task_param_obj, false);
  r.i("task_param_comp", m->task_param_comp, false);
  r.f("task_param_default", m->task_param_default, false);
  r.f("task_act_mid", m->task_act_mid, false);
  r.f("task_act_rng", m->task_act_rng, false);
  m->pen_length = aw_blob_opt(blob, nbytes, "task_pen_length", 1.0);
  m->tar_length = aw_blob_opt(blob, nbytes, "task_tar_length", 1.0);
  return 0;
}

void init_data(const Model* m, Data* d) {
  int nb = m->nbody, nv = m->nv, ng = m->ngeom, ns = m->nsite, nt = m->ntendon;
  d->body_pos = m->body_pos; d->body_quat = m->body_quat; d->site_pos = m->site_pos;
  d->body_mass = m->body_mass; d->geom_pos = m->geom_pos; d->geom_size = m->geom_size;
  d->qpos.assign(m->nq, 0); d->qvel.assign(nv, 0); d->qacc_warmstart.assign(nv, 0);
  d->ctrl.assign(m->nu, 0); d->time = 0;
  d->xpos.assign(3 * nb, 0); d->xquat.assign(4 * nb, 0); d->xmat.assign(9 * nb, 0);
  d->xipos.assign(3 * nb, 0); d->ximat.assign(9 * nb, 0);
  d->xanchor.assign(3 * m->njnt, 0); d->xaxis.assign(3 * m->njnt, 0);
  d->geom_xpos.assign(3 * ng, 0); d->geom_xmat.assign(9 * ng, 0);
  d->site_xpos.assign(3 * ns, 0); d->site_xmat.assign(9 * ns, 0);
  d->subtree_com.assign(3 * nb, 0); d->cinert.assign(10 * nb, 0); d->cdof.assign(6 * nv, 0);
  d->crb.assign(10 * nb, 0); d->ten_length.assign(nt, 0); d->ten_J.assign((size_t)nt * nv, 0);
  d->qM.assign((size_t)nv * nv, 0); d->qLD.assign((size_t)nv * nv, 0); d->qLDiagInv.assign(nv, 0);
  d->qH.assign((size_t)nv * nv, 0); d->qHDiagInv.assign(nv, 0);
  d->actuator_length.assign(m->nu, 0); d->actuator_velocity.assign(m->nu, 0);
  d->cvel.assign(6 * nb, 0); d->cdof_dot.assign(6 * nv, 0);
  d->qfrc_bias.assign(nv, 0); d->qfrc_passive.assign(nv, 0);
  d->actuator_force.assign(m->nu, 0); d->qfrc_actuator.assign(nv, 0);
  d->qfrc_smooth.assign(nv, 0); d->qacc_smooth.assign(nv, 0); d->qfrc_constraint.assign(nv, 0);
  d->qacc.assign(nv, 0);
  d->ncon = 0; d->contact.resize(m->max_con);
  d->nefc = 0;
  int E = m->max_efc;
  d->efc_type.assign(E, 0); d->efc_id.assign(E, 0); d->efc_state.assign(E, 0);
  d->efc_J.assign((size_t)E * nv, 0);
  d->efc_pos.assign(E, 0); d->efc_margin.assign(E, 0); d->efc_frictionloss.assign(E, 0);
  d->efc_diagApprox.assign(E, 0); d->efc_R.assign(E, 0); d->efc_D.assign(E, 0);
  d->efc_aref.assign(E, 0); d->efc_vel.assign(E, 0); d->efc_force.assign(E, 0);
  d->efc_b.assign(E, 0);
  d->sensordata.assign(m->nsensor, 0);
  d->solver_iter = d->noslip_iter = d->ls_iter = 0;
  d->status = 0;
}

void apply_params(const Model* m, Data* d, const num* params) {
  d->body_pos = m->body_pos; d->body_quat = m->body_quat; d->site_pos = m->site_pos;
  d->body_mass = m->body_mass; d->geom_pos = m->geom_pos; d->geom_size = m->geom_size;
  for (int p = 0; p < m->task_nparam; p++) {
    int o = m->task_param_obj[p], c = m->task_param_comp[p];
    num v = params ? params[p] : m->task_param_default[p];
    switch (m->task_param_field[p]) {
      case 0: d->body_pos[3 * o + c] = v; break;
      case 1: d->body_quat[4 * o + c] = v; break;
      case 2: d->site_pos[3 * o + c] = v; break;
      case 3: d->body_mass[o] = v; break;
      case 4: d->geom_pos[3 * o + c] = v; break;
      case 5: d->geom_size[3 * o + c] = v; break;
    }
  }
}

}  // namespace orc
