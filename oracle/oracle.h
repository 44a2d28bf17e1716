/* oracle.h -- fp64 CPU restatement of the Adroit hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle and the timed CPU baseline ("port") for mj_envs_amd.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  It is never
 * linked into, or called by, the product library (mj_envs_amd/libadroit_hip.so).
 *
 * What it restates:
 *   - the task layer of the reference exactly: hammer_v0.py:54-132, door_v0.py:55-119,
 *     pen_v0.py:65-132, relocate_v0.py:46-103, utils/quatmath.py:79-164 (quat2euler);
 *   - MuJoCo 2.1.0's mj_step (mj_forward + mj_Euler) for the model features the Adroit
 *     MJCF uses.  MuJoCo 2.1 and mujoco-py are third-party, absent from
 *     /root/reference and not installed here: physics parity with the real
 *     mujoco-py path is UNPINNED.  The restatement follows MuJoCo's published computation
 *     model; where the exact 2.1 code is not recoverable the choice made is documented at
 *     the function (and in DESIGN.md).  The task layer IS pinned by golden vectors
 *     generated from the reference's own modules (tests/golden/).
 */
#ifndef AW_ORACLE_H
#define AW_ORACLE_H

#include <stdint.h>
#include <stddef.h>
#include <vector>

namespace orc {

typedef double num;

/* disable bits: MuJoCo 2.1 mjtDisableBit values, plus two of ours */
enum {
  DSBL_CONSTRAINT = 1 << 0,
  DSBL_EQUALITY = 1 << 1,
  DSBL_FRICTIONLOSS = 1 << 2,
  DSBL_LIMIT = 1 << 3,
  DSBL_CONTACT = 1 << 4,
  DSBL_PASSIVE = 1 << 5,
  DSBL_GRAVITY = 1 << 6,
  DSBL_CLAMPCTRL = 1 << 7,
  DSBL_WARMSTART = 1 << 8,
  DSBL_FILTERPARENT = 1 << 9,
  DSBL_ACTUATION = 1 << 10,
  DSBL_REFSAFE = 1 << 11,
  DSBL_SENSOR = 1 << 12,
  DSBL_NOSLIP = 1 << 14,    /* ours: skip the noslip pass */
  DSBL_EULERDAMP = 1 << 15, /* ours: explicit (not implicit) joint damping in Euler */
};

/* per-env status flags (shared meaning with include/adroit_wave.h) */
enum {
  ST_BADQPOS = 1,
  ST_BADQVEL = 2,
  ST_BADQACC = 4,
  ST_CON_OVERFLOW = 8,
  ST_EFC_OVERFLOW = 16,
};

enum { GEOM_PLANE = 0, GEOM_SPHERE = 2, GEOM_CAPSULE = 3, GEOM_ELLIPSOID = 4, GEOM_CYLINDER = 5, GEOM_BOX = 6, GEOM_MESH = 7 };
enum { JNT_SLIDE = 2, JNT_HINGE = 3 };
enum { CNSTR_FRICTION_DOF = 0, CNSTR_FRICTION_TENDON = 1, CNSTR_LIMIT_JOINT = 2, CNSTR_LIMIT_TENDON = 3,
       CNSTR_CONTACT_FRICTIONLESS = 4, CNSTR_CONTACT_PYRAMIDAL = 5 };
enum { CSTATE_SATISFIED = 0, CSTATE_QUADRATIC = 1, CSTATE_LINEARNEG = 2, CSTATE_LINEARPOS = 3 };

struct Model {
  int nq, nv, nu, nbody, njnt, ngeom, nsite, ntendon, nwrap, nsensor, npair, ncand;
  num timestep, gravity[3], tolerance, noslip_tolerance, impratio, mpr_tolerance, meaninertia;
  int iterations, noslip_iterations, mpr_iterations;
  int disableflags;
  int max_con, max_efc;
  /* test hook (or_set_margin_nudge): the margin of the geom pair (nudge_g1, nudge_g2), either order,
   * shifted by nudge_delta -- the parity classifier's causal check of a near-margin contact */
  int nudge_g1 = -1, nudge_g2 = -1;
  num nudge_delta = 0;

  std::vector<int> body_parentid, body_rootid, body_weldid, body_jntnum, body_jntadr, body_dofnum,
      body_dofadr, body_mocap;
  std::vector<num> body_pos, body_quat, body_ipos, body_iquat, body_mass, body_inertia,
      body_invweight0, body_subtreemass;
  std::vector<int> jnt_type, jnt_bodyid, jnt_qposadr, jnt_dofadr, jnt_limited;
  std::vector<num> jnt_pos, jnt_axis, jnt_range, jnt_margin, jnt_solref, jnt_solimp;
  std::vector<int> dof_bodyid, dof_jntid, dof_parentid;
  std::vector<num> dof_armature, dof_damping, dof_frictionloss, dof_solref, dof_solimp,
      dof_invweight0;
  std::vector<int> geom_type, geom_bodyid, geom_contype, geom_conaffinity, geom_condim,
      geom_priority;
  std::vector<num> geom_size, geom_pos, geom_quat, geom_friction, geom_solmix, geom_solref,
      geom_solimp, geom_margin, geom_gap, geom_rbound;
  std::vector<int> site_type, site_bodyid;
  std::vector<num> site_size, site_pos, site_quat;
  std::vector<int> tendon_adr, tendon_num, tendon_limited, wrap_jnt;
  std::vector<num> tendon_range, tendon_margin, tendon_solref, tendon_solimp,
      tendon_frictionloss, tendon_invweight0, wrap_coef;
  std::vector<int> actuator_trnid, actuator_ctrllimited, actuator_forcelimited;
  std::vector<num> actuator_gear, actuator_gainprm, actuator_biasprm, actuator_ctrlrange,
      actuator_forcerange;
  std::vector<int> sensor_type, sensor_objid, sensor_adr;
  std::vector<int> pair_geom1, pair_geom2, pair_condim, cand_geom1, cand_geom2;
  std::vector<num> pair_friction, pair_solref, pair_solimp, pair_margin, pair_gap;
  std::vector<num> qpos0;

  /* task block */
  int task_kind, task_frame_skip, task_horizon, task_obs_dim, task_nparam;
  std::vector<int> task_idx, task_param_field, task_param_obj, task_param_comp;
  std::vector<num> task_param_default, task_act_mid, task_act_rng;
  num pen_length, tar_length;
};

struct Contact {
  num dist, pos[3], frame[9], includemargin, friction[5], solref[2], solimp[5];
  int dim, geom1, geom2, efc_address;
};

struct Data {
  /* per-env model overrides (copies of the overridable model fields) */
  std::vector<num> body_pos, body_quat, site_pos, body_mass, geom_pos, geom_size;
  /* state */
  std::vector<num> qpos, qvel, qacc_warmstart, ctrl;
  num time;
  /* position-dependent */
  std::vector<num> xpos, xquat, xmat, xipos, ximat, xanchor, xaxis, geom_xpos, geom_xmat,
      site_xpos, site_xmat, subtree_com, cinert, cdof, crb, ten_length, ten_J, qM, qLD,
      qLDiagInv, qH, qHDiagInv, actuator_length;
  /* velocity-dependent */
  std::vector<num> cvel, cdof_dot, qfrc_bias, qfrc_passive, actuator_velocity;
  /* forces / accelerations */
  std::vector<num> actuator_force, qfrc_actuator, qfrc_smooth, qacc_smooth, qfrc_constraint,
      qacc;
  /* contacts and constraints */
  int ncon;
  std::vector<Contact> contact;
  int nefc;
  std::vector<int> efc_type, efc_id, efc_state;
  std::vector<num> efc_J, efc_pos, efc_margin, efc_frictionloss, efc_diagApprox, efc_R, efc_D,
      efc_aref, efc_vel, efc_force, efc_b;
  std::vector<num> sensordata;
  int solver_iter, noslip_iter;
  int ls_iter;          /* line-search derivative evaluations of the last Newton solve (incl. alpha = 0) */
  uint32_t status;
  /* scratch */
  std::vector<num> scratch;
};

/* model.cc */
int load_model(Model* m, const void* blob, size_t nbytes);
void init_data(const Model* m, Data* d);
void apply_params(const Model* m, Data* d, const num* params);

/* mjstep.cc */
void kinematics(const Model* m, Data* d);
void com_pos(const Model* m, Data* d);
void tendon(const Model* m, Data* d);
void crb(const Model* m, Data* d);
void factor_lower(const Model* m, const num* M, num* LD, num* diaginv);
void solve_ld(const Model* m, const num* LD, const num* diaginv, num* x);
void com_vel(const Model* m, Data* d);
void rne(const Model* m, Data* d);
void passive(const Model* m, Data* d);
void actuation(const Model* m, Data* d);
void forward(const Model* m, Data* d);
void euler(const Model* m, Data* d);
void step(const Model* m, Data* d);
void reset_data(const Model* m, Data* d);
void sensors(const Model* m, Data* d);
void mul_M(const Model* m, const Data* d, const num* x, num* y);

/* collide.cc */
void collision(const Model* m, Data* d);
int collide_geoms(const Model* m, const Data* d, int g1, int g2, num margin, Contact* out, int maxout);
int collide_raw(const Model* m, int t1, const num* p1, const num* m1, const num* s1, int t2, const num* p2,
                const num* m2, const num* s2, num margin, Contact* out);
num ray_geom(const num* pos, const num* mat, const num* size, const num* pnt, const num* vec, int type);

/* solver.cc */
void make_constraint(const Model* m, Data* d);
void fwd_constraint(const Model* m, Data* d);
void contact_force(const Model* m, const Data* d, int i, num* result6);

/* task.cc */
void task_obs(const Model* m, const Data* d, num* obs);
void task_reward(const Model* m, const Data* d, num* reward, uint8_t* done, uint8_t* goal,
                 int starting_up);
void quat2euler(const num* q, num* euler);

/* small vector helpers */
static inline num dot3(const num* a, const num* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline void cross3(num* r, const num* a, const num* b) {
  num t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static inline void sub3(num* r, const num* a, const num* b) { r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2]; }
static inline void add3(num* r, const num* a, const num* b) { r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2]; }
static inline void scl3(num* r, const num* a, num s) { r[0] = a[0] * s; r[1] = a[1] * s; r[2] = a[2] * s; }
static inline void copy3(num* r, const num* a) { r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; }
num norm3(const num* a);
num normalize3(num* a);
void mul_mat_vec3(num* r, const num* mat, const num* v);   /* r = mat * v (row-major 3x3) */
void mul_matT_vec3(num* r, const num* mat, const num* v);  /* r = mat' * v */
void mul_quat(num* r, const num* a, const num* b);
void rot_vec_quat(num* r, const num* v, const num* q);
void quat2mat(num* mat, const num* q);
void axis_angle2quat(num* q, const num* axis, num angle);
void normalize4(num* q);
void mul_mat_mat3(num* r, const num* a, const num* b);
void make_frame(num* frame);

}  // namespace orc

#endif
