// aw_common.h -- device model, per-env LDS layout and wave primitives for the Adroit kernels.
//
// Execution model (MI355X / gfx950): one 64-lane wavefront simulates one env; a workgroup is
// exactly one wave, so the per-env working set lives in that workgroup's LDS and lanes map to
// bodies / dofs / geom pairs / constraint rows as each stage needs.  Matrices whose rows are
// consumed lane-parallel (M, H, M + hD) live in VGPRs, one row per lane, and are factored with
// v_readlane broadcasts (no LDS round trips in the Cholesky inner loop).  The model (fp32,
// ~25 KB) is read from HBM through the L1/L2; every wave reads the same bytes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define AW_DEV __device__ __attribute__((always_inline)) inline

namespace aw {

constexpr int MAXV = 36;      // dofs (relocate: 36)
constexpr int CHOL_P = 4;      // Cholesky panel width (aw_solver.h chol_factor)
constexpr int VS = 36;        // J row stride: 144 B rows keep 16-byte alignment, so broadcast reads of a row are ds_read_b128
constexpr int MAXB = 32;      // bodies incl. world
constexpr int MAXG = 36;      // collidable geoms (compact list)
constexpr int MAXS = 32;      // sites
constexpr int MAXT = 44;      // tendons
constexpr int MAXU = 30;      // actuators
// Constraint capacities: the fast / wide tiers below.  The fast tier's were sized from the
// oracle's work counts at MuJoCo's own capacities (nconmax 100 / njmax 500, DAPG_assets.xml:4)
// under the reference's pretrained DAPG policies (profiles/work_counts_*_dapg.json: max ncon 20,
// nefc 130, dense rows 98 over 4 tasks x 32 envs x one horizon).
constexpr int MAXJB = 6;      // joints of one body (the free objects' 3 slides + 3 hinges)
constexpr int MAXP = 8;       // per-env model parameters
constexpr int MAXLEV = 16;    // kinematic tree depth
constexpr int MAXTOUCH = 4;   // task touch sensors
constexpr int MAXPAIRCON = 8; // contacts per geom pair
constexpr int NCLASS = 5;      // collider classes: plane-*, round-round, round-box, box-box, MPR

}  // namespace aw

// ---------------------------------------------------------------------------------------
// Two capacity tiers, one source.  The FAST tier (k_step, two waves per SIMD) holds the
// constraint sizes above, which cover all but ~1e-5 of env-steps (relocate's random-action tail
// reaches 126 dense rows in 1 024 envs x 200 steps, tools/capacity_tail.py).  An env-step that
// needs more is not truncated: the fast tier abandons it before writing anything and queues it
// for the WIDE tier (k_step_wide, the same code compiled with -DAW_WIDE), which holds MuJoCo's
// own capacities -- nconmax 100 contacts and njmax 500 constraint rows (DAPG_assets.xml:4) -- and
// re-runs the env-step from its unchanged pre-step state.  So the only constraints ever dropped
// are the ones MuJoCo drops, with its ST_*_OVERFLOW flags.  Every Env-dependent definition lives in
// a per-tier inline namespace, so the two translation units that instantiate the same functions
// with different capacities never share a (mangled) name.
namespace aw {
// Fast-tier dense-row capacity per task: 128 (the DAPG regimes peak at 98, random hammer at 37);
// relocate's random-action tail -- the hand cupping the ball, 25-30 pyramidal contacts -- reaches
// 126-140 dense rows, so relocate's fast tier holds 192 (its whole row capacity) and the wide tier
// sees 2 instead of 10 of 16 384 envs per 200 steps: config 3 relocate -4.4 %, hammer unchanged
// (r05q A/B).  The host allocates the spill blocks for the largest value.
constexpr int fast_maxdense_of(int task) { return task == 3 ? 192 : 128; }
constexpr int FAST_MAXDENSE_ALLOC = 192;
// The value is a preprocessor literal (AW_FAST_MD) because it also names the fast tier's inline
// namespace (fast128 / fast192 below): relocate's task unit and the others compile Env -- and every
// always-inline function taking one -- at different sizes, so their mangled names must differ too.
#if defined(AW_FAST_MAXDENSE)
#define AW_FAST_MD AW_FAST_MAXDENSE   // explicit override (tools/build_variant.py): a literal
#elif (defined(AW_TASK_TU) && AW_TASK_TU == 3) || (defined(AW_ONLY_TASK) && AW_ONLY_TASK == 3)
#define AW_FAST_MD 192
#else
#define AW_FAST_MD 128   // the other tasks, the API unit, single-TU builds of all four tasks
#endif
#if defined(AW_TASK_TU) && !defined(AW_FAST_MAXDENSE)
static_assert(AW_FAST_MD == fast_maxdense_of(AW_TASK_TU), "fast_maxdense_of and AW_FAST_MD disagree");
#elif defined(AW_ONLY_TASK) && !defined(AW_FAST_MAXDENSE)
static_assert(AW_FAST_MD == fast_maxdense_of(AW_ONLY_TASK), "fast_maxdense_of and AW_FAST_MD disagree");
#endif
constexpr int FAST_MAXCON = 48, FAST_NRL = 3, FAST_MAXDENSE = AW_FAST_MD;
static_assert(FAST_MAXDENSE <= FAST_MAXDENSE_ALLOC, "fast spill blocks are allocated for FAST_MAXDENSE_ALLOC");
#define AW_CAT2(a, b) a##b
#define AW_CAT(a, b) AW_CAT2(a, b)
// the wide tier STORES up to 128 raw contacts (two 64-lane chunks) and keeps MuJoCo's nconmax of them:
// the near-margin candidates the fp64 decision drops (aw_collide.h DEC_EPS) never cost a real contact
// its slot, and past nconmax the kept ones are the first 100 in pair order, as mj_collision keeps them
constexpr int WIDE_MAXCON = 128, WIDE_NRL = 8, WIDE_MAXDENSE = 500;
constexpr int NCONMAX = 100, NJMAX = 500;   // the reference model's caps (DAPG_assets.xml:4)
#ifdef AW_WIDE
inline namespace wide {
constexpr bool WIDE = true;
constexpr int MAXCON = WIDE_MAXCON;   // contacts stored per env (64 per chunk in the lane-per-contact stages)
constexpr int CON_CAP = NCONMAX;      // contacts kept: MuJoCo's nconmax (DAPG_assets.xml:4)
constexpr int NRL = WIDE_NRL;         // constraint rows per lane in the Newton solver
constexpr int EFC_CAP = NJMAX;        // rows kept (MuJoCo's njmax), storage MAXEFC >= EFC_CAP
constexpr int MAXDENSE = WIDE_MAXDENSE;
#else
inline namespace AW_CAT(fast, AW_FAST_MD) {   // fast128 / fast192
constexpr bool WIDE = false;
constexpr int MAXCON = FAST_MAXCON;   // contacts per env (one lane each in the sort)
constexpr int CON_CAP = FAST_MAXCON;  // a raw candidate past the storage defers the env-step to the wide tier
constexpr int NRL = FAST_NRL;         // constraint rows per lane in the Newton solver
constexpr int EFC_CAP = 64 * FAST_NRL;
constexpr int MAXDENSE = FAST_MAXDENSE;  // dense (contact) rows
#endif
constexpr int MAXEFC = 64 * NRL;      // constraint rows (fast 192, wide 512)
static_assert(CON_CAP <= MAXCON, "contact storage");
constexpr int NCH = (MAXCON + 63) / 64;      // 64-contact chunks of the lane-per-contact stages
constexpr int NDCH = (MAXDENSE + 63) / 64;   // 64-row chunks of the dense rows (noslip pair scan)
constexpr int JL = 32;        // dense J rows kept in LDS; rows [JL, MAXDENSE) live in the env's global
                              // spill block (DModel::jspill), read back through L1 / L2
constexpr int JSPILL = (MAXDENSE - JL) * VS;  // floats per slot in the spill block (row stride VS)
static_assert(EFC_CAP <= MAXEFC && MAXDENSE <= EFC_CAP, "constraint capacities");
}  // inline namespace
}  // namespace aw

#ifdef AW_STAGE_PROF
extern __device__ unsigned long long g_stage_prof[];   // adroit_wave.hip (stage profiler builds)
#endif
namespace aw {
constexpr int JSPILL_FAST = (FAST_MAXDENSE_ALLOC - 32) * VS, JSPILL_WIDE = (WIDE_MAXDENSE - 32) * VS;
#ifdef AW_WIDE
#define AW_TIER wide
#else
#define AW_TIER AW_CAT(fast, AW_FAST_MD)
#endif

constexpr float MINVAL = 1e-15f;

// Stage profiler (diagnostic builds only, -DAW_STAGE_PROF): shader-clock cycles per stage,
// summed over waves; read back through aw_stage_profile().
constexpr int AW_NPROF = 44;
enum {
  PR_PRE = 0, PR_KIN, PR_COLL, PR_CRB, PR_SMOOTH, PR_CONSTR, PR_NEWTON, PR_NOSLIP, PR_JT_TOUCH,
  PR_EULER, PR_TASK, PR_RESET, PR_CHECK, PR_CALLS, PR_SUBSTEPS,
  PR_NEWTON_IT, PR_NOSLIP_IT, PR_NEFC, PR_NCON,
  PR_NT_INIT, PR_NT_HESS, PR_NT_CHOL, PR_NT_SOLVE, PR_NT_LS, PR_NT_UPD, PR_NS_MINV, PR_NS_SETUP, PR_NS_ITER,
  PR_CO_BROAD, PR_CO_NARROW, PR_COM, PR_RNE, PR_CO_C0, PR_CO_C1, PR_CO_C2, PR_CO_C3,
  PR_NT_HSPARSE, PR_NT_HOFFD, PR_NT_OFFD_ROWS, PR_CO_KIN64, PR_CS_SPARSE, PR_CS_J,
  PR_MPR_PAIRS, PR_MPR_CONTACTS   // counts: MPR pairs past the midphase, contacts they emitted
};
static_assert(PR_MPR_CONTACTS < AW_NPROF, "stage profiler ids");
// Event counts (calls, substeps, iterations, rows, contacts, MPR pairs) and the stages timed once
// per env-step or cheap (pre, task, reset, checks, plane / sphere colliders) go straight to the
// device global (lane-0 atomics); the other timed stages keep a per-env 32-bit accumulator in LDS at
// a compact slot, so the profiling build's Env stays inside the product's 20 480-byte LDS granule.
__host__ __device__ constexpr bool prof_is_count(int id) {
  return (id >= PR_CALLS && id <= PR_NCON) || id == PR_NT_OFFD_ROWS || id >= PR_MPR_PAIRS;
}
__host__ __device__ constexpr bool prof_global(int id) {
  return prof_is_count(id) || id == PR_PRE || id == PR_TASK || id == PR_RESET || id == PR_CHECK || id == PR_CO_C0 ||
         id == PR_CO_C1;
}
__host__ __device__ constexpr int prof_slot(int id) {
  int k = 0;
  for (int i = 0; i < id; i++) k += prof_global(i) ? 0 : 1;
  return k;
}
constexpr int AW_NPROF_T = prof_slot(AW_NPROF);
static_assert(AW_NPROF_T == 29, "stage profiler slots");
#ifdef AW_STAGE_PROF
#define AW_PROF_START(S)                                            \
  do {                                                              \
    unsigned _t = (unsigned)__builtin_amdgcn_s_memtime();           \
    if (threadIdx.x == 0) {                                         \
      for (int _i = 0; _i < AW_NPROF_T; _i++) (S).prof_acc[_i] = 0; \
      (S).prof_t = _t;                                              \
    }                                                               \
  } while (0)
#define AW_PROF(S, ID)                                              \
  do {                                                              \
    __syncthreads();                                                \
    unsigned _t = (unsigned)__builtin_amdgcn_s_memtime();           \
    if (threadIdx.x == 0) {                                         \
      if (prof_global(ID))                                          \
        atomicAdd(&::g_stage_prof[ID], (unsigned long long)(_t - (S).prof_t)); \
      else                                                          \
        (S).prof_acc[prof_slot(ID)] += _t - (S).prof_t;             \
      (S).prof_t = _t;                                              \
    }                                                               \
  } while (0)
#define AW_PROF_COUNT(S, ID) do { if (threadIdx.x == 0) atomicAdd(&::g_stage_prof[ID], 1ull); } while (0)
#define AW_PROF_ADD(S, ID, V) do { if (threadIdx.x == 0) atomicAdd(&::g_stage_prof[ID], (unsigned long long)(V)); } while (0)
#elif defined(AW_TRACE)   // debugging builds: every stage boundary printed by lane 0 (device printf)
#define AW_PROF_START(S) ((void)0)
#define AW_PROF(S, ID) do { if (threadIdx.x == 0) printf("wg %d stage %d\n", (int)blockIdx.x, (int)(ID)); } while (0)
#define AW_PROF_COUNT(S, ID) ((void)0)
#define AW_PROF_ADD(S, ID, V) ((void)0)
#else
#define AW_PROF_START(S) ((void)0)
#define AW_PROF(S, ID) ((void)0)
#define AW_PROF_COUNT(S, ID) ((void)0)
#define AW_PROF_ADD(S, ID, V) ((void)0)
#endif

enum { GEOM_PLANE = 0, GEOM_SPHERE = 2, GEOM_CAPSULE = 3, GEOM_CYLINDER = 5, GEOM_BOX = 6 };
enum { JNT_SLIDE = 2, JNT_HINGE = 3 };
enum { C_FRIC_DOF = 0, C_FRIC_TEN = 1, C_LIM_JNT = 2, C_LIM_TEN = 3, C_CON_FRICTIONLESS = 4, C_CON_PYRAMIDAL = 5 };
enum { S_SAT = 0, S_QUAD = 1, S_LNEG = 2, S_LPOS = 3 };

// disable bits (MuJoCo 2.1 mjtDisableBit values + ours), see include/adroit_wave.h
enum {
  DSBL_CONSTRAINT = 1 << 0, DSBL_FRICTIONLOSS = 1 << 2, DSBL_LIMIT = 1 << 3, DSBL_CONTACT = 1 << 4,
  DSBL_PASSIVE = 1 << 5, DSBL_GRAVITY = 1 << 6, DSBL_CLAMPCTRL = 1 << 7, DSBL_WARMSTART = 1 << 8,
  DSBL_ACTUATION = 1 << 10, DSBL_REFSAFE = 1 << 11, DSBL_SENSOR = 1 << 12, DSBL_NOSLIP = 1 << 14,
  DSBL_EULERDAMP = 1 << 15,
};
// ST_WIDE: the env-step (or reset / set_state forward) ran in the wide tier (informational)
enum { ST_BADQPOS = 1, ST_BADQVEL = 2, ST_BADQACC = 4, ST_CON_OVERFLOW = 8, ST_EFC_OVERFLOW = 16, ST_WIDE = 32 };

// ---------------------------------------------------------------------------------------
// Device model.  Every per-object array sits at a compile-time offset inside ONE read-only
// table (MData, fixed capacities), so a kernel holds a single uniform base pointer and each
// model read is base + constant + 32-bit lane offset.  (One pointer per array made the
// compiler keep ~100 per-lane 64-bit addresses live across a substep -- spills.)
constexpr int MAXPAIR = 320;  // explicit pairs + broadphase candidates
constexpr int MAXTIDX = 16;   // task object ids
constexpr int MAXRG = 64;     // rendered (primitive) geoms

#define AW_MODEL_ARRAYS(X)                                                                     \
  X(int, body_parentid, MAXB) X(int, body_rootid, MAXB) X(int, body_dofnum, MAXB)               \
  X(int, body_dofadr, MAXB) X(int, body_depth, MAXB) X(int, body_subtree_end, MAXB) X(int, level_start, MAXLEV + 1)      \
  X(int, level_body, MAXB) X(float, body_pos, MAXB * 3) X(float, body_quat, MAXB * 4)           \
  X(float, body_ipos, MAXB * 3) X(float, body_iquat, MAXB * 4) X(float, body_mass, MAXB)        \
  X(float, body_inertia, MAXB * 3) X(float, body_invweight0, MAXB * 2)                          \
  X(float, body_subtreemass, MAXB)                                                             \
  X(unsigned long long, body_dofmask, MAXB) /* dofs moving the body (ancestor chain) */        \
  X(int, jnt_type, MAXV) X(int, jnt_bodyid, MAXV) X(int, jnt_limited, MAXV)                     \
  X(float, jnt_pos, MAXV * 3) X(float, jnt_axis, MAXV * 3) X(float, jnt_range, MAXV * 2)        \
  X(float, jnt_margin, MAXV) X(float, jnt_solref, MAXV * 2) X(float, jnt_solimp, MAXV * 5)      \
  /* limit activation in fp64 (the reference's arithmetic): range, margin, tendon coefficients */ \
  X(double, jnt_range64, MAXV * 2) X(double, jnt_margin64, MAXV) X(double, ten_range64, MAXT * 2) \
  X(double, ten_margin64, MAXT) X(double, ten_c0_64, MAXT) X(double, ten_c1_64, MAXT)              \
  X(int, dof_bodyid, MAXV) X(int, dof_act, MAXV) /* actuator driving the dof or -1 */          \
  X(int, fl_dof, MAXV) X(int, fl_row, MAXV) /* frictionloss row r -> dof, dof -> row / -1 */   \
  X(unsigned long long, dof_ancmask, MAXV) /* strict ancestor dofs */                          \
  X(float, dof_armature, MAXV) X(float, dof_damping, MAXV) X(float, dof_frictionloss, MAXV)     \
  X(float, dof_invweight0, MAXV) X(float, dof_solref, MAXV * 2) X(float, dof_solimp, MAXV * 5)  \
  X(int, geom_type, MAXG) X(int, geom_bodyid, MAXG) X(float, geom_pos, MAXG * 3)                \
  X(float, geom_quat, MAXG * 4) X(float, geom_size, MAXG * 3) X(float, geom_rbound, MAXG)       \
  X(int, site_bodyid, MAXS) X(float, site_pos, MAXS * 3) X(float, site_quat, MAXS * 4)          \
  X(int, touch_site, MAXTOUCH) X(int, touch_adr, MAXTOUCH) X(int, touch_type, MAXTOUCH)         \
  X(float, touch_size, MAXTOUCH * 3)                                                           \
  X(int, ten_d0, MAXT) X(int, ten_d1, MAXT) X(int, ten_limited, MAXT) X(float, ten_c0, MAXT)    \
  X(float, ten_c1, MAXT) X(float, ten_range, MAXT * 2) X(float, ten_margin, MAXT)               \
  X(float, ten_solref, MAXT * 2) X(float, ten_solimp, MAXT * 5) X(float, ten_invweight0, MAXT)  \
  X(int, act_ctrllimited, MAXU) X(int, act_forcelimited, MAXU) X(float, act_gear, MAXU)         \
  X(float, act_gain, MAXU) X(float, act_bias, MAXU * 3) X(float, act_ctrlrange, MAXU * 2)       \
  X(float, act_forcerange, MAXU * 2)                                                           \
  /* explicit pairs first, then dynamic candidates; params pre-mixed on the host */           \
  X(int, cp_g1, MAXPAIR) X(int, cp_g2, MAXPAIR) X(int, cp_condim, MAXPAIR)                      \
  X(float, cp_friction, MAXPAIR * 5) X(float, cp_solref, MAXPAIR * 2)                           \
  X(float, cp_solimp, MAXPAIR * 5) X(float, cp_margin, MAXPAIR) X(float, cp_gap, MAXPAIR)       \
  /* broadphase: collider class of each pair, bounding radius sum (< 0: plane pair) */        \
  X(int, cp_class, MAXPAIR) X(float, cp_rb, MAXPAIR)                                           \
  X(int, cp_pack, MAXPAIR) /* class | g1 << 8 | g2 << 16, one load per broadphase test */     \
  /* per-pair body data for the constraint rows (one model load per contact, not a chain) */    \
  X(float, cp_tran, MAXPAIR) X(float, cp_rot, MAXPAIR) X(int, cp_root1, MAXPAIR)                \
  X(int, cp_root2, MAXPAIR) X(unsigned long long, cp_mask1, MAXPAIR)                           \
  X(unsigned long long, cp_mask2, MAXPAIR)                                                     \
  X(int, body_ovr, MAXB) X(int, site_ovr, MAXS) X(int, geom_ovr, MAXG) /* 1: overridden */    \
  X(int, task_idx, MAXTIDX) X(int, param_field, MAXP) X(int, param_obj, MAXP)                   \
  X(int, param_comp, MAXP) X(float, act_mid, MAXU) X(float, act_rng, MAXU)                      \
  X(float, param_default, MAXP) X(float, draw_lo, 8) X(float, draw_hi, 8)                      \
  X(int, param_draw, MAXP) /* reset source of each param: draw index / -1 default / -2 neck */  \
  /* depth renderer: every primitive geom (model order), its collidable index or -1 */        \
  X(int, rg_type, MAXRG) X(int, rg_body, MAXRG) X(int, rg_cgeom, MAXRG)                         \
  X(float, rg_pos, MAXRG * 3) X(float, rg_quat, MAXRG * 4) X(float, rg_size, MAXRG * 3)         \
  X(float, rg_rbound, MAXRG)                                                                   \
  /* fp64 geometry of the MPR (cylinder) pairs: the model constants of MuJoCo's fp64 kinematics */ \
  X(double, body_pos64, MAXB * 3) X(double, body_quat64, MAXB * 4) X(double, jnt_pos64, MAXV * 3) \
  X(double, jnt_axis64, MAXV * 3) X(double, geom_pos64, MAXG * 3) X(double, geom_quat64, MAXG * 4) \
  X(double, geom_size64, MAXG * 3) X(double, cp_margin64, MAXPAIR)                                 \
  X(unsigned long long, cp_kin64, MAXPAIR) /* bodies of the pair's geoms + their ancestors */

struct MData {
#define AW_X(T, name, n) T name[n];
  AW_MODEL_ARRAYS(AW_X)
#undef AW_X
};

// model read: uniform table base + zero-extended 32-bit byte offset, which maps onto the
// global_load saddr form (SGPR base, one VGPR offset) instead of a 64-bit per-lane address
// The table lives in device global memory: reading it through a global-address-space pointer
// emits global_load (vmcnt only) instead of flat_load, whose completion also holds lgkmcnt and
// so makes every LDS wait in flight behind it wait for the model read too.  The table is read-only
// for the life of a launch, so it is read through the constant address space (4): a read at a
// wave-uniform offset becomes a scalar load (no VGPR, no vmcnt), a per-lane one stays a
// global_load (A/B r03g: -1.1 % k_step against address space 1).
#ifndef AW_MD_AS
#define AW_MD_AS 4
#endif
template <class T>
AW_DEV T mld(const T* base, unsigned i) {
  typedef const __attribute__((address_space(AW_MD_AS))) T GT;
  typedef const __attribute__((address_space(AW_MD_AS))) char GC;
  return *(GT*)((GC*)base + i * (unsigned)sizeof(T));
}
#define MD(name, idx) ::aw::mld(m.d->name, (unsigned)(idx))
// device-global views of model / state arrays (global_load / global_store, not flat)
template <class T> using gp_t = __attribute__((address_space(1))) T*;
template <class T> AW_DEV gp_t<const T> gcp(const T* p) { return (gp_t<const T>)p; }
template <class T> AW_DEV gp_t<T> gmp(T* p) { return (gp_t<T>)p; }
#define MDP(name, idx) ::aw::gcp(&m.d->name[idx])

struct DModel {
  int nq, nv, nu, nbody, njnt, ngeom, nsite, ntendon, npairall, nlevel;
  int nfl;                // dofs with frictionloss (rows 0..nfl-1 are these, in dof order)
  int ntouch;
  int ndraw;              // reset uniform draws
  int task_kind, frame_skip, horizon, obs_dim, nparam, variation;
  int success_steps;      // evaluate_success: an episode succeeds with > success_steps goal steps
  int iterations, noslip_iterations, mpr_iterations, disableflags;
  float timestep, gravity[3], tolerance, noslip_tolerance, mpr_tolerance, meaninertia;
  float pen_length, tar_length;
  double mpr_tolerance64;
  int cls_start[NCLASS + 1];  // collider class c owns pair-list slots [cls_start[c], cls_start[c+1])
  int nrgeom;                 // rendered geoms
  int force_wide;             // test hook (aw_set_tier): every forward of the fast tier defers to the wide tier
  int fault_flrow;            // test hook (aw_set_fault, kind 2): this frictionloss row never slides; -1: off
  const MData* __restrict__ d;
  float* jspill;              // dense-J rows past JL, one block of the tier's JSPILL floats per workgroup slot (device)
  unsigned long long env_offset;   // global id of env 0 of this handle (shards): Philox keys
};

// ---------------------------------------------------------------------------------------
// Per-env working set in LDS (one wave per workgroup, one env per wave).  Sized to stay under
// 20 KiB so EIGHT envs share a CU (two waves per SIMD: the second wave issues while the first
// waits on LDS / L1, and VALU issue doubles from one-per-4-cycles to one-per-2).  Storage is
// overlaid by liveness within a substep:
//   persistent   state, body / site frames read by the task layer, per-env overrides
//   contacts     collision -> touch sensor
//   rows         constraint rows + dense contact Jacobian: constraints -> end of forward
//   phase K      kinematics / com / RNE / CRB temporaries, dead once the Jacobian exists
//   phase S      packed Cholesky factor and solver vectors (smooth solve, Newton, noslip, Euler)
// dof vectors with only lane-local use (qacc, qacc_smooth, qfrc_smooth, qfrc_con) are VGPRs.
// packed lower triangle with every row padded to a multiple of 4 floats: row j starts at a
// 16-byte aligned tri(j), so uniform reads along a row are ds_read_b128 broadcasts
__host__ __device__ constexpr int tri(int j) { return 4 * (j + 2 * (j / 4) * (j / 4 - 1) + (j % 4) * (j / 4)); }
constexpr int NPACK = tri(MAXV);

inline namespace AW_TIER {   // Env-dependent definitions: per capacity tier
struct __attribute__((aligned(16))) Env {
  union {
    struct {  // phase K
      float xipos[MAXB][3], subcom[MAXB][3];
      float cinert[MAXB][10];   // cinert; overwritten in place by crb once RNE is done
      float cdof[MAXV][6];
      union {
        struct { float gxpos[MAXG][3], gxquat[MAXG][4], xaxis[MAXV][3], xanchor[MAXV][3]; };  // kin -> com
        struct { float cvel[MAXB][6], cacc[MAXB][6]; };                                      // RNE
        float buf[MAXV][6];                                                                   // CRB
      };
    };
    struct {  // phase S
      float4 colbuf[MAXV];    // Cholesky panel broadcast: row k's U_k,j0..j0+3 (b128 reads)
      float L[NPACK];         // Cholesky factor, packed lower triangle (rows padded to 4)
      float vec[MAXV], vec2[MAXV], hdiag[MAXV];
    };
  };
  // persistent
  float qpos[MAXV], qvel[MAXV], warm[MAXV], ctrl[MAXV];
  float qlo[MAXV];          // qpos = qpos + qlo inside an env-step (mj_Euler's fp64 position sum; 0 at its start)
  float xpos[MAXB][3], xquat[MAXB][4];
  float sxpos[MAXS][3];
  float txmat[MAXTOUCH][9];
  float gsize[MAXG][3];     // per-env copy (overridable, read by every collider)
  float bmass[MAXB];        // per-env copy (overridable, subtree sums)
  float prm[MAXP];          // this env's model parameters
  float touch[MAXTOUCH];
  // contacts (normal only: the tangent frame is rebuilt where it is used)
  int ncon;
  int con_key[MAXCON], con_pair[MAXCON], con_efc[MAXCON];
  float con_dist[MAXCON], con_pos[MAXCON][3], con_nrm[MAXCON][3];
  // constraint rows: [0, nsparse) sparse (<= 2 nonzeros), [nsparse, nefc) dense (J rows)
  int nefc, nsparse, ndense;
  unsigned char efc_type[MAXEFC], efc_id[MAXEFC];
  signed char efc_i0[MAXEFC], efc_i1[MAXEFC];
  float efc_v0[MAXEFC], efc_v1[MAXEFC], efc_floss[MAXEFC], efc_D[MAXEFC];
  float efc_aref[MAXEFC], efc_force[MAXEFC];
  float J[JL][VS] __attribute__((aligned(16)));
  float rowbuf[MAXEFC];
  unsigned status;
  unsigned long long kin64_mask;   // bodies whose fp64 frames this substep's MPR pairs read
  int slot;                   // workgroup slot: selects the dense-J spill and M-factor blocks,
                              // reused by every env the persistent k_step workgroup processes
  int it_newton, it_noslip;   // iterations of the last solve (introspection)
#ifdef AW_STAGE_PROF
  // 32-bit: one env-step's cycles per stage (summed into 64-bit globals after each env-step); keeps
  // the profiling build's Env inside k_step's 20 480-byte LDS granule, i.e. at the product's occupancy
  unsigned prof_acc[AW_NPROF_T];
  unsigned prof_t;
#endif
};

// The persistent arrays start on 16-byte boundaries.  A layout that put them at 8 mod 16 (ctrl sized
// by MAXU, r06 bisection: tools/diag_tiers.py) made the fast and the wide tier diverge bitwise in
// hammer's free-object dofs after a few env-steps -- an alignment-phase dependence not root-caused
// (DESIGN.md §7); held here so no layout change reintroduces it unnoticed.
static_assert(offsetof(Env, xpos) % 16 == 0 && offsetof(Env, xquat) % 16 == 0 && offsetof(Env, gsize) % 16 == 0,
              "persistent Env arrays must keep their 16-byte alignment phase");
// fp64 body frames of the MPR (cylinder) geometry, stage_kin64 -> narrowphase: [MAXB][8] doubles
// (xpos[3], xquat[4], pad) in the dense-J storage, dead from kinematics until the constraint rows;
// its first MAXPAIR shorts hold the broadphase pair list
constexpr int KIN64_OFF = MAXPAIR * 2;
static_assert(KIN64_OFF % 16 == 0 && KIN64_OFF + MAXB * 8 * 8 <= JL * VS * 4, "fp64 frames do not fit in the dense-J rows");
// joint position j in fp64: the env-step's compensated sum qpos + qlo (the fp64 consumers: frames of
// the MPR / near-margin contact decisions, joint and tendon limit activation)
// AW_QPOS_COMP (default 0): carry qpos + qlo across the substeps (adroit_wave.hip euler).  Measured
// r06x / r06z: DAPG headline misses 41 -> 13 of 20 480 (0.99937); off by default because one relocate
// config-3 wide-tier env-step then meets a capsule-box point choice the classifier cannot yet prove a
// tie.
#ifndef AW_QPOS_COMP
#define AW_QPOS_COMP 0
#endif
AW_DEV double qpos64(const Env& s, int j) {
#if AW_QPOS_COMP
  return (double)s.qpos[j] + (double)s.qlo[j];
#else
  return (double)s.qpos[j];
#endif
}
AW_DEV double* kin64(Env& s, int b) {
  return reinterpret_cast<double*>(reinterpret_cast<char*>(&s.J[0][0]) + KIN64_OFF) + 8 * b;
}
// joint j's record for stage_kin64 (half-angle sin / cos, axis, kind), after the frames
constexpr int KIN64_SC_OFF = KIN64_OFF + MAXB * 8 * 8;
constexpr int KIN64_SC_W = 6;   // doubles per joint record: sin, cos (hinges), axis, kind
static_assert(KIN64_SC_OFF + MAXV * KIN64_SC_W * 8 <= JL * VS * 4, "fp64 joint records do not fit in the dense-J rows");
AW_DEV double* kin64_sc(Env& s, int j) {
  return reinterpret_cast<double*>(reinterpret_cast<char*>(&s.J[0][0]) + KIN64_SC_OFF) + KIN64_SC_W * j;
}

}  // inline namespace AW_TIER

// ---------------------------------------------------------------------------------------
// wave primitives
AW_DEV float rlane(float x, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}
AW_DEV int rlane_i(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
// b in lane l, a in the other lanes: v_cndmask against the constant lane mask 1 << l (an SGPR
// constant, no v_cmp); l must be a compile-time constant after unrolling
AW_DEV float sel_lane(float a, float b, int l) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(1ull << l));
  return r;
}
// An opaque copy of a lane-dependent value: values derived from it cannot be hoisted above this
// point (out of the substep loop) to sit in registers across every stage.
AW_DEV int opaque(int x) {
  int y;
  asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
  return y;
}
AW_DEV float opaque(float x) {
  float y;
  asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
  return y;
}
// Intra-wave LDS hand-off.  Every workgroup is exactly one wave64: LDS operations of a wave
// execute in issue order, so cross-lane communication through LDS needs only a compiler-level
// ordering point, not s_barrier + a full s_waitcnt drain (which would serialise every
// outstanding load at each hand-off).  A wavefront-scope fence emits no instruction.
AW_DEV void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// DPP butterfly reductions (VALU only: no LDS round trip as __shfl_xor / ds_bpermute would
// take).  quad_perm [1,0,3,2] and [2,3,0,1], row_half_mirror and row_mirror leave every lane of
// a 16-lane row holding the row total; row_bcast15 (rows 1,3) and row_bcast31 (rows 2,3) fold
// the rows so lane 63 holds the wave total, which readlane broadcasts (uniform result).
template <int CTRL, int ROWMASK = 0xF>
AW_DEV float dpp_f(float old, float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old),
                                                               __builtin_bit_cast(int, x), CTRL, ROWMASK, 0xF, false));
}
AW_DEV float wave_sum(float x) {
  x += dpp_f<0xB1>(0.f, x);
  x += dpp_f<0x4E>(0.f, x);
  x += dpp_f<0x141>(0.f, x);
  x += dpp_f<0x140>(0.f, x);
  x += dpp_f<0x142, 0xA>(0.f, x);
  x += dpp_f<0x143, 0xC>(0.f, x);
  return rlane(x, 63);
}
AW_DEV float wave_max(float x) {
  constexpr float NEG = -3.402823466e38f;
  x = fmaxf(x, dpp_f<0xB1>(NEG, x));
  x = fmaxf(x, dpp_f<0x4E>(NEG, x));
  x = fmaxf(x, dpp_f<0x141>(NEG, x));
  x = fmaxf(x, dpp_f<0x140>(NEG, x));
  x = fmaxf(x, dpp_f<0x142, 0xA>(NEG, x));
  x = fmaxf(x, dpp_f<0x143, 0xC>(NEG, x));
  return rlane(x, 63);
}
// exclusive prefix sum of small non-negative ints (< 2^BITS) across the wave, bit-sliced: one
// ballot + popcount per bit (scalar work), no lane shuffles through the LDS crossbar
template <int BITS>
AW_DEV int wave_excl_scan(int x, int lane, int* total) {
  const unsigned long long below = (1ull << lane) - 1ull;
  int pre = 0, tot = 0;
#pragma unroll
  for (int b = 0; b < BITS; b++) {
    const unsigned long long mk = __ballot((x >> b) & 1);
    pre += __popcll(mk & below) << b;
    tot += __popcll(mk) << b;
  }
  *total = tot;
  return pre;
}

// ---------------------------------------------------------------------------------------
// fp32 3D helpers
AW_DEV float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
AW_DEV void cross3(float* r, const float* a, const float* b) {
  float t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
AW_DEV void sub3(float* r, const float* a, const float* b) { r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2]; }
AW_DEV void add3(float* r, const float* a, const float* b) { r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2]; }
AW_DEV void scl3(float* r, const float* a, float s) { r[0] = a[0] * s; r[1] = a[1] * s; r[2] = a[2] * s; }
AW_DEV void copy3(float* r, const float* a) { r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; }
AW_DEV float norm3(const float* a) { return sqrtf(dot3(a, a)); }
AW_DEV float normalize3(float* a) {
  float n = norm3(a);
  if (n < MINVAL) { a[0] = 1; a[1] = 0; a[2] = 0; return n; }
  float in = 1.0f / n;
  a[0] *= in; a[1] *= in; a[2] *= in;
  return n;
}
AW_DEV void mulmv3(float* r, const float* m, const float* v) {
  float t0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  float t1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  float t2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
AW_DEV void mulmtv3(float* r, const float* m, const float* v) {
  float t0 = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  float t1 = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  float t2 = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
AW_DEV void mulq(float* r, const float* a, const float* b) {
  float t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  float t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  float t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  float t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
AW_DEV void rotvq(float* r, const float* v, const float* q) {
  float u[3] = {q[1], q[2], q[3]}, t[3], t2[3];
  cross3(t, u, v);
  scl3(t, t, 2.0f);
  cross3(t2, u, t);
  r[0] = v[0] + q[0] * t[0] + t2[0];
  r[1] = v[1] + q[0] * t[1] + t2[1];
  r[2] = v[2] + q[0] * t[2] + t2[2];
}
AW_DEV void q2m(float* m, const float* q) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = 1 - 2 * (x * x + y * y);
}
AW_DEV void normq(float* q) {
  float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  float in = 1.0f / n;
  q[0] *= in; q[1] *= in; q[2] *= in; q[3] *= in;
}
AW_DEV float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

// fp64 overloads of the 3D helpers (MPR runs in double: aw_collide.h)
AW_DEV double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
AW_DEV void cross3(double* r, const double* a, const double* b) {
  double t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
AW_DEV void sub3(double* r, const double* a, const double* b) { r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2]; }
AW_DEV void add3(double* r, const double* a, const double* b) { r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2]; }
AW_DEV void scl3(double* r, const double* a, double s) { r[0] = a[0] * s; r[1] = a[1] * s; r[2] = a[2] * s; }
AW_DEV void copy3(double* r, const double* a) { r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; }
AW_DEV void mulmv3(double* r, const double* m, const double* v) {
  double t0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  double t1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  double t2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
AW_DEV void mulmtv3(double* r, const double* m, const double* v) {
  double t0 = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  double t1 = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  double t2 = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}

AW_DEV void mulq(double* r, const double* a, const double* b) {
  double t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  double t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  double t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  double t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
AW_DEV void rotvq(double* r, const double* v, const double* q) {
  double u[3] = {q[1], q[2], q[3]}, t[3], t2[3];
  cross3(t, u, v);
  scl3(t, t, 2.0);
  cross3(t2, u, t);
  r[0] = v[0] + q[0] * t[0] + t2[0];
  r[1] = v[1] + q[0] * t[1] + t2[1];
  r[2] = v[2] + q[0] * t[2] + t2[2];
}
AW_DEV void q2m(double* m, const double* q) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = 1 - 2 * (y * y + z * z); m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = 1 - 2 * (x * x + z * z); m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = 1 - 2 * (x * x + y * y);
}

// mju_makeFrame
AW_DEV void make_frame(float* f) {
  normalize3(f);
  if (norm3(f + 3) < 0.5f) {
    if (fabsf(f[1]) < 0.5f) { f[3] = 0; f[4] = 1; f[5] = 0; }
    else { f[3] = 0; f[4] = 0; f[5] = 1; }
  }
  float d = dot3(f, f + 3);
  f[3] -= d * f[0]; f[4] -= d * f[1]; f[5] -= d * f[2];
  normalize3(f + 3);
  cross3(f + 6, f, f + 3);
}

// spatial algebra, MuJoCo layout (motion = [ang; lin]; cinert = [Ixx Iyy Izz Ixy Ixz Iyz mc m])
AW_DEV void mul_inert_vec(float* r, const float* i, const float* v) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
AW_DEV void cross_motion(float* r, const float* v, const float* u) {
  float t[6];
  t[0] = -v[2] * u[1] + v[1] * u[2];
  t[1] = v[2] * u[0] - v[0] * u[2];
  t[2] = -v[1] * u[0] + v[0] * u[1];
  t[3] = -v[2] * u[4] + v[1] * u[5] - v[5] * u[1] + v[4] * u[2];
  t[4] = v[2] * u[3] - v[0] * u[5] + v[5] * u[0] - v[3] * u[2];
  t[5] = -v[1] * u[3] + v[0] * u[4] - v[4] * u[0] + v[3] * u[1];
#pragma unroll
  for (int k = 0; k < 6; k++) r[k] = t[k];
}
AW_DEV void cross_force(float* r, const float* v, const float* f) {
  float t[6];
  t[0] = -v[2] * f[1] + v[1] * f[2] - v[5] * f[4] + v[4] * f[5];
  t[1] = v[2] * f[0] - v[0] * f[2] + v[5] * f[3] - v[3] * f[5];
  t[2] = -v[1] * f[0] + v[0] * f[1] - v[4] * f[3] + v[3] * f[4];
  t[3] = -v[2] * f[4] + v[1] * f[5];
  t[4] = v[2] * f[3] - v[0] * f[5];
  t[5] = -v[1] * f[3] + v[0] * f[4];
#pragma unroll
  for (int k = 0; k < 6; k++) r[k] = t[k];
}
AW_DEV float dot6(const float* a, const float* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

}  // namespace aw
