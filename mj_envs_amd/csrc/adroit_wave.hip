// adroit_wave.hip -- MI355X batched Adroit simulator: kernels + C-ABI (include/adroit_wave.h).
//
// One workgroup = one 64-lane wave = one env.  A step launch runs frame_skip x mj_step
// (forward + Euler) and the task layer for every env; the per-env working set stays in LDS /
// VGPRs for the whole launch, so HBM traffic is the compulsory state + action + obs bytes.
//
// Build split (__graft_entry__.py): the library is this file compiled five times in parallel and
// linked -- once per task with -DAW_TASK_TU=<task> (that task's kernels and its launcher table,
// task_ops<TASK>) and once with -DAW_API_TU (the C-ABI and the task-independent kernels, no
// per-task instantiation).  A plain compile of the file (diagnostic builds: -DAW_ONLY_TASK,
// -DAW_STAGE_PROF) is the whole library in one translation unit.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/adroit_wave.h"
#include "../../include/aw_blob.h"
#include "aw_collide.h"
#include "aw_common.h"
#include "aw_dynamics.h"
#include "aw_render.h"
#ifndef AW_TASK_TU
#include "aw_policy.h"
#endif
#include "aw_solver.h"
#include "aw_task.h"
#include "aw_tree.h"

using namespace aw;

// k_step is allocated for two waves per SIMD (<= 256 VGPRs): its LDS footprint (< 20 KiB)
// already admits 8 envs per CU, and the register allocator left alone would take 350+
#ifndef AW_KSTEP_ATTR
#define AW_KSTEP_ATTR __attribute__((amdgpu_waves_per_eu(2, 2)))
#endif

#ifdef AW_STAGE_PROF
#if defined(AW_TASK_TU) || defined(AW_API_TU)
#error "the stage profiler counts into one device global: build it as a single translation unit"
#endif
__device__ unsigned long long g_stage_prof[AW_NPROF];
#endif
#ifndef AW_ENV_LANE
// opaque env-level lane ids: per-lane state / obs addresses are formed where they are used, not
// once per env and spilled.  With the env index scalar (readfirstlane claim) this takes k_step's
// scratch 280 -> 92 B/lane and its HBM traffic 7.9 -> 1.7 KB per env-step, +1.7 % (DAPG +2.1 %,
// A/B r03za); -DAW_ENV_LANE= (plain lane ids) restores the old form.
#define AW_ENV_LANE(x) opaque(x)
#endif

// ---------------------------------------------------------------------------------------
// device-side state owned by the handle
struct DState {
  float* qpos; float* qvel; float* warm; float* params;
  int* ep_len; float* ep_ret; int* ep_goal; int* episode; unsigned* status;
  float* last_ret; int* last_goal; int* last_len;
  unsigned* status_acc;   // OR of every step's flags since create / aw_clear_status (sticky)
  float* sum_ret;         // sum of the returns of every finished episode
  int* n_success;         // finished episodes with > success_steps goal steps (evaluate_success)
};

// ---------------------------------------------------------------------------------------
// contacts -> (pair, emission) key order: rank of each key among the n keys (keys are unique),
// then a scatter to that slot; normals are normalised on the way
AW_DEV void sort_contacts(Env& s, int lane) {
  int n = s.ncon;
  if (n > MAXCON) n = MAXCON;
  // lane = contact, in chunks of 64 (the wide tier's 100 contacts take two)
  int key[NCH], rank[NCH], pair[NCH];
  float dist[NCH], pos[NCH][3], nrm[NCH][3];
#pragma unroll
  for (int h = 0; h < NCH; h++) {
    const int c = lane + 64 * h;
    key[h] = c < n ? s.con_key[c] : 0x7fffffff;
    rank[h] = 0;
  }
  if constexpr (NCH == 1) {
    for (int j = 0; j < n; j++) rank[0] += rlane_i(key[0], j) < key[0] ? 1 : 0;
  } else {
    for (int j = 0; j < n; j++) {
      const int kj = s.con_key[j];
#pragma unroll
      for (int h = 0; h < NCH; h++) rank[h] += kj < key[h] ? 1 : 0;
    }
  }
#pragma unroll
  for (int h = 0; h < NCH; h++) {
    const int c = lane + 64 * h;
    dist[h] = 0.f;
    pair[h] = 0;
    for (int k = 0; k < 3; k++) pos[h][k] = nrm[h][k] = 0.f;
    if (c < n) {
      dist[h] = s.con_dist[c];
      pair[h] = s.con_pair[c];
      for (int k = 0; k < 3; k++) { pos[h][k] = s.con_pos[c][k]; nrm[h][k] = s.con_nrm[c][k]; }
    }
  }
  wsync();
#pragma unroll
  for (int h = 0; h < NCH; h++) {
    if (lane + 64 * h < n) {
      const int r = rank[h];
      s.con_key[r] = key[h];
      s.con_dist[r] = dist[h];
      s.con_pair[r] = pair[h];
      copy3(s.con_pos[r], pos[h]);
      normalize3(nrm[h]);         // mju_makeFrame's first step; tangents are rebuilt where used
      copy3(s.con_nrm[r], nrm[h]);
    }
  }
  if (lane == 0) {
    s.ncon = n - (int)s.kin64_mask;   // fp64-dropped candidates sorted last (stage_collision)
    // the wide tier's nconmax applies to the decided contacts, in pair order (mj_collision)
    if (s.ncon > CON_CAP) { s.ncon = CON_CAP; s.status |= ST_CON_OVERFLOW; }
  }
  wsync();
}

// Midphase of collider class C (2, 3, 4), lane per pair: a pair whose geoms provably stay farther
// apart than margin + 1e-4 (aw_collide.h *_may_touch: exact lower bounds on the distance) emits
// nothing in its collider either and is dropped; the survivors are compacted in place at the
// front of the class's slice of the list.  Returns their count.
template <int C>
AW_DEV int midphase(const DModel& m, Env& s, short* list, int cnt, int lane) {
  int nsurv = 0;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int base = 0; base < cnt; base += 64) {
    const int i = base + lane;
    const int pair = i < cnt ? list[i] : 0;
    bool keep = false;
    if (i < cnt) {
      if constexpr (C == 2) keep = capbox_may_touch(m, s, pair);
      else if constexpr (C == 3) keep = boxbox_may_touch(m, s, pair);
      else keep = mpr_may_touch(m, s, pair);
    }
    const unsigned long long mask = __ballot(keep);
    wsync();
    if (keep) list[nsurv + __popcll(mask & below)] = (short)pair;
    nsurv += __popcll(mask);
    wsync();
  }
  return nsurv;
}

// narrowphase over the broadphase survivors of one collider class
template <int C>
AW_DEV void narrow_class(const DModel& m, Env& s, const short* plist, int cnt, int lane) {
  const int st = m.cls_start[C];
  if constexpr (C == 2) {
    // sphere / capsule - box: midphase, then one survivor per 16-lane DPP row, four per round
    // (capsule-box's 43-candidate minimiser search is spread over the row, capbox_tstar_row)
    short* list = const_cast<short*>(plist) + st;
    const int nsurv = midphase<C>(m, s, list, cnt, lane);
    for (int i0 = 0; i0 < nsurv; i0 += 4) {
      const int i = i0 + (lane >> 4);
      if (i < nsurv) collide_pair<C>(m, s, list[i], lane & 15);
    }
  } else if constexpr (C == 3) {
    short* list = const_cast<short*>(plist) + st;
    const int nsurv = midphase<C>(m, s, list, cnt, lane);
    for (int i = lane; i < nsurv; i += 64) collide_pair<C>(m, s, list[i]);
  } else if constexpr (C == 4) {
    // MPR: two lanes per pair (aw_collide.h swap_pair), 32 pairs per round
    for (int i0 = 0; i0 < cnt; i0 += 32) {
      const int i = i0 + (lane >> 1);
      if (i < cnt) collide_pair<C>(m, s, plist[st + i], lane & 1);
    }
  } else {
    for (int i = lane; i < cnt; i += 64) collide_pair<C>(m, s, plist[st + i]);
  }
}

// mj_collision: bounding-sphere broadphase over the static candidate list (one pair per lane,
// 64 per round), survivors compacted class-major into an LDS list (ballot + mbcnt), then ONE
// narrowphase loop over the list: lanes of a round mostly share a collider, instead of every
// round executing every collider branch its lanes happen to need.  MPR pairs (class 4) run on
// fp64 geometry: stage_kin64 computes their bodies' frames once the broadphase has kept one.
AW_DEV void stage_collision(const DModel& m, Env& s, int lane) {
  if (lane == 0) s.ncon = 0;
  wsync();
  if (!(m.disableflags & (DSBL_CONSTRAINT | DSBL_CONTACT))) {
    short* plist = reinterpret_cast<short*>(&s.J[0][0]);   // dense J rows are dead until stage_constraints
    int cnt[NCLASS];
#pragma unroll
    for (int c = 0; c < NCLASS; c++) cnt[c] = 0;
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int base = 0; base < m.npairall; base += 64) {   // rounds of 64 pairs
      const int p = base + lane;
      bool pass = false;
      int cls = -1;
      if (p < m.npairall) {
        const int pk = MD(cp_pack, p);
        const float rb = MD(cp_rb, p);
        cls = pk & 0xff;
        const int g1 = (pk >> 8) & 0xff, g2 = pk >> 16;
        float dif[3];
        sub3(dif, s.gxpos[g2], s.gxpos[g1]);
        if (rb < 0.f) {
          // plane (g1) pair: the other geom's bounding sphere against the plane through the plane
          // geom's centre, normal = its z axis (every plane collider emits only within the margin)
          const float* q = s.gxquat[g1];
          const float n[3] = {2.f * (q[1] * q[3] + q[0] * q[2]), 2.f * (q[2] * q[3] - q[0] * q[1]),
                              1.f - 2.f * (q[1] * q[1] + q[2] * q[2])};
          pass = !(dot3(n, dif) > -rb - 1.f + 1e-4f);
        } else {
          pass = !(dot3(dif, dif) > rb * rb);
        }
      }
#pragma unroll
      for (int c = 0; c < NCLASS; c++) {
        const bool mine = pass && cls == c;
        const unsigned long long mask = __ballot(mine);
        if (mine) plist[m.cls_start[c] + cnt[c] + __popcll(mask & below)] = (short)p;
        cnt[c] += __popcll(mask);
      }
    }
    AW_PROF(s, PR_CO_BROAD);
    wsync();
    narrow_class<0>(m, s, plist, cnt[0], lane);
    AW_PROF(s, PR_CO_C0);
    narrow_class<1>(m, s, plist, cnt[1], lane);
    AW_PROF(s, PR_CO_C1);
    narrow_class<2>(m, s, plist, cnt[2], lane);
    AW_PROF(s, PR_CO_C2);
    narrow_class<3>(m, s, plist, cnt[3], lane);
    AW_PROF(s, PR_CO_C3);
    // contacts of the sphere / capsule classes within DEC_EPS of their margin (aw_collide.h): their
    // activation is decided in fp64 below, so their bodies' fp64 frames are staged with the MPR ones
    wsync();
    const int nc0 = s.ncon < MAXCON ? s.ncon : MAXCON;
    unsigned long long km = 0ull;
    bool und[NCH];
#pragma unroll
    for (int h = 0; h < NCH; h++) {
      const int c = lane + 64 * h;
      und[h] = false;
      if (c < nc0) {
        const int pr = s.con_pair[c];
        const int cls = MD(cp_pack, pr) & 0xff;
        und[h] = (cls == 1 || cls == 2) && fabsf(s.con_dist[c] - MD(cp_margin, pr)) <= DEC_EPS;
        if (und[h]) km |= MD(cp_kin64, pr);
      }
    }
    // MPR (cylinder) pairs: the midphase first (fp32 frames, exact distance lower bounds), so
    // that only pairs that can touch request fp64 frames and run fp64 MPR (hammer: the upright
    // wall's bounding sphere covers the scene, 5 of its 6 broadphase survivors never touch)
    if (cnt[4] > 0) cnt[4] = midphase<4>(m, s, plist + m.cls_start[4], cnt[4], lane);
    // the surviving MPR pairs' body closures: only those frames are computed in fp64
    for (int i = lane; i < cnt[4]; i += 64) km |= MD(cp_kin64, plist[m.cls_start[4] + i]);
    if (__ballot(km != 0ull)) {
      if (lane == 0) s.kin64_mask = 0ull;
      wsync();
      if (km) atomicOr(&s.kin64_mask, km);
      wsync();
      stage_kin64(m, s, lane);
      AW_PROF(s, PR_CO_KIN64);
#ifdef AW_STAGE_PROF
      const int nc_before = s.ncon;
      AW_PROF_ADD(s, PR_MPR_PAIRS, cnt[4]);
#endif
      if (cnt[4] > 0) narrow_class<4>(m, s, plist, cnt[4], lane);
#ifdef AW_STAGE_PROF
      wsync();
      AW_PROF_ADD(s, PR_MPR_CONTACTS, s.ncon - nc_before);
#endif
      // fp64 activation: drop a candidate beyond its margin (its key moves past every valid key, so
      // the sort puts it last and cuts it), keep the others with their fp64 distance
      int ndrop = 0;
#pragma unroll
      for (int h = 0; h < NCH; h++) {
        const int c = lane + 64 * h;
        bool drop = false;
        if (und[h]) {
          const double d64 = contact_dist64(m, s, c);
          drop = d64 > MD(cp_margin64, s.con_pair[c]);
          if (drop) s.con_key[c] = 0x7fff0000 + c;
          else s.con_dist[c] = (float)d64;
        }
        ndrop += __popcll(__ballot(drop));
      }
      if (lane == 0) s.kin64_mask = (unsigned long long)ndrop;   // handed to the sort (frames are dead)
    } else if (lane == 0) {
      s.kin64_mask = 0ull;
    }
  } else if (lane == 0) {
    s.kin64_mask = 0ull;
  }
  wsync();
  AW_PROF(s, PR_CO_NARROW);
  sort_contacts(s, lane);
}

// lane-local dof vectors of a forward pass (VGPRs; lane = dof)
struct Dof {
  float qacc, qacc_smooth, qfrc_smooth, qfrc_con;
};

// mj_forward: everything up to qacc / forces / sensors; Mrow is left in registers.  Stage order
// follows the LDS overlays (aw_common.h Env): the constraint rows are assembled while the
// phase-K arrays (cdof, subcom) are alive, then the solver phase reuses that storage.
// ROWST (aw_forward_dump only): the Newton solve's final row states (S_*) go to rowst[r]
template <int TASK, bool ROWST = false>
AW_DEV void forward(const DModel& m, Env& s, int lane, float (&Mrow)[Tree<TASK>::NV], Dof& d, float* rowst = nullptr) {
  constexpr int NV = Tree<TASK>::NV;
  stage_kinematics(m, s, lane);
  AW_PROF(s, PR_KIN);
  stage_collision(m, s, lane);
  AW_PROF(s, PR_COLL);
  stage_com(m, s, lane);
  AW_PROF(s, PR_COM);
  d.qfrc_smooth = stage_velocity(m, s, lane);
  AW_PROF(s, PR_RNE);
  stage_crb<NV>(m, s, lane, Mrow);
  AW_PROF(s, PR_CRB);
  if (lane == 0) { s.it_newton = 1000 * NT_EXIT_NOROWS; s.it_noslip = 0; }
  stage_constraints<NV>(m, s, lane);
  AW_PROF(s, PR_CONSTR);
  // qacc_smooth = M \ qfrc_smooth: mj_factorM + mj_solveM over the dof tree (aw_tree.h)
  {
    float row[NV];
#pragma unroll
    for (int k = 0; k < NV; k++) row[k] = Mrow[k];
    float invd;
    tree_factor<TASK>(row, invd, lane);
    d.qacc_smooth = tree_solve<TASK>(row, invd, d.qfrc_smooth, lane);
  }
  AW_PROF(s, PR_SMOOTH);
  if (s.nefc == 0) {
    d.qacc = d.qacc_smooth;
    d.qfrc_con = 0.f;
  } else {
    float a = 0.f;
    solve_newton<NV, ROWST>(m, s, lane, Mrow, a, d.qfrc_smooth, d.qacc_smooth, rowst);
    AW_PROF(s, PR_NEWTON);
    if (m.noslip_iterations > 0 && !(m.disableflags & DSBL_NOSLIP)) solve_noslip<TASK>(m, s, lane, Mrow, a);
    AW_PROF(s, PR_NOSLIP);
    for (int r = lane; r < s.nefc; r += 64) s.rowbuf[r] = s.efc_force[r];
    wsync();
    float qc = jt_mul<NV>(m, s, lane);
    d.qacc = lane < NV ? a : 0.f;
    d.qfrc_con = lane < NV ? qc : 0.f;
  }
  stage_touch(m, s, lane);
  AW_PROF(s, PR_JT_TOUCH);
}

// mj_Euler: implicit joint damping (M + h D factored over the dof tree, aw_tree.h),
// semi-implicit positions, warmstart <- qacc
template <int TASK>
AW_DEV void euler(const DModel& m, Env& s, int lane, const float (&Mrow)[Tree<TASK>::NV], const Dof& d) {
  constexpr int NV = Tree<TASK>::NV;
  const float h = m.timestep;
  const bool dmp = !(m.disableflags & (DSBL_EULERDAMP | DSBL_PASSIVE));
  float acc;
  if (dmp) {
    float row[NV];
    const float dd = lane < NV ? h * MD(dof_damping, lane) : 0.f;
#pragma unroll
    for (int k = 0; k < NV; k++) row[k] = Mrow[k] + (k == lane ? dd : 0.f);
    float invd;
    tree_factor<TASK>(row, invd, lane);
    acc = tree_solve<TASK>(row, invd, d.qfrc_smooth + d.qfrc_con, lane);
  } else {
    acc = d.qacc;
  }
  if (lane < NV) {
    float v = s.qvel[lane] + h * acc;
    s.qvel[lane] = v;
#if AW_QPOS_COMP
    // qpos += h v as MuJoCo's fp64 sum: qpos + qlo carries the position to ~2^-48 relative across the
    // env-step's substeps (TwoProduct of h v, TwoSum into qpos, renormalised), so the fp64 consumers
    // (qpos64) see the reference's positions at substeps 2.. instead of a rounding per substep
    const float q = s.qpos[lane], p = h * v, pe = fmaf(h, v, -p);
    const float sm = q + p, bb = sm - q, e = (q - (sm - bb)) + (p - bb);
    const float lo = s.qlo[lane] + (pe + e), hi = sm + lo;
    s.qpos[lane] = hi;
    s.qlo[lane] = lo - (hi - sm);
#else
    s.qpos[lane] += h * v;
#endif
    s.warm[lane] = d.qacc;
  }
  wsync();
}

// mj_resetData on the state: qpos0 (= 0 for these models), qvel, warmstart and ctrl zeroed --
// after a bad-state reset inside an env-step, the remaining substeps run with ctrl = 0, as the
// reference's do_simulation writes ctrl once before its frame_skip mj_step calls
template <int NV>
AW_DEV void reset_state(Env& s, int lane) {
  if (lane < NV) { s.qpos[lane] = 0.f; s.qlo[lane] = 0.f; s.qvel[lane] = 0.f; s.warm[lane] = 0.f; s.ctrl[lane] = 0.f; }
  wsync();
}

AW_DEV bool bad_value(float x) { return !(fabsf(x) <= 1e10f); }

// mj_checkPos / mj_checkVel: bad state -> flag + reset to qpos0 / 0
template <int NV>
AW_DEV void check_state(Env& s, int lane) {
  bool bp = lane < NV && bad_value(s.qpos[lane]);
  bool bv = lane < NV && bad_value(s.qvel[lane]);
  unsigned long long bpm = __ballot(bp), bvm = __ballot(bv);
  if (bpm | bvm) {
    if (lane == 0) s.status |= (bpm ? ST_BADQPOS : 0u) | (bvm ? ST_BADQVEL : 0u);
    reset_state<NV>(s, lane);
  }
}
// mj_checkAcc: bad qacc -> flag + reset; the caller re-runs forward
template <int NV>
AW_DEV bool check_acc(Env& s, int lane, const Dof& d) {
  if (__ballot(lane < NV && bad_value(d.qacc))) {
    if (lane == 0) s.status |= ST_BADQACC;
    reset_state<NV>(s, lane);
    return true;
  }
  return false;
}

// ---------------------------------------------------------------------------------------
template <int NV>
AW_DEV void load_env(const DModel& m, Env& s, const DState& st, int env, int lane) {
  if (lane < NV) {
    s.qpos[lane] = st.qpos[(size_t)env * m.nq + lane];
    s.qlo[lane] = 0.f;   // the stored state is fp32: the env-step starts from it exactly
    s.qvel[lane] = st.qvel[(size_t)env * m.nv + lane];
    s.warm[lane] = st.warm[(size_t)env * m.nv + lane];
  }
  if (lane == 0) { s.status = 0u; s.slot = blockIdx.x; }
}
template <int NV>
AW_DEV void store_env(const DModel& m, Env& s, const DState& st, int env, int lane) {
  if (lane < NV) {
    st.qpos[(size_t)env * m.nq + lane] = s.qpos[lane];
    st.qvel[(size_t)env * m.nv + lane] = s.qvel[lane];
    st.warm[(size_t)env * m.nv + lane] = s.warm[lane];
  }
}
AW_DEV void write_obs(const DModel& m, Env& s, int lane, float* out) {
  task_obs(m, s, lane, s.rowbuf);
  wsync();
  for (int o = lane; o < m.obs_dim; o += 64) out[o] = s.rowbuf[o];
  wsync();
}

// reset bookkeeping + parameters (given or sampled) + qpos0; forward runs in the caller
template <int NV>
AW_DEV void reset_prepare(const DModel& m, Env& s, const DState& st, int env, int lane,
                          const float* params_in, uint64_t seed) {
  float* prm = st.params + (size_t)env * m.nparam;
  if (lane == 0) {
    if (params_in) {
      for (int p = 0; p < m.nparam; p++) prm[p] = params_in[(size_t)env * m.nparam + p];
    } else {
      float tmp[MAXP];
#pragma unroll
      for (int p = 0; p < MAXP; p++) tmp[p] = p < m.nparam ? prm[p] : 0.f;
      sample_params(m, seed, (uint32_t)(m.env_offset + (unsigned long long)env), (uint32_t)st.episode[env], tmp);
#pragma unroll
      for (int p = 0; p < MAXP; p++)
        if (p < m.nparam) prm[p] = tmp[p];
    }
    st.ep_len[env] = 0;
    st.ep_ret[env] = 0.f;
    st.ep_goal[env] = 0;
  }
  __threadfence_block();
  wsync();
  if (lane < m.nu) s.ctrl[lane] = 0.f;
  reset_state<NV>(s, lane);
  stage_model(m, s, prm, lane);
}

// reset one env in LDS: params (given or sampled), qpos0/0/0, forward, obs
template <int TASK>
AW_DEV void reset_env(const DModel& m, Env& s, const DState& st, int env, int lane,
                      const float* params_in, uint64_t seed, float* obs) {
  constexpr int NV = Tree<TASK>::NV;
  reset_prepare<NV>(m, s, st, env, lane, params_in, seed);
  float Mrow[NV];
  Dof d;
  forward<TASK>(m, s, lane, Mrow, d);
  if (obs) write_obs(m, s, lane, obs + (size_t)env * m.obs_dim);
}

// ---------------------------------------------------------------------------------------
// The wide-tier queue (aw_common.h, two capacity tiers): q[0] = entries, q[1] = the wide kernel's
// claim counter, q[2 + k] = env | kind << 30.  DK_STEP: the whole env-step is re-run from the
// unchanged pre-step state (the fast tier wrote nothing for it); DK_FORWARD: the state, params and
// bookkeeping are written, only mj_forward + obs are re-run (a reset / set_state forward, ctrl 0).
enum { DK_STEP = 0, DK_FORWARD = 1 };
constexpr unsigned ST_OVF = ST_CON_OVERFLOW | ST_EFC_OVERFLOW;
AW_DEV void defer_env(int* q, int env, int kind, int lane) {
  if (lane == 0) {
    const int k = atomicAdd(q, 1);
    q[2 + k] = env | (kind << 30);
  }
}
// fast tier: did the forward just run drop a contact or a row (uniform LDS read)?  (aw_set_tier's
// test mode sends every forward to the wide tier)
AW_DEV bool fast_overflow(const DModel& m, const Env& s) { return !WIDE && ((s.status & ST_OVF) != 0u || m.force_wide); }

// The per-launch I/O of an env-step, parked in LDS by the launching kernel: env_step reads each
// pointer where it is used (the substep loop's memory clobber keeps the reads there), instead of
// ~16 SGPRs of kernel arguments -- and the per-env addresses formed from them -- held live across
// the whole env-step, which the register allocator spilled to scratch once per env (r05h: +2 KB of
// HBM writes per env-step).
struct StepIO {
  const float* actions;
  float *obs, *reward, *terminal_obs;
  uint8_t *done, *goal;
  int* defer;        // fast tier: the wide-tier queue; nullptr in the wide tier
  uint64_t seed;
  int autoreset;
  unsigned* cost;    // per env: shader cycles of its last env-step (k_order's sort key); nullptr: off
  const int* perm;   // claim position -> env (k_order: each XCD class's envs, most expensive first)
  unsigned long long t0;   // this workgroup's current env-step start (s_memtime)
};
// LDS budgets (one wave per workgroup): the fast tier's Env + StepIO inside the 20 480-byte granule
// that gives eight envs per CU (two waves per SIMD); the wide tier's inside 40 KiB (four per CU, one
// wave per SIMD).  A layout change that breaks either is a compile error, not an occupancy surprise.
static_assert(WIDE || sizeof(Env) + sizeof(StepIO) <= 20480, "fast-tier LDS past the two-waves-per-SIMD budget");
static_assert(!WIDE || sizeof(Env) + sizeof(StepIO) <= 40960, "wide-tier LDS past the one-wave-per-SIMD budget");
static_assert(sizeof(((Env*)nullptr)->rowbuf) / sizeof(float) >= 64 * FAST_NRL, "row buffer holds the observation");

AW_DEV void park_io(StepIO& io, int lane, const float* actions, float* obs, float* reward, uint8_t* done,
                    uint8_t* goal, float* terminal_obs, int autoreset, uint64_t seed, int* defer) {
  if (lane == 0) {
    io.actions = actions; io.obs = obs; io.reward = reward; io.terminal_obs = terminal_obs;
    io.done = done; io.goal = goal; io.defer = defer; io.seed = seed; io.autoreset = autoreset;
    io.cost = nullptr; io.perm = nullptr; io.t0 = 0;
  }
  wsync();
}

// One env-step of env `env`: frame_skip x (forward + Euler), task layer, and the auto-reset.
// forward<NV> has exactly ONE inlined call site (the loop below drives substeps, the mj_checkAcc
// retry and the reset forward through it), which keeps the code object small enough for the
// instruction cache.  Fast tier (defer != nullptr): a forward that overflows the fast capacities
// abandons the env-step before anything is written and queues it for the wide tier (or, in the
// reset forward, queues that forward alone).  kind DK_FORWARD (wide tier): only mj_forward + obs of
// the stored state with ctrl 0 -- the reset forward's path through the same loop.
template <int TASK>
AW_DEV void env_step(const DModel& m, Env& s, const DState& st, int env, int lane, StepIO& io,
                     int kind = DK_STEP) {
  constexpr int NV = Tree<TASK>::NV;
  wsync();
  AW_PROF_START(s);
  if (lane == 0 && io.cost) io.t0 = __builtin_amdgcn_s_memtime();
  {
    // an opaque lane id here and in the env-step tail below: per-lane state / obs addresses
    // are formed where they are used instead of once per env and spilled to scratch
    const int el = AW_ENV_LANE(lane);
    load_env<NV>(m, s, st, env, el);
    if (WIDE && el == 0) s.status = ST_WIDE;
    if (el < m.nu) {
      float c = 0.f;
      if (kind == DK_STEP) c = MD(act_mid, el) + clampf(io.actions[(size_t)env * m.nu + el], -1.f, 1.f) * MD(act_rng, el);
      s.ctrl[el] = c;
    }
    stage_model(m, s, st.params + (size_t)env * m.nparam, el);
  }
  float Mrow[NV];
  Dof d;
  int sub = 0;
  bool resetting = kind == DK_FORWARD, retry = false;
  AW_PROF(s, PR_PRE);
#pragma nounroll
  while (true) {
    // memory clobber: keeps LICM from hoisting the (loop-invariant) model loads of a whole
    // substep out of this loop, which would pin them in registers across every stage
    asm volatile("" ::: "memory");
    // and no lane-dependent value is hoisted out of the loop either (the lane id is re-derived
    // per substep): loop-invariant masks and offsets would otherwise occupy SGPRs / VGPRs across
    // every stage of the substep
    const int sl = opaque(lane);
    if (!resetting && !retry) check_state<NV>(s, sl);
    AW_PROF(s, PR_CHECK);
    forward<TASK>(m, s, sl, Mrow, d);
    if (fast_overflow(m, s)) {
      if (!resetting) {            // nothing of this env-step is written: the wide tier re-runs it
        defer_env(io.defer, env, DK_STEP, sl);
        return;
      }
      break;                       // the reset forward alone goes to the wide tier (below)
    }
    if (resetting) break;
    if (!retry && check_acc<NV>(s, sl, d)) { retry = true; continue; }
    retry = false;
    euler<TASK>(m, s, sl, Mrow, d);
    AW_PROF(s, PR_EULER);
    AW_PROF_COUNT(s, PR_SUBSTEPS);
    if (++sub < m.frame_skip) continue;
    // env-step complete: observation, reward, episode bookkeeping
    const int tl = AW_ENV_LANE(lane);
    write_obs(m, s, tl, io.obs + (size_t)env * m.obs_dim);
    int term = 0, trunc = 0;
    if (tl == 0) {
      float r;
      int dn, gl;
      task_reward(m, s, &r, &dn, &gl);
      io.reward[env] = r;
      io.goal[env] = (uint8_t)gl;
      int t = st.ep_len[env] + 1;
      term = dn;
      trunc = (m.horizon > 0 && t >= m.horizon) ? 1 : 0;
      io.done[env] = (uint8_t)(term | (trunc << 1));
      float ret = st.ep_ret[env] + r;
      int gcount = st.ep_goal[env] + gl;
      st.ep_len[env] = t;
      st.ep_ret[env] = ret;
      st.ep_goal[env] = gcount;
      st.status[env] = s.status;
      st.status_acc[env] |= s.status;
      if (term || trunc) {
        st.last_ret[env] = ret;
        st.last_goal[env] = gcount;
        st.last_len[env] = t;
        st.episode[env] += 1;
        st.sum_ret[env] += ret;
        st.n_success[env] += gcount > m.success_steps ? 1 : 0;
      }
    }
    store_env<NV>(m, s, st, env, tl);
    AW_PROF(s, PR_TASK);
    const int ended = __builtin_amdgcn_readfirstlane(term | trunc);
    if (!(io.autoreset && ended)) break;
    __threadfence_block();
    if (float* tob = io.terminal_obs)
      for (int o = tl; o < m.obs_dim; o += 64) tob[(size_t)env * m.obs_dim + o] = s.rowbuf[o];
    wsync();
    reset_prepare<NV>(m, s, st, env, tl, nullptr, io.seed);
    if (WIDE && tl == 0) s.status |= ST_WIDE;
    AW_PROF(s, PR_RESET);
    resetting = true;
  }
  if (resetting) {
    const int rl = AW_ENV_LANE(lane);
    store_env<NV>(m, s, st, env, rl);
    if (fast_overflow(m, s)) {
      if (rl == 0) st.status_acc[env] |= s.status & ~ST_OVF;
      defer_env(io.defer, env, DK_FORWARD, rl);
    } else {
      if (float* ob = io.obs) write_obs(m, s, rl, ob + (size_t)env * m.obs_dim);
      if (rl == 0) {
        st.status_acc[env] |= s.status;
        if (kind == DK_FORWARD) st.status[env] |= s.status;
      }
    }
  }
  // this env-step's cost for the next launch's claim order (k_order)
  if (lane == 0 && io.cost) {
    const unsigned long long dt = __builtin_amdgcn_s_memtime() - io.t0;
    io.cost[env] = dt > 0xffffffffull ? 0xffffffffu : (unsigned)dt;
  }
#ifdef AW_STAGE_PROF
  AW_PROF(s, PR_TASK);
  AW_PROF_COUNT(s, PR_CALLS);
  if (lane == 0)
    for (int i = 0; i < AW_NPROF; i++)
      if (!prof_global(i)) atomicAdd(&g_stage_prof[i], (unsigned long long)s.prof_acc[prof_slot(i)]);
#endif
}

#ifndef AW_WIDE
// The next env for a persistent k_step workgroup, XCD-aware.  Workgroups b and b + 8 share an XCD
// (round-robin dispatch, MI355X_MICROARCH.md -- for speed only, correctness never depends on it),
// so workgroup class c = b % 8 owns envs [n c / 8, n (c + 1) / 8): its first round takes the class's
// first gridDim.x / 8 envs, the rest are claimed from the class's own counter.  Neighbouring envs,
// whose rows share 32-byte sectors (state and obs rows, the 1- and 4-byte per-env scalars), are then
// written through ONE L2, where the partial sectors merge before write-back: k_step's HBM traffic
// 1.81 -> 1.30 KB per env-step (r04p, raw counters).  A class whose range is exhausted claims from
// the next classes, so the tail stays balanced.  Returns n when every class is exhausted.
AW_DEV int claim_env(int* next_env, int n, int lane) {
  const int c0 = blockIdx.x & 7, share = gridDim.x >> 3;
  for (int t = 0; t < 8; t++) {
    const int c = (c0 + t) & 7;
    const int lo = (int)((long long)n * c / 8), hi = (int)((long long)n * (c + 1) / 8);
    if (lo + share >= hi) continue;   // the class's first round covered it
    int k = 0;
    if (lane == 0) k = atomicAdd(next_env + c, 1);
    // readfirstlane: env stays a scalar (SGPR addresses, no per-lane pointer spills)
    const int e = lo + share + __builtin_amdgcn_readfirstlane(k);
    if (e < hi) return e;
  }
  return n;
}

// One launch = one env-step of every env (fast tier).  next_env[0..7]: the per-XCD claim
// counters, next_env[8..]: the wide-tier queue (defer_env).
template <int TASK>
__global__ void __launch_bounds__(64) AW_KSTEP_ATTR k_step(DModel mval, const DModel* __restrict__ mptr, DState stval,
                                             int n, const float* __restrict__ actions,
                                             float* obs, float* reward, uint8_t* done, uint8_t* goal,
                                             float* terminal_obs, int autoreset, uint64_t seed,
                                             int* __restrict__ next_env) {
  // model scalars read from the device copy on demand (scalar loads behind the loop's memory
  // clobber) instead of ~50 kernel-argument SGPRs held live across the whole launch
  const DModel& m = *mptr;
  (void)mval;
  // the state pointers read from the device header where they are used (the loop's memory
  // clobber forces the reload) instead of ~30 SGPRs of kernel arguments live across the launch
  const DState& st = *reinterpret_cast<const DState*>(mptr + 1);   // DState follows DModel in the header
  (void)stval;
  __shared__ Env s;
  __shared__ StepIO io;
  const int lane = threadIdx.x;
  park_io(io, lane, actions, obs, reward, done, goal, terminal_obs, autoreset, seed, next_env + 8);
  const bool xmap = (int)gridDim.x < n && (gridDim.x & 7) == 0;
  // claim positions map to envs through k_order's permutation (same XCD class, costliest first:
  // the launch's last claims are its cheapest envs, r05 A/B -0.3 % random, -2.9 % DAPG)
  if (lane == 0) {
    io.cost = xmap ? reinterpret_cast<unsigned*>(next_env + 10 + n) : nullptr;
    io.perm = xmap ? next_env + 10 + 2 * n : nullptr;
  }
  wsync();
  auto env_of = [&](int pos) {
    if (!io.perm) return pos;
    const int e = io.perm[pos];
    return (unsigned)e < (unsigned)n ? e : pos;
  };
  // Persistent workgroups: the grid is one workgroup per resident slot (launch_step); each takes
  // a first env, then the next unclaimed ones from the launch's counters, so the per-slot spill
  // block (s.slot) is rewritten in the XCD's L2 instead of streaming a per-env block to memory.
  // Envs go out in XCD-contiguous ranges (claim_env above); grids that are not a multiple of 8
  // workgroups (AW_STEP_GRID) take env blockIdx.x first and then claim from one counter.  Every
  // workgroup exits once the counters pass n.
  int env = xmap ? (int)((long long)n * (blockIdx.x & 7) / 8) + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  if (xmap && env >= (int)((long long)n * ((blockIdx.x & 7) + 1) / 8)) env = claim_env(next_env, n, lane);
  while (env < n) {
    env_step<TASK>(m, s, st, env_of(env), lane, io);
    if ((int)gridDim.x >= n) break;            // one env per workgroup: no counter
    int claim = 0;
    if (xmap) {
      env = claim_env(next_env, n, lane);
      continue;
    }
    if (lane == 0) claim = atomicAdd(next_env, 1);
    // readfirstlane, not a shuffle: env stays a scalar, so the addresses formed from it are
    // SGPR values instead of per-lane 64-bit VGPR pairs spilled to scratch once per env
    env = (int)gridDim.x + __builtin_amdgcn_readfirstlane(claim);
  }
}

template <int TASK>
__global__ void __launch_bounds__(64) k_reset(DModel m, DState st, int n, const uint8_t* mask,
                                              const float* params, uint64_t seed, float* obs, int* defer) {
  constexpr int NV = Tree<TASK>::NV;
  __shared__ Env s;
  const int env = blockIdx.x, lane = threadIdx.x;
  if (env >= n) return;
  if (mask && !mask[env]) return;
  if (lane == 0) { s.status = 0u; s.slot = blockIdx.x; }
  reset_prepare<NV>(m, s, st, env, lane, params, seed);
  float Mrow[NV];
  Dof d;
  forward<TASK>(m, s, lane, Mrow, d);
  store_env<NV>(m, s, st, env, lane);
  if (fast_overflow(m, s)) {
    if (lane == 0) { st.status[env] = s.status & ~ST_OVF; st.status_acc[env] |= s.status & ~ST_OVF; }
    defer_env(defer, env, DK_FORWARD, lane);
    return;
  }
  if (obs) write_obs(m, s, lane, obs + (size_t)env * m.obs_dim);
  if (lane == 0) { st.status[env] = s.status; st.status_acc[env] |= s.status; }
}

template <int TASK>
__global__ void __launch_bounds__(64) k_set_state(DModel m, DState st, int n, const float* qpos,
                                                  const float* qvel, const float* warm,
                                                  const float* params, float* obs, int* defer) {
  constexpr int NV = Tree<TASK>::NV;
  __shared__ Env s;
  const int env = blockIdx.x, lane = threadIdx.x;
  if (env >= n) return;
  load_env<NV>(m, s, st, env, lane);
  if (lane < NV) {
    if (qpos) s.qpos[lane] = qpos[(size_t)env * m.nq + lane];
    if (qvel) s.qvel[lane] = qvel[(size_t)env * m.nv + lane];
    if (warm) s.warm[lane] = warm[(size_t)env * m.nv + lane];
  }
  if (params && lane < m.nparam) st.params[(size_t)env * m.nparam + lane] = params[(size_t)env * m.nparam + lane];
  __threadfence_block();
  wsync();
  if (lane < m.nu) s.ctrl[lane] = 0.f;
  stage_model(m, s, st.params + (size_t)env * m.nparam, lane);
  float Mrow[NV];
  Dof d;
  forward<TASK>(m, s, lane, Mrow, d);
  store_env<NV>(m, s, st, env, lane);
  if (fast_overflow(m, s)) {
    if (lane == 0) { st.status[env] = s.status & ~ST_OVF; st.status_acc[env] |= s.status & ~ST_OVF; }
    defer_env(defer, env, DK_FORWARD, lane);
    return;
  }
  if (obs) write_obs(m, s, lane, obs + (size_t)env * m.obs_dim);
  if (lane == 0) { st.status[env] = s.status; st.status_acc[env] |= s.status; }
}
#else  // AW_WIDE
#ifdef AW_WIDE_TWO_SITES
// DIAGNOSTIC ONLY (tools/debug_wide.py, DESIGN.md "the wide-tier hang"): round 5's variant with a
// second inlined forward call site for the queue's forward-only entries (-DAW_WIDE_TWO_SITES_NOINLINE:
// the same code as a called function instead)
#ifdef AW_WIDE_TWO_SITES_NOINLINE
#define AW_FS_ATTR __device__ __attribute__((noinline))
#else
#define AW_FS_ATTR AW_DEV
#endif
template <int TASK>
AW_FS_ATTR void forward_stored(const DModel& m, Env& s, const DState& st, int env, int lane, float* obs) {
  constexpr int NV = Tree<TASK>::NV;
  wsync();
#ifdef AW_TRACE
  if (lane == 0) printf("forward_stored: env %d st.status %p st.status_acc %p &st %p\n", env, (void*)st.status,
                        (void*)st.status_acc, (const void*)&st);
#endif
  load_env<NV>(m, s, st, env, lane);
  if (lane == 0) s.status = ST_WIDE;
  if (lane < m.nu) s.ctrl[lane] = 0.f;
  stage_model(m, s, st.params + (size_t)env * m.nparam, lane);
  float Mrow[NV];
  Dof d;
  forward<TASK>(m, s, lane, Mrow, d);
#ifdef AW_TRACE
  if (lane == 0) printf("forward_stored: env %d forward done, obs %p obs_dim %d\n", env, obs, m.obs_dim);
#endif
  if (obs) {
    task_obs(m, s, lane, s.rowbuf);
#ifdef AW_TRACE
    if (lane == 0) printf("forward_stored: task_obs done\n");
#endif
    wsync();
    for (int o = lane; o < m.obs_dim; o += 64) obs[(size_t)env * m.obs_dim + o] = s.rowbuf[o];
    wsync();
#ifdef AW_TRACE
    if (lane == 0) printf("forward_stored: obs stored; env %d st.status %p st.status_acc %p &st %p s.status %u\n", env,
                          (void*)st.status, (void*)st.status_acc, (const void*)&st, s.status);
#endif
  }
#ifdef AW_TRACE
  {
    const unsigned long long ex0 = __builtin_amdgcn_read_exec();
    if (lane == 0) printf("forward_stored: exec before the status block %llx\n", ex0);
  }
#endif
#ifdef AW_TRACE
  if (lane == 0) {
    const unsigned a = st.status[env];
    printf("forward_stored: status loaded %u\n", a);
    st.status[env] = a | s.status;
    printf("forward_stored: status written\n");
    st.status_acc[env] |= s.status;
    printf("forward_stored: status_acc written\n");
  }
#else
  if (lane == 0) { st.status[env] |= s.status; st.status_acc[env] |= s.status; }
#endif
#ifdef AW_TRACE
  {
    // exec as the scalar unit sees it after the block: a zero exec runs no vector instruction (no
    // printf) and makes the claim loop spin -- restore it only to report
    const unsigned long long ex = __builtin_amdgcn_read_exec();
    if (ex != ~0ull) {
      asm volatile("s_mov_b64 exec, -1" ::: "memory");
      if (lane == 0) printf("forward_stored: EXEC AFTER THE STATUS BLOCK %llx\n", ex);
    }
    if (lane == 0) printf("forward_stored: status stored\n");
  }
#endif
}
#endif
// The wide tier: persistent workgroups drain the queue the fast launch before it filled (q[0]
// entries; an empty queue ends every workgroup at its first claim).  Same env-step code with
// MuJoCo's capacities; mptr is the wide header (its jspill: one JSPILL_WIDE block per workgroup).
// The claim loop is bounded by the handle's env count (the queue holds at most one entry per env and
// launch), so every wave reaches its exit whatever the queue words hold; an entry that is not a valid
// (env < n, kind DK_STEP / DK_FORWARD) pair is skipped -- -DAW_DEVICE_ASSERT traps instead.
template <int TASK>
__global__ void __launch_bounds__(64) k_step_wide(const DModel* __restrict__ mptr, const float* __restrict__ actions,
                                                  float* obs, float* reward, uint8_t* done, uint8_t* goal,
                                                  float* terminal_obs, int autoreset, uint64_t seed,
                                                  int* __restrict__ q, int n) {
  const DModel& m = *mptr;
  const DState& st = *reinterpret_cast<const DState*>(mptr + 1);
  __shared__ Env s;
  __shared__ StepIO io;
  const int lane = threadIdx.x;
  park_io(io, lane, actions, obs, reward, done, goal, terminal_obs, autoreset, seed, nullptr);
  for (int claims = 0; claims <= n; claims++) {
    int k = 0;
    if (lane == 0) k = atomicAdd(q + 1, 1);
    k = __builtin_amdgcn_readfirstlane(k);
#ifdef AW_TRACE
    if (lane == 0) printf("wide wg %d: claimed %d, q0 %d\n", (int)blockIdx.x, k, q[0]);
#endif
    const int nq = q[0];
#ifdef AW_DEVICE_ASSERT
    if ((unsigned)nq > (unsigned)n) __builtin_trap();
#endif
    if (k >= nq || k >= n) break;
    const int ent = q[2 + k];
    const int env = ent & 0x3fffffff, kind = ent >> 30;
    if ((unsigned)env >= (unsigned)n || kind > DK_FORWARD) {
#ifdef AW_DEVICE_ASSERT
      __builtin_trap();
#endif
      continue;
    }
#ifdef AW_TRACE
    if (lane == 0) printf("wide wg %d claim %d of %d: env %d kind %d\n", (int)blockIdx.x, k, q[0], env, kind);
#endif
#ifdef AW_WIDE_TWO_SITES
    if (kind == DK_FORWARD) {
      forward_stored<TASK>(m, s, st, env, lane, io.obs);
      continue;
    }
#endif
    env_step<TASK>(m, s, st, env, lane, io, kind);
  }
#ifdef AW_TRACE
  if (lane == 0) printf("wide wg %d: exit\n", (int)blockIdx.x);
#endif
}
#endif  // AW_WIDE

// introspection: one forward of one env, both tiers (aw_forward_dump / aw_forward_dump_wide)
// dump layout (floats): see mj_envs_amd/_native.py dump_layout (same offsets from the tier's capacities)
constexpr int DUMP_SCAL = 1760, DUMP_CON = 1768, DUMP_EFC = DUMP_CON + 14 * MAXCON;
static_assert(DUMP_EFC + 5 * MAXEFC == (WIDE ? AW_DUMP_SIZE_WIDE : AW_DUMP_SIZE), "AW_DUMP_SIZE(_WIDE) out of date");
// distinct kernel names per tier: the fast and wide translation units both instantiate it
#ifdef AW_WIDE
#define AW_K_DUMP k_dump_wide
#else
#define AW_K_DUMP k_dump
#endif
template <int TASK>
__global__ void __launch_bounds__(64) AW_K_DUMP(DModel m, DState st, int env, const float* ctrl, float* out) {
  constexpr int NV = Tree<TASK>::NV;
  __shared__ Env s;
  const int lane = threadIdx.x;
  load_env<NV>(m, s, st, env, lane);
  if (lane < m.nu) s.ctrl[lane] = ctrl ? ctrl[lane] : 0.f;
  stage_model(m, s, st.params + (size_t)env * m.nparam, lane);
  float Mrow[NV];
  Dof d;
  for (int r = lane; r < MAXEFC; r += 64) out[DUMP_EFC + 4 * MAXEFC + r] = -1.f;
  forward<TASK, true>(m, s, lane, Mrow, d, out + DUMP_EFC + 4 * MAXEFC);   // + the Newton row states
  for (int i = lane; i < MAXB * 3; i += 64) out[i] = i < m.nbody * 3 ? (&s.xpos[0][0])[i] : 0.f;
  for (int i = lane; i < MAXB * 4; i += 64) out[96 + i] = i < m.nbody * 4 ? (&s.xquat[0][0])[i] : 0.f;
  for (int i = lane; i < MAXS * 3; i += 64) out[224 + i] = i < m.nsite * 3 ? (&s.sxpos[0][0])[i] : 0.f;
  if (lane < MAXV) {
    bool v = lane < NV;
    out[320 + lane] = v ? d.qacc_smooth : 0.f;
    out[356 + lane] = v ? d.qfrc_smooth : 0.f;
    out[392 + lane] = v ? d.qacc : 0.f;
    out[428 + lane] = v ? d.qfrc_con : 0.f;
  }
  for (int k = 0; k < NV; k++)
    if (lane < NV) out[464 + lane * NV + k] = Mrow[k];
  if (lane == 0) {
    out[DUMP_SCAL] = (float)s.ncon; out[DUMP_SCAL + 1] = (float)s.nefc; out[DUMP_SCAL + 2] = (float)s.nsparse;
    out[DUMP_SCAL + 3] = (float)s.ndense; out[DUMP_SCAL + 4] = s.touch[0]; out[DUMP_SCAL + 5] = (float)s.status;
    out[DUMP_SCAL + 6] = (float)s.it_newton; out[DUMP_SCAL + 7] = (float)s.it_noslip;
  }
  for (int c = lane; c < MAXCON; c += 64) {
    bool v = c < s.ncon;
    out[DUMP_CON + c] = v ? s.con_dist[c] : 0.f;
    for (int k = 0; k < 3; k++) out[DUMP_CON + MAXCON + 3 * c + k] = v ? s.con_pos[c][k] : 0.f;
    float fr[9];
    for (int k = 0; k < 3; k++) { fr[k] = v ? s.con_nrm[c][k] : 1.f; fr[3 + k] = 0.f; }
    make_frame(fr);
    for (int k = 0; k < 9; k++) out[DUMP_CON + 4 * MAXCON + 9 * c + k] = v ? fr[k] : 0.f;
    out[DUMP_CON + 13 * MAXCON + c] = v ? (float)s.con_pair[c] : -1.f;
  }
  for (int r = lane; r < MAXEFC; r += 64) {
    bool v = r < s.nefc;
    out[DUMP_EFC + r] = v ? s.efc_force[r] : 0.f;
    out[DUMP_EFC + MAXEFC + r] = v ? s.efc_aref[r] : 0.f;
    out[DUMP_EFC + 2 * MAXEFC + r] = v ? s.efc_D[r] : 0.f;
    out[DUMP_EFC + 3 * MAXEFC + r] = v ? (float)s.efc_type[r] : -1.f;
  }
}

#ifndef AW_TASK_TU   // task-independent kernels: in the API translation unit only
__global__ void __launch_bounds__(64) k_task_eval(DModel m, int n, const float* qpos, const float* qvel,
                                                  const float* xpos, const float* xquat, const float* sxpos,
                                                  const float* touch, float* obs, float* reward, uint8_t* done,
                                                  uint8_t* goal) {
  __shared__ Env s;
  const int i = blockIdx.x, lane = threadIdx.x;
  if (i >= n) return;
  if (lane < m.nq) { s.qpos[lane] = qpos[(size_t)i * m.nq + lane]; s.qlo[lane] = 0.f; }
  if (lane < m.nv) s.qvel[lane] = qvel[(size_t)i * m.nv + lane];
  for (int k = lane; k < m.nbody * 3; k += 64) (&s.xpos[0][0])[k] = xpos[(size_t)i * m.nbody * 3 + k];
  for (int k = lane; k < m.nbody * 4; k += 64) (&s.xquat[0][0])[k] = xquat[(size_t)i * m.nbody * 4 + k];
  for (int k = lane; k < m.nsite * 3; k += 64) (&s.sxpos[0][0])[k] = sxpos[(size_t)i * m.nsite * 3 + k];
  if (lane == 0) s.touch[0] = touch ? touch[i] : 0.f;
  wsync();
  write_obs(m, s, lane, obs + (size_t)i * m.obs_dim);
  if (lane == 0) {
    float r;
    int dn, gl;
    task_reward(m, s, &r, &dn, &gl);
    reward[i] = r; done[i] = (uint8_t)dn; goal[i] = (uint8_t)gl;
  }
}

// Test hook (aw_collide_test): the narrowphase of one primitive pair per workgroup, given world
// poses -- exact-geometry collider tests against the oracle's colliders.
// Lanes 0..15 call it with the same pair (gl = lane): capsule-box runs on the 16-lane row and MPR
// on lanes 0 and 1 as in the narrowphase, every other collider on lane 0.
AW_DEV void collide_gv(const DModel& m, const GV& a, const GV& b, float margin, Emit& e, int gl) {
  const int lo = a.type, hi = b.type;   // a.type <= b.type
  if (hi == GEOM_BOX && lo == GEOM_CAPSULE) {
    c_capsule_box(a, b, margin, e, gl);
    return;
  }
  if (lo != GEOM_PLANE && (lo == GEOM_CYLINDER || hi == GEOM_CYLINDER)) {   // MPR on lanes 0 and 1
    if (gl > 1) return;
    const GV& g = gl ? b : a;
    mpr::GVdT<double> own;
    for (int k = 0; k < 3; k++) { own.pos[k] = g.pos[k]; own.size[k] = g.size[k]; }
    for (int k = 0; k < 9; k++) own.mat[k] = g.mat[k];
    own.type = g.type;
    c_convex64(m, own, gl, (double)margin, e);
    return;
  }
  if (gl != 0) return;
  if (lo == GEOM_PLANE) {
    if (hi == GEOM_SPHERE) c_plane_sphere(a.pos, a.mat, b.pos, b.size[0], margin, e);
    else if (hi == GEOM_CAPSULE) c_plane_capsule(a, b, margin, e);
    else if (hi == GEOM_CYLINDER) c_plane_cylinder(a, b, margin, e);
    else if (hi == GEOM_BOX) c_plane_box(a, b, margin, e);
  } else if (hi == GEOM_BOX && lo == GEOM_BOX) {
    c_box_box(a, b, margin, e);
  } else if (hi == GEOM_BOX) {
    c_sphere_box_pt(a.pos, a.size[0], b, margin, e);
  } else if (lo == GEOM_SPHERE && hi == GEOM_SPHERE) {
    c_sphere_sphere(a.pos, a.size[0], b.pos, b.size[0], margin, e);
  } else if (lo == GEOM_SPHERE) {
    c_sphere_capsule(a, b, margin, e);
  } else {
    c_capsule_capsule(a, b, margin, e);
  }
}

__global__ void __launch_bounds__(64) k_collide_test(DModel m, int n, const int* types, const float* pos,
                                                     const float* mat, const float* size, const float* margin,
                                                     float* out, int* count, double* out64) {
  __shared__ Env s;
  const int i = blockIdx.x, lane = threadIdx.x;
  if (i >= n) return;
  if (lane == 0) { s.ncon = 0; s.status = 0u; }
  wsync();
  if (lane < 16) {
    GV g[2];
    for (int q = 0; q < 2; q++) {
      g[q].type = types[2 * i + q];
      for (int k = 0; k < 3; k++) { g[q].pos[k] = pos[6 * i + 3 * q + k]; g[q].size[k] = size[6 * i + 3 * q + k]; }
      for (int k = 0; k < 9; k++) g[q].mat[k] = mat[18 * i + 9 * q + k];
    }
    const int f = g[0].type <= g[1].type ? 0 : 1;
    Emit e{&s, 0, 0, out64 ? out64 + (size_t)i * MAXPAIRCON * 7 : nullptr};
    collide_gv(m, g[f], g[1 - f], margin[i], e, lane);
  }
  wsync();
  const int nc = s.ncon < MAXPAIRCON ? s.ncon : MAXPAIRCON;
  if (lane == 0) count[i] = nc;
  if (lane < nc) {
    float* o = out + ((size_t)i * MAXPAIRCON + s.con_key[lane]) * 7;   // emission order
    o[0] = s.con_dist[lane];
    for (int k = 0; k < 3; k++) { o[1 + k] = s.con_pos[lane][k]; o[4 + k] = s.con_nrm[lane][k]; }
  }
}

#endif  // AW_TASK_TU

// depth frame of every env's current state: wave 0 runs the kinematics, then all four waves
// cast the pixels (one workgroup per env; render geom poses staged in LDS)
struct CamRec {
  float c[AW_CAM_FLOATS];
};
template <int TASK>
__global__ void __launch_bounds__(256) k_depth(DModel m, DState st, int n, CamRec cam, int W, int H, float* out) {
  constexpr int NV = Tree<TASK>::NV;
  __shared__ Env s;
  __shared__ RGeoms rg;
  const int env = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  if (env >= n) return;
  if (tid < 64) {
    if (lane < NV) { s.qpos[lane] = st.qpos[(size_t)env * m.nq + lane]; s.qlo[lane] = 0.f; }
    wsync();
    stage_model(m, s, st.params + (size_t)env * m.nparam, lane);
    stage_kinematics(m, s, lane);
  }
  __syncthreads();
  render_geoms(m, s, rg, cam.c, tid, 256);
  __syncthreads();
  float* o = out + (size_t)env * W * H;
  for (int p0 = (tid >> 6) * 64; p0 < W * H; p0 += 256) render_span(rg, m.nrgeom, cam.c, W, H, p0, lane, o);
}

#ifndef AW_TASK_TU
__global__ void k_random_actions(int n, int nu, uint64_t seed, uint64_t step, uint64_t env_offset, float* out) {
  int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n) return;
  const uint32_t genv = (uint32_t)(env_offset + (uint64_t)env);   // global env id (shard offset)
  for (int blk = 0; blk * 4 < nu; blk++) {
    uint32_t c[4] = {genv, (uint32_t)step, (uint32_t)(step >> 32), (uint32_t)blk};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    for (int k = 0; k < 4 && blk * 4 + k < nu; k++) out[(size_t)env * nu + blk * 4 + k] = 2.f * u01(c[k]) - 1.f;
  }
}

#endif  // AW_TASK_TU

// ---------------------------------------------------------------------------------------
// host side
#ifndef AW_TASK_TU
namespace {
thread_local std::string g_err;
int fail(int code, const std::string& msg) { g_err = msg; return code; }
#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return fail(AW_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); } while (0)

struct Blob {
  const void* p; size_t n;
  bool has(const char* name) const { aw_blob_entry e; return aw_blob_find(p, n, name, &e); }
  std::vector<double> f(const char* name) const {
    aw_blob_entry e;
    std::vector<double> out;
    if (!aw_blob_find(p, n, name, &e)) return out;
    size_t cnt = (size_t)e.rows * e.cols;
    out.resize(cnt);
    const char* d = (const char*)e.data;
    for (size_t i = 0; i < cnt; i++) {
      if (e.kind == 0) { double v; memcpy(&v, d + 8 * i, 8); out[i] = v; }
      else { int32_t v; memcpy(&v, d + 4 * i, 4); out[i] = v; }
    }
    return out;
  }
  std::vector<int> i(const char* name) const {
    std::vector<double> v = f(name);
    return std::vector<int>(v.begin(), v.end());
  }
  int dim(const char* name, int dflt = -1) const { return aw_blob_dim(p, n, name, dflt); }
  double opt(const char* name, double dflt) const { return aw_blob_opt(p, n, name, dflt); }
};

template <class T, size_t N, class U>
bool put_arr(T (&dst)[N], const std::vector<U>& v) {
  if (v.size() > N) return false;
  for (size_t i = 0; i < v.size(); i++) dst[i] = (T)v[i];
  return true;
}
#define PUT(name, ...)                                                                        \
  do {                                                                                        \
    if (!put_arr(md.name, __VA_ARGS__)) return fail(AW_EUNSUPPORTED, "model field " #name " exceeds kernel capacity"); \
  } while (0)

std::vector<float> tof(const std::vector<double>& v) { return std::vector<float>(v.begin(), v.end()); }
}  // namespace

#endif  // AW_TASK_TU

struct aw_handle {
  int device, nenv, NV;
  DModel m;
  DState st;
  void* dmodel = nullptr;
  void* dmhdr = nullptr;   // device copy of m (k_step reads its scalars from here)
  void* dstate = nullptr;
  int* next_env = nullptr;   // [0, 8): k_step's per-XCD claim counters; [8, 10 + nenv): the wide-tier
                             // queue (count, claim counter, entries; adroit_wave.hip defer_env);
                             // [10 + nenv, 10 + 2 nenv): per-env env-step cycles, [10 + 2 nenv,
                             // 10 + 3 nenv): the claim permutation (k_order)
  int slots = 0;             // persistent k_step grid: resident workgroups of the selected instantiation,
                             // or AW_STEP_GRID (read at aw_create; 0 = one workgroup per env)
  int grid_env = -1;         // AW_STEP_GRID at create (-1: unset)
  void* dmhdr_wide = nullptr;   // the wide tier's header: m with jspill -> jspill_wide, then st
  float* jspill_wide = nullptr; // one JSPILL_WIDE block per wide workgroup
  int wide_grid = 0;            // persistent k_step_wide workgroups (resident slots, capped at nenv)
  // aw_set_fault: the model table's pair margins / broadphase radii as built (restored by kind 0)
  std::vector<float> fault_margin0, fault_rb0;
  std::vector<double> fault_margin64_0;
  std::vector<int> fault_cls;
};

#ifndef AW_TASK_TU
static int upload_header(aw_handle* h) {
  HIPCHK(hipMemcpy(h->dmhdr, &h->m, sizeof(DModel), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy((DModel*)h->dmhdr + 1, &h->st, sizeof(DState), hipMemcpyHostToDevice));
  DModel mw = h->m;
  mw.jspill = h->jspill_wide;
  HIPCHK(hipMemcpy(h->dmhdr_wide, &mw, sizeof(DModel), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy((DModel*)h->dmhdr_wide + 1, &h->st, sizeof(DState), hipMemcpyHostToDevice));
  return AW_OK;
}

static int build_model(const Blob& B, DModel& m, MData& md) {
  memset(&m, 0, sizeof(m));
  int nq = B.dim("nq"), nv = B.dim("nv"), nu = B.dim("nu"), nbody = B.dim("nbody"), njnt = B.dim("njnt");
  int ngeom_all = B.dim("ngeom"), nsite = B.dim("nsite"), ntendon = B.dim("ntendon");
  int npair = B.dim("npair"), ncand = B.dim("ncand"), nsensor = B.dim("nsensor");
  if (nq < 0 || nv < 0 || nbody < 0 || B.dim("task_kind") < 0) return fail(AW_EBLOB, "model table lacks dims / task block");
  if (nq != nv || njnt != nv) return fail(AW_EUNSUPPORTED, "only hinge/slide joints are supported");
  if (nv > MAXV || nbody > MAXB || nsite > MAXS || ntendon > MAXT || nu > MAXU)
    return fail(AW_EUNSUPPORTED, "model exceeds kernel capacity");
  m.nq = nq; m.nv = nv; m.nu = nu; m.nbody = nbody; m.njnt = njnt; m.nsite = nsite; m.ntendon = ntendon;
  m.timestep = (float)B.opt("timestep", 0.002);
  m.gravity[0] = (float)B.opt("gravity_x", 0); m.gravity[1] = (float)B.opt("gravity_y", 0);
  m.gravity[2] = (float)B.opt("gravity_z", -9.81);
  m.iterations = (int)B.opt("iterations", 100);
  m.tolerance = (float)B.opt("tolerance", 1e-8);
  m.noslip_iterations = (int)B.opt("noslip_iterations", 0);
  m.noslip_tolerance = (float)B.opt("noslip_tolerance", 1e-6);
  m.mpr_tolerance = (float)B.opt("mpr_tolerance", 1e-6);
  m.mpr_iterations = (int)B.opt("mpr_iterations", 50);
  m.mpr_tolerance64 = B.opt("mpr_tolerance", 1e-6);
  m.meaninertia = (float)B.opt("meaninertia", 1);
  // pyramidal cones only: R = max(mjMINVAL, (1 - imp) / imp * diagApprox) per edge row, diagApprox =
  // invweight_tran + friction^2 * invweight_(tran|rot); impratio (the elliptic cones' friction /
  // normal impedance ratio) is restated only at its default 1, where it is the identity
  if (B.opt("impratio", 1) != 1.0) return fail(AW_EUNSUPPORTED, "impratio != 1");
  m.pen_length = (float)B.opt("task_pen_length", 1);
  m.tar_length = (float)B.opt("task_tar_length", 1);
  m.task_kind = B.dim("task_kind"); m.frame_skip = B.dim("task_frame_skip", 1);
  m.horizon = B.dim("task_horizon", 0); m.obs_dim = B.dim("task_obs_dim", 0);
  // the observation is assembled in the row buffer (write_obs): it must fit the fast tier's
  if (m.obs_dim < 0 || m.obs_dim > 64 * FAST_NRL) return fail(AW_EUNSUPPORTED, "observation larger than the row buffer");
  m.success_steps = B.dim("task_success_steps", 25);
  m.nparam = B.dim("task_nparam", 0); m.variation = B.dim("task_variation", 0);
  if (m.nparam > MAXP) return fail(AW_EUNSUPPORTED, "too many per-env params");
  m.disableflags = 0;
  m.fault_flrow = -1;

  std::vector<int> parent = B.i("body_parentid"), rootid = B.i("body_rootid"), dofnum = B.i("body_dofnum"),
                   dofadr = B.i("body_dofadr");
  for (int b = 0; b < nbody; b++)
    if (dofnum[b] > MAXJB) return fail(AW_EUNSUPPORTED, "more than MAXJB joints in one body");
  // subtree ends (DFS order), levels, dof masks
  std::vector<int> send(nbody), depth(nbody, 0);
  for (int b = 0; b < nbody; b++) send[b] = b + 1;
  for (int b = nbody - 1; b > 0; b--) send[parent[b]] = std::max(send[parent[b]], send[b]);
  for (int b = 1; b < nbody; b++) depth[b] = depth[parent[b]] + 1;
  int nlev = 0;
  for (int b = 0; b < nbody; b++) nlev = std::max(nlev, depth[b] + 1);
  if (nlev > MAXLEV) return fail(AW_EUNSUPPORTED, "tree too deep");
  std::vector<int> lstart(nlev + 1, 0), lbody;
  for (int l = 0; l < nlev; l++) {
    lstart[l] = (int)lbody.size();
    for (int b = 0; b < nbody; b++)
      if (depth[b] == l) lbody.push_back(b);
  }
  lstart[nlev] = (int)lbody.size();
  m.nlevel = nlev;
  std::vector<int> dparent = B.i("dof_parentid");
  std::vector<unsigned long long> bmask(nbody, 0), amask(nv, 0);
  for (int b = 1; b < nbody; b++) {
    int a = b;
    while (a > 0) {
      for (int k = 0; k < dofnum[a]; k++) bmask[b] |= 1ull << (dofadr[a] + k);
      a = parent[a];
    }
  }
  for (int j = 0; j < nv; j++)
    for (int a = dparent[j]; a >= 0; a = dparent[a]) amask[j] |= 1ull << a;

  PUT(body_parentid, parent); PUT(body_rootid, rootid); PUT(body_dofnum, dofnum);
  PUT(body_dofadr, dofadr); PUT(body_depth, depth); PUT(body_subtree_end, send); PUT(level_start, lstart);
  PUT(level_body, lbody);
  PUT(body_pos, tof(B.f("body_pos"))); PUT(body_quat, tof(B.f("body_quat")));
  PUT(body_ipos, tof(B.f("body_ipos"))); PUT(body_iquat, tof(B.f("body_iquat")));
  PUT(body_mass, tof(B.f("body_mass"))); PUT(body_inertia, tof(B.f("body_inertia")));
  PUT(body_invweight0, tof(B.f("body_invweight0")));
  PUT(body_subtreemass, tof(B.f("body_subtreemass")));
  PUT(body_dofmask, bmask);
  PUT(body_pos64, B.f("body_pos")); PUT(body_quat64, B.f("body_quat"));
  PUT(jnt_pos64, B.f("jnt_pos")); PUT(jnt_axis64, B.f("jnt_axis"));

  std::vector<int> jtype = B.i("jnt_type");
  for (int t : jtype) if (t != JNT_HINGE && t != JNT_SLIDE) return fail(AW_EUNSUPPORTED, "joint type");
  PUT(jnt_type, jtype); PUT(jnt_bodyid, B.i("jnt_bodyid")); PUT(jnt_limited, B.i("jnt_limited"));
  PUT(jnt_pos, tof(B.f("jnt_pos"))); PUT(jnt_axis, tof(B.f("jnt_axis")));
  PUT(jnt_range, tof(B.f("jnt_range"))); PUT(jnt_margin, tof(B.f("jnt_margin")));
  PUT(jnt_solref, tof(B.f("jnt_solref"))); PUT(jnt_solimp, tof(B.f("jnt_solimp")));
  PUT(jnt_range64, B.f("jnt_range")); PUT(jnt_margin64, B.f("jnt_margin"));

  // actuators (joint transmission, one per dof)
  std::vector<int> trn = B.i("actuator_trnid");
  std::vector<int> dact(nv, -1);
  for (int u = 0; u < nu; u++) {
    if (dact[trn[u]] >= 0) return fail(AW_EUNSUPPORTED, "two actuators on one joint");
    dact[trn[u]] = u;
  }
  std::vector<double> floss = B.f("dof_frictionloss");
  std::vector<int> fl_dof, fl_row(nv, -1);
  for (int j = 0; j < nv; j++)
    if (floss[j] > 0) { fl_row[j] = (int)fl_dof.size(); fl_dof.push_back(j); }
  m.nfl = (int)fl_dof.size();
  PUT(dof_bodyid, B.i("dof_bodyid")); PUT(dof_act, dact); PUT(fl_dof, fl_dof);
  PUT(fl_row, fl_row); PUT(dof_ancmask, amask);
  PUT(dof_armature, tof(B.f("dof_armature"))); PUT(dof_damping, tof(B.f("dof_damping")));
  PUT(dof_frictionloss, tof(floss)); PUT(dof_invweight0, tof(B.f("dof_invweight0")));
  PUT(dof_solref, tof(B.f("dof_solref"))); PUT(dof_solimp, tof(B.f("dof_solimp")));

  // compact collidable geoms
  std::vector<int> gtype = B.i("geom_type"), gcon = B.i("geom_contype"), gaff = B.i("geom_conaffinity"),
                   gbody = B.i("geom_bodyid");
  std::vector<double> gpos = B.f("geom_pos"), gquat = B.f("geom_quat"), gsize = B.f("geom_size"),
                      grb = B.f("geom_rbound");
  std::vector<int> gmap(ngeom_all, -1), ctype, cbody;
  std::vector<float> cpos, cquat, csize, crb;
  std::vector<double> cpos64, cquat64, csize64;
  for (int g = 0; g < ngeom_all; g++) {
    if (gtype[g] == 7 || (gcon[g] == 0 && gaff[g] == 0)) continue;
    gmap[g] = (int)ctype.size();
    ctype.push_back(gtype[g]); cbody.push_back(gbody[g]);
    for (int k = 0; k < 3; k++) { cpos.push_back((float)gpos[3 * g + k]); csize.push_back((float)gsize[3 * g + k]); }
    for (int k = 0; k < 4; k++) cquat.push_back((float)gquat[4 * g + k]);
    for (int k = 0; k < 3; k++) { cpos64.push_back(gpos[3 * g + k]); csize64.push_back(gsize[3 * g + k]); }
    for (int k = 0; k < 4; k++) cquat64.push_back(gquat[4 * g + k]);
    crb.push_back((float)grb[g]);
  }
  PUT(geom_pos64, cpos64); PUT(geom_quat64, cquat64); PUT(geom_size64, csize64);
  m.ngeom = (int)ctype.size();
  if (m.ngeom > MAXG) return fail(AW_EUNSUPPORTED, "too many collidable geoms");
  PUT(geom_type, ctype); PUT(geom_bodyid, cbody); PUT(geom_pos, cpos);
  PUT(geom_quat, cquat); PUT(geom_size, csize); PUT(geom_rbound, crb);

  PUT(site_bodyid, B.i("site_bodyid")); PUT(site_pos, tof(B.f("site_pos")));
  PUT(site_quat, tof(B.f("site_quat")));

  // tendons: fixed, <= 2 joints
  std::vector<int> tadr = B.i("tendon_adr"), tnum = B.i("tendon_num"), wj = B.i("wrap_jnt");
  std::vector<double> wc = B.f("wrap_coef"), tfl = B.f("tendon_frictionloss");
  std::vector<int> d0(ntendon), d1(ntendon);
  std::vector<float> c0(ntendon), c1(ntendon);
  for (int t = 0; t < ntendon; t++) {
    if (tnum[t] < 1 || tnum[t] > 2) return fail(AW_EUNSUPPORTED, "tendon with != 1..2 joints");
    if (tfl[t] > 0) return fail(AW_EUNSUPPORTED, "tendon frictionloss");
    d0[t] = wj[tadr[t]]; c0[t] = (float)wc[tadr[t]];
    d1[t] = tnum[t] > 1 ? wj[tadr[t] + 1] : -1; c1[t] = tnum[t] > 1 ? (float)wc[tadr[t] + 1] : 0.f;
  }
  PUT(ten_d0, d0); PUT(ten_d1, d1); PUT(ten_limited, B.i("tendon_limited"));
  PUT(ten_c0, c0); PUT(ten_c1, c1); PUT(ten_range, tof(B.f("tendon_range")));
  PUT(ten_margin, tof(B.f("tendon_margin"))); PUT(ten_solref, tof(B.f("tendon_solref")));
  PUT(ten_solimp, tof(B.f("tendon_solimp"))); PUT(ten_invweight0, tof(B.f("tendon_invweight0")));
  PUT(ten_range64, B.f("tendon_range")); PUT(ten_margin64, B.f("tendon_margin"));
  {
    std::vector<double> a0(ntendon), a1(ntendon);
    for (int t = 0; t < ntendon; t++) { a0[t] = wc[tadr[t]]; a1[t] = tnum[t] > 1 ? wc[tadr[t] + 1] : 0.0; }
    PUT(ten_c0_64, a0); PUT(ten_c1_64, a1);
  }

  std::vector<double> gain = B.f("actuator_gainprm");
  std::vector<float> g0(nu);
  for (int u = 0; u < nu; u++) g0[u] = (float)gain[3 * u];
  PUT(act_ctrllimited, B.i("actuator_ctrllimited")); PUT(act_forcelimited, B.i("actuator_forcelimited"));
  PUT(act_gear, tof(B.f("actuator_gear"))); PUT(act_gain, g0);
  PUT(act_bias, tof(B.f("actuator_biasprm"))); PUT(act_ctrlrange, tof(B.f("actuator_ctrlrange")));
  PUT(act_forcerange, tof(B.f("actuator_forcerange")));

  // unified pair list: explicit pairs (own params), then candidates (params mixed here in fp64,
  // mj_contactParam with equal priorities)
  std::vector<int> pg1, pg2, pcd;
  std::vector<float> pfr, psr, psi, pmg, pgp;
  std::vector<double> pmg64;
  {
    std::vector<int> e1 = B.i("pair_geom1"), e2 = B.i("pair_geom2"), ecd = B.i("pair_condim");
    std::vector<double> efr = B.f("pair_friction"), esr = B.f("pair_solref"), esi = B.f("pair_solimp"),
                        emg = B.f("pair_margin"), egp = B.f("pair_gap");
    for (int p = 0; p < npair; p++) {
      if (gmap[e1[p]] < 0 || gmap[e2[p]] < 0) return fail(AW_EUNSUPPORTED, "pair with a visual geom");
      pg1.push_back(gmap[e1[p]]); pg2.push_back(gmap[e2[p]]); pcd.push_back(ecd[p]);
      for (int k = 0; k < 5; k++) pfr.push_back((float)efr[5 * p + k]);
      for (int k = 0; k < 2; k++) psr.push_back((float)esr[2 * p + k]);
      for (int k = 0; k < 5; k++) psi.push_back((float)esi[5 * p + k]);
      pmg.push_back((float)emg[p]); pgp.push_back((float)egp[p]); pmg64.push_back(emg[p]);
    }
    std::vector<int> c1v = B.i("cand_geom1"), c2v = B.i("cand_geom2"), gcd = B.i("geom_condim");
    std::vector<double> gfr = B.f("geom_friction"), gsm = B.f("geom_solmix"), gsr = B.f("geom_solref"),
                        gsi = B.f("geom_solimp"), gmg = B.f("geom_margin"), ggp = B.f("geom_gap");
    for (int c = 0; c < ncand; c++) {
      int a = c1v[c], b = c2v[c];
      pg1.push_back(gmap[a]); pg2.push_back(gmap[b]);
      pcd.push_back(std::max(gcd[a], gcd[b]));
      double s1 = gsm[a], s2 = gsm[b], mix;
      if (s1 >= 1e-15 && s2 >= 1e-15) mix = s1 / (s1 + s2);
      else if (s1 < 1e-15 && s2 < 1e-15) mix = 0.5;
      else mix = s1 < 1e-15 ? 0.0 : 1.0;
      double f0 = std::max(gfr[3 * a], gfr[3 * b]), f1 = std::max(gfr[3 * a + 1], gfr[3 * b + 1]),
             f2 = std::max(gfr[3 * a + 2], gfr[3 * b + 2]);
      double fr[5] = {f0, f0, f1, f2, f2};
      for (int k = 0; k < 5; k++) pfr.push_back((float)fr[k]);
      for (int k = 0; k < 2; k++) psr.push_back((float)(mix * gsr[2 * a + k] + (1 - mix) * gsr[2 * b + k]));
      for (int k = 0; k < 5; k++) psi.push_back((float)(mix * gsi[5 * a + k] + (1 - mix) * gsi[5 * b + k]));
      pmg.push_back((float)std::max(gmg[a], gmg[b])); pgp.push_back((float)std::max(ggp[a], ggp[b]));
      pmg64.push_back(std::max(gmg[a], gmg[b]));
    }
  }
  m.npairall = (int)pg1.size();
  {
    // collider class per pair (aw_collide.h collide_pair dispatch) and the broadphase radius
    std::vector<int> pcls(m.npairall);
    std::vector<float> prb(m.npairall);
    int ccount[NCLASS] = {0, 0, 0, 0, 0};
    for (int p = 0; p < m.npairall; p++) {
      int a = pg1[p], b = pg2[p];
      int ta = ctype[a], tb = ctype[b];
      int lo = std::min(ta, tb), hi = std::max(ta, tb);
      int c;
      if (lo == GEOM_PLANE) c = 0;
      else if (lo == GEOM_CYLINDER || hi == GEOM_CYLINDER) c = 4;
      else if (hi == GEOM_BOX && lo == GEOM_BOX) c = 3;
      else if (hi == GEOM_BOX) c = 2;
      else c = 1;
      pcls[p] = c;
      ccount[c]++;
      // plane pairs: -(1 + rbound of the other geom + margin) (< -1: the broadphase's plane test)
      prb[p] = lo == GEOM_PLANE ? (float)(-1.0 - (double)crb[ta == GEOM_PLANE ? b : a] - (double)pmg[p])
                                : (float)((double)crb[a] + (double)crb[b] + (double)pmg[p]);
    }
    m.cls_start[0] = 0;
    for (int c = 0; c < NCLASS; c++) m.cls_start[c + 1] = m.cls_start[c] + ccount[c];
    if (m.npairall > JL * VS * 2) return fail(AW_EUNSUPPORTED, "too many collision pairs");
    PUT(cp_class, pcls); PUT(cp_rb, prb); PUT(cp_margin64, pmg64);
    // per pair: the bodies whose fp64 frames its geometry needs (stage_kin64), with ancestors
    // (every class: the sphere / capsule pairs' near-margin contacts are decided on fp64 frames too)
    std::vector<unsigned long long> k64(m.npairall, 0ull);
    for (int p = 0; p < m.npairall; p++)
      for (int g : {pg1[p], pg2[p]})
        for (int b = cbody[g]; b > 0; b = parent[b]) k64[p] |= 1ull << b;
    PUT(cp_kin64, k64);
    std::vector<int> ppack(m.npairall);
    for (int p = 0; p < m.npairall; p++) ppack[p] = pcls[p] | (pg1[p] << 8) | (pg2[p] << 16);
    PUT(cp_pack, ppack);
  }
  {
    std::vector<double> iw = B.f("body_invweight0");
    std::vector<float> ptran(pg1.size()), prot(pg1.size());
    std::vector<int> pr1(pg1.size()), pr2(pg1.size());
    std::vector<unsigned long long> pm1(pg1.size()), pm2(pg1.size());
    for (size_t p = 0; p < pg1.size(); p++) {
      const int b1 = cbody[pg1[p]], b2 = cbody[pg2[p]];
      ptran[p] = (float)iw[2 * b1] + (float)iw[2 * b2];
      prot[p] = (float)iw[2 * b1 + 1] + (float)iw[2 * b2 + 1];
      pr1[p] = rootid[b1]; pr2[p] = rootid[b2];
      pm1[p] = bmask[b1]; pm2[p] = bmask[b2];
    }
    PUT(cp_tran, ptran); PUT(cp_rot, prot); PUT(cp_root1, pr1); PUT(cp_root2, pr2);
    PUT(cp_mask1, pm1); PUT(cp_mask2, pm2);
  }
  PUT(cp_g1, pg1); PUT(cp_g2, pg2); PUT(cp_condim, pcd); PUT(cp_friction, pfr);
  PUT(cp_solref, psr); PUT(cp_solimp, psi); PUT(cp_margin, pmg); PUT(cp_gap, pgp);

  // task block
  std::vector<int> tidx = B.i("task_idx"), pf = B.i("task_param_field"), po = B.i("task_param_obj"),
                   pc = B.i("task_param_comp");
  for (int p = 0; p < m.nparam; p++)
    if (pf[p] == 4 || pf[p] == 5) {
      if (gmap[po[p]] < 0) return fail(AW_EUNSUPPORTED, "param on a visual geom");
      po[p] = gmap[po[p]];
    }
  // touch sensors read by the task (hammer: S_nail, task_idx[5] = its sensordata address)
  std::vector<int> ts, ttype;
  std::vector<float> tsize;
  if (m.task_kind == 0 && tidx.size() > 5) {
    std::vector<int> stype = B.i("sensor_type"), sobj = B.i("sensor_objid"), sadr = B.i("sensor_adr");
    std::vector<int> sitetype = B.i("site_type");
    std::vector<double> ssize = B.f("site_size");
    for (int k = 0; k < nsensor; k++)
      if (sadr[k] == tidx[5] && stype[k] == 0) {
        ts.push_back(sobj[k]); ttype.push_back(sitetype[sobj[k]]);
        for (int q = 0; q < 3; q++) tsize.push_back((float)ssize[3 * sobj[k] + q]);
      }
  }
  m.ntouch = (int)ts.size();
  PUT(touch_site, ts); PUT(touch_adr, ts); PUT(touch_type, ttype); PUT(touch_size, tsize);
  {
    // depth renderer: every primitive (non-mesh) geom in model order
    std::vector<int> rt, rb, rc;
    std::vector<double> rp, rq, rs, rr;
    for (int g = 0; g < ngeom_all; g++) {
      if (gtype[g] == 7) continue;
      rt.push_back(gtype[g]); rb.push_back(gbody[g]); rc.push_back(gmap[g]);
      for (int k = 0; k < 3; k++) { rp.push_back(gpos[3 * g + k]); rs.push_back(gsize[3 * g + k]); }
      for (int k = 0; k < 4; k++) rq.push_back(gquat[4 * g + k]);
      rr.push_back(grb[g]);
    }
    m.nrgeom = (int)rt.size();
    PUT(rg_type, rt); PUT(rg_body, rb); PUT(rg_cgeom, rc); PUT(rg_pos, rp); PUT(rg_quat, rq);
    PUT(rg_size, rs); PUT(rg_rbound, rr);
  }
  {
    // per-object "some parameter overrides this" flags (kinematics applies those overrides inline)
    std::vector<int> bo(nbody, 0), so(std::max(nsite, 1), 0), go(std::max(m.ngeom, 1), 0);
    for (int p = 0; p < m.nparam; p++) {
      if (pf[p] == 0 || pf[p] == 1 || pf[p] == 3) bo[po[p]] = 1;
      else if (pf[p] == 2) so[po[p]] = 1;
      else if (pf[p] == 4 || pf[p] == 5) go[po[p]] = 1;
    }
    PUT(body_ovr, bo); PUT(site_ovr, so); PUT(geom_ovr, go);
  }
  PUT(task_idx, tidx); PUT(param_field, pf); PUT(param_obj, po); PUT(param_comp, pc);
  PUT(act_mid, tof(B.f("task_act_mid"))); PUT(act_rng, tof(B.f("task_act_rng")));
  PUT(param_default, tof(B.f("task_param_default")));
  PUT(param_draw, B.i("task_param_draw"));
  std::vector<double> dlo = B.f("task_draw_lo"), dhi = B.f("task_draw_hi");
  m.ndraw = (int)dlo.size();
  if (m.ndraw > 8) return fail(AW_EUNSUPPORTED, "too many reset draws");
  PUT(draw_lo, tof(dlo)); PUT(draw_hi, tof(dhi));
  return AW_OK;
}

#endif  // AW_TASK_TU

// The wide tier's launcher table, defined in the -DAW_WIDE -DAW_TASK_TU=TASK translation unit
// (k_step_wide<TASK>): `run` drains the queue that the fast launch before it filled.
struct WideOps {
  int (*slots)(int device);
  void (*run)(aw_handle*, const float*, float*, float*, uint8_t*, uint8_t*, float*, int, uint64_t, hipStream_t);
  void (*dump)(aw_handle*, int, const float*, float*, hipStream_t);   // aw_forward_dump_wide
};
template <int TASK> const WideOps* wide_ops();

#ifdef AW_WIDE
template <int TASK>
static int wide_slots(int device) {
  int per_cu = 0, cus = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_step_wide<TASK>, 64, 0);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  return std::max(per_cu, 1) * std::max(cus, 1);
}
template <int TASK>
static void launch_wide(aw_handle* h, const float* a, float* obs, float* rew, uint8_t* done, uint8_t* goal,
                        float* tobs, int autoreset, uint64_t seed, hipStream_t st) {
  hipLaunchKernelGGL((k_step_wide<TASK>), dim3(h->wide_grid), dim3(64), 0, st, (const DModel*)h->dmhdr_wide, a, obs, rew,
                     done, goal, tobs, autoreset, seed, h->next_env + 8, h->nenv);
}
template <int TASK>
static void launch_dump_wide(aw_handle* h, int env, const float* ctrl, float* out, hipStream_t st) {
  DModel mw = h->m;
  mw.jspill = h->jspill_wide;   // the dense rows past JL in the wide tier's spill block (slot 0)
  hipLaunchKernelGGL((k_dump_wide<TASK>), dim3(1), dim3(64), 0, st, mw, h->st, env, ctrl, out);
}
template <int TASK> const WideOps* wide_ops() {
  static const WideOps ops = {wide_slots<TASK>, launch_wide<TASK>, launch_dump_wide<TASK>};
  return &ops;
}
template const WideOps* wide_ops<AW_TASK_TU>();
#else
// resident k_step workgroups on the handle's device (occupancy x CUs): the persistent grid
template <int TASK>
static int step_slots(int device) {
  int per_cu = 0, cus = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_step<TASK>, 64, 0);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  return std::max(per_cu, 1) * std::max(cus, 1);
}
// Claim order for the next k_step launch (longest processing time first): per XCD class c (k_step's
// env range [n c / 8, n (c + 1) / 8)) the envs are bucketed by their last env-step's shader cycles
// on a quarter-octave scale and written costliest bucket first into perm (positions of the same
// range), so the launch's last claims are its cheapest envs.  One workgroup per class.
static __device__ int cost_bucket(unsigned c) {
  if (c < (1u << 16)) return 0;
  const int e = 31 - __clz(c);                       // floor(log2 c) >= 16
  const int key = 4 * e + (int)((c >> (e - 2)) & 3);  // quarter octaves
  const int b = key - 4 * 16;
  return b > 63 ? 63 : b;
}
static __global__ void __launch_bounds__(1024) k_order(const unsigned* __restrict__ cost, int* __restrict__ perm, int n) {
  const int c = blockIdx.x;
  const int lo = (int)((long long)n * c / 8), hi = (int)((long long)n * (c + 1) / 8);
  __shared__ int hist[64];
  if (threadIdx.x < 64) hist[threadIdx.x] = 0;
  __syncthreads();
  for (int i = lo + (int)threadIdx.x; i < hi; i += blockDim.x) atomicAdd(&hist[cost_bucket(cost[i])], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int b = 63; b >= 0; b--) { const int h = hist[b]; hist[b] = acc; acc += h; }
  }
  __syncthreads();
  for (int i = lo + (int)threadIdx.x; i < hi; i += blockDim.x) {
    const int k = atomicAdd(&hist[cost_bucket(cost[i])], 1);
    perm[lo + k] = i;
  }
}

// every launch that runs a fast-tier forward clears the wide queue first and drains it after
static void clear_queue(aw_handle* h, bool counters, hipStream_t st) {
  if (counters) (void)hipMemsetAsync(h->next_env, 0, 10 * sizeof(int), st);   // XCD counters + queue heads
  else (void)hipMemsetAsync(h->next_env + 8, 0, 2 * sizeof(int), st);
}
template <int TASK>
static void launch_step(aw_handle* h, const float* a, float* obs, float* rew, uint8_t* done, uint8_t* goal,
                        float* tobs, int autoreset, uint64_t seed, hipStream_t st) {
  // grid = the handle's persistent slot count (aw_create / aw_set_option), capped at nenv
  const int grid = std::min(h->nenv, h->slots);
  clear_queue(h, grid < h->nenv, st);
  if (grid < h->nenv && (grid & 7) == 0)   // the XCD-class claim path (k_step xmap)
    hipLaunchKernelGGL(k_order, dim3(8), dim3(1024), 0, st, reinterpret_cast<const unsigned*>(h->next_env + 10 + h->nenv),
                       h->next_env + 10 + 2 * h->nenv, h->nenv);
  hipLaunchKernelGGL((k_step<TASK>), dim3(grid), dim3(64), 0, st, h->m, (const DModel*)h->dmhdr, h->st, h->nenv, a, obs, rew, done,
                     goal, tobs, autoreset, seed, h->next_env);
  wide_ops<TASK>()->run(h, a, obs, rew, done, goal, tobs, autoreset, seed, st);
}
template <int TASK>
static void launch_reset(aw_handle* h, const uint8_t* mask, const float* params, uint64_t seed, float* obs,
                         hipStream_t st) {
  clear_queue(h, false, st);
  hipLaunchKernelGGL((k_reset<TASK>), dim3(h->nenv), dim3(64), 0, st, h->m, h->st, h->nenv, mask, params, seed, obs,
                     h->next_env + 8);
  wide_ops<TASK>()->run(h, nullptr, obs, nullptr, nullptr, nullptr, nullptr, 0, seed, st);
}
template <int TASK>
static void launch_set(aw_handle* h, const float* q, const float* v, const float* w, const float* p, float* obs,
                       hipStream_t st) {
  clear_queue(h, false, st);
  hipLaunchKernelGGL((k_set_state<TASK>), dim3(h->nenv), dim3(64), 0, st, h->m, h->st, h->nenv, q, v, w, p, obs,
                     h->next_env + 8);
  wide_ops<TASK>()->run(h, nullptr, obs, nullptr, nullptr, nullptr, nullptr, 0, 0, st);
}
template <int TASK>
static void launch_dump(aw_handle* h, int env, const float* ctrl, float* out, hipStream_t st) {
  hipLaunchKernelGGL((k_dump<TASK>), dim3(1), dim3(64), 0, st, h->m, h->st, env, ctrl, out);
}

template <int TASK>
static void launch_depth(aw_handle* h, const CamRec& cam, int W, int H, float* out, hipStream_t st) {
  hipLaunchKernelGGL((k_depth<TASK>), dim3(h->nenv), dim3(256), 0, st, h->m, h->st, h->nenv, cam, W, H, out);
}
#endif  // AW_WIDE

// The launchers of one task, behind one table.  Split build: task_ops<TASK> is defined (and with
// it every kernel of TASK instantiated) only in the -DAW_TASK_TU=TASK translation unit; the API
// unit sees the declaration and calls it across the link.  The wide tier's table (wide_ops) comes
// from the -DAW_WIDE unit of the same task in every build.
struct TaskOps {
  int (*slots)(int device);
  void (*step)(aw_handle*, const float*, float*, float*, uint8_t*, uint8_t*, float*, int, uint64_t, hipStream_t);
  void (*reset)(aw_handle*, const uint8_t*, const float*, uint64_t, float*, hipStream_t);
  void (*set)(aw_handle*, const float*, const float*, const float*, const float*, float*, hipStream_t);
  void (*dump)(aw_handle*, int, const float*, float*, hipStream_t);
  void (*depth)(aw_handle*, const CamRec&, int, int, float*, hipStream_t);
};
template <int TASK> const TaskOps* task_ops();
#if !defined(AW_API_TU) && !defined(AW_WIDE)
template <int TASK> const TaskOps* task_ops() {
  static const TaskOps ops = {step_slots<TASK>, launch_step<TASK>, launch_reset<TASK>, launch_set<TASK>,
                              launch_dump<TASK>, launch_depth<TASK>};
  return &ops;
}
#endif
#if defined(AW_TASK_TU) && !defined(AW_WIDE)
template const TaskOps* task_ops<AW_TASK_TU>();
#endif
#ifndef AW_TASK_TU

// kernels are instantiated per task (the dof tree of aw_trees.h is a template argument)
#ifdef AW_ONLY_TASK
#define DISPATCH_TASK(T, CALL)                                                     \
  switch (T) {                                                                     \
    case AW_ONLY_TASK: CALL(AW_ONLY_TASK); break;                                  \
    default: return fail(AW_EUNSUPPORTED, "task not instantiated in this build");  \
  }
#else
#define DISPATCH_TASK(T, CALL)                                                     \
  switch (T) {                                                                     \
    case 0: CALL(0); break;                                                        \
    case 1: CALL(1); break;                                                        \
    case 2: CALL(2); break;                                                        \
    case 3: CALL(3); break;                                                        \
    default: return fail(AW_EUNSUPPORTED, "task kind not instantiated (0..3)");   \
  }
#endif

// the model's dof tree must be the compiled one of its task (aw_trees.h, tools/gen_trees.py)
template <int TASK>
static bool tree_matches(const std::vector<int>& par) {
  if ((int)par.size() != TreeDef<TASK>::NV) return false;
  for (int j = 0; j < TreeDef<TASK>::NV; j++)
    if (par[j] != TreeDef<TASK>::parent[j]) return false;
  return true;
}
static int check_tree(const Blob& B, int task_kind) {
  const std::vector<int> par = B.i("dof_parentid");
  bool ok = false;
  switch (task_kind) {
    case 0: ok = tree_matches<0>(par); break;
    case 1: ok = tree_matches<1>(par); break;
    case 2: ok = tree_matches<2>(par); break;
    case 3: ok = tree_matches<3>(par); break;
    default: return fail(AW_EUNSUPPORTED, "unknown task kind");
  }
  if (!ok) return fail(AW_EUNSUPPORTED, "model dof tree differs from the compiled tree of its task "
                                        "(mj_envs_amd/csrc/aw_trees.h: run tools/gen_trees.py and rebuild)");
  return AW_OK;
}

// the fast tier's dense-row capacity of the handle's task: per task in the split build (each task's
// translation unit compiles its own, aw_common.h), the single value of a one-TU diagnostic build
static int fast_maxdense_handle(const aw_handle* h) {
#ifdef AW_API_TU
  return fast_maxdense_of(h->m.task_kind);
#else
  (void)h;
  return FAST_MAXDENSE;
#endif
}

// persistent grid of the k_step instantiation the handle currently selects
static int update_slots(aw_handle* h) {
  if (h->grid_env >= 0) {
    h->slots = h->grid_env > 0 ? h->grid_env : (1 << 30);
    return AW_OK;
  }
#define CALL(TT) (h->slots = task_ops<TT>()->slots(h->device))
  DISPATCH_TASK(h->m.task_kind, CALL)
#undef CALL
  return AW_OK;
}

extern "C" {

const char* aw_last_error(void) { return g_err.c_str(); }

static void free_handle(aw_handle* h) {
  if (!h) return;
  if (h->dmodel) (void)hipFree(h->dmodel);
  if (h->dmhdr) (void)hipFree(h->dmhdr);
  if (h->dstate) (void)hipFree(h->dstate);
  if (h->m.jspill) (void)hipFree(h->m.jspill);
  if (h->next_env) (void)hipFree(h->next_env);
  if (h->dmhdr_wide) (void)hipFree(h->dmhdr_wide);
  if (h->jspill_wide) (void)hipFree(h->jspill_wide);
  delete h;
}

// carve the per-env state arrays out of one allocation (each 256-byte aligned)
static size_t layout_state(aw_handle* h, char* base) {
  size_t N = (size_t)h->nenv, nq = h->m.nq, nv = h->m.nv, np = std::max(h->m.nparam, 1);
  uintptr_t p = (uintptr_t)base;   // base == nullptr: dry run, only the size is used
  auto take = [&](size_t b) { uintptr_t r = p; p += (b + 255) & ~size_t(255); return (char*)r; };
  DState& st = h->st;
  st.qpos = (float*)take(N * nq * 4); st.qvel = (float*)take(N * nv * 4); st.warm = (float*)take(N * nv * 4);
  st.params = (float*)take(N * np * 4); st.ep_len = (int*)take(N * 4); st.ep_ret = (float*)take(N * 4);
  st.ep_goal = (int*)take(N * 4); st.episode = (int*)take(N * 4); st.status = (unsigned*)take(N * 4);
  st.last_ret = (float*)take(N * 4); st.last_goal = (int*)take(N * 4); st.last_len = (int*)take(N * 4);
  st.status_acc = (unsigned*)take(N * 4); st.sum_ret = (float*)take(N * 4); st.n_success = (int*)take(N * 4);
  return (size_t)(p - (uintptr_t)base);
}

int aw_create(const void* blob, size_t nbytes, int n_envs, int device, aw_handle** out) {
  if (!blob || !out || n_envs <= 0) return fail(AW_EINVAL, "aw_create: bad arguments");
  *out = nullptr;
  Blob B{blob, nbytes};
  std::unique_ptr<aw_handle, void (*)(aw_handle*)> h(new aw_handle(), free_handle);
  h->device = device;
  h->nenv = n_envs;
  std::unique_ptr<MData> md(new MData());   // value-initialised: zero
  if (int rc = build_model(B, h->m, *md)) return rc;
  h->NV = h->m.nv;
  if (int rc = check_tree(B, h->m.task_kind)) return rc;
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipMalloc(&h->dmodel, sizeof(MData)));
  HIPCHK(hipMemcpy(h->dmodel, md.get(), sizeof(MData), hipMemcpyHostToDevice));
  h->m.d = (const MData*)h->dmodel;
  // fast tier: one spill block per workgroup of k_reset / k_set_state (one per env)
  HIPCHK(hipMalloc((void**)&h->m.jspill, (size_t)n_envs * JSPILL_FAST * sizeof(float)));
  HIPCHK(hipMalloc(&h->dmhdr, sizeof(DModel) + sizeof(DState)));
  const size_t nq = 10 + 3 * (size_t)n_envs;   // + per-env costs and the claim permutation (k_order)
  HIPCHK(hipMalloc((void**)&h->next_env, nq * sizeof(int)));
  HIPCHK(hipMemset(h->next_env, 0, nq * sizeof(int)));
  // wide tier: its persistent grid and one spill block per wide workgroup
#define CALL(TT) (h->wide_grid = std::min(n_envs, wide_ops<TT>()->slots(device)))
  DISPATCH_TASK(h->m.task_kind, CALL)
#undef CALL
  HIPCHK(hipMalloc((void**)&h->jspill_wide, (size_t)h->wide_grid * JSPILL_WIDE * sizeof(float)));
  HIPCHK(hipMalloc(&h->dmhdr_wide, sizeof(DModel) + sizeof(DState)));
  const size_t bytes = layout_state(h.get(), nullptr);   // dry run: sizes only
  HIPCHK(hipMalloc(&h->dstate, bytes));
  HIPCHK(hipMemset(h->dstate, 0, bytes));
  layout_state(h.get(), (char*)h->dstate);
  // default params for every env
  size_t N = (size_t)n_envs, np = std::max(h->m.nparam, 1);
  std::vector<float> prm(N * np, 0.f);
  std::vector<double> def = B.f("task_param_default");
  for (size_t e = 0; e < N; e++)
    for (int k = 0; k < h->m.nparam; k++) prm[e * np + k] = (float)def[k];
  HIPCHK(hipMemcpy(h->st.params, prm.data(), prm.size() * 4, hipMemcpyHostToDevice));
  if (int rc2 = upload_header(h.get())) return rc2;
  if (const char* e = getenv("AW_STEP_GRID")) h->grid_env = std::max(atoi(e), 0);
  if (int rc3 = update_slots(h.get())) return rc3;
  *out = h.release();
  return AW_OK;
}

int aw_destroy(aw_handle* h) {
  if (!h) return AW_OK;
  (void)hipSetDevice(h->device);
  free_handle(h);
  return AW_OK;
}

int aw_dims(const aw_handle* h, int* d) {
  if (!h || !d) return fail(AW_EINVAL, "aw_dims: null");
  const DModel& m = h->m;
  int v[AW_NDIMS] = {m.nq, m.nv, m.nu, m.obs_dim, m.nparam, m.frame_skip, m.horizon, m.task_kind, h->nenv,
                     m.nbody, m.nsite, m.ngeom, m.npairall, NCONMAX, NJMAX, WIDE_MAXDENSE, std::min(h->slots, h->nenv),
                     FAST_MAXCON, 64 * FAST_NRL, fast_maxdense_handle(h), h->wide_grid};
  memcpy(d, v, sizeof(v));
  return AW_OK;
}

int aw_set_option(aw_handle* h, int disableflags, int iterations, int noslip_iterations) {
  if (!h) return fail(AW_EINVAL, "aw_set_option: null");
  if (disableflags >= 0 && (disableflags & ~0xFFFF))
    return fail(AW_EUNSUPPORTED, "aw_set_option: only MuJoCo's disable bits 0..15 (the MPR collider always runs in fp64)");
  if (disableflags >= 0) h->m.disableflags = disableflags;
  if (iterations >= 0) h->m.iterations = iterations;
  if (noslip_iterations >= 0) h->m.noslip_iterations = noslip_iterations;
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());   // steps already queued on any stream read the old header
  return upload_header(h);
}

int aw_set_tier(aw_handle* h, int mode) {
  if (!h || mode < 0 || mode > 1) return fail(AW_EINVAL, "aw_set_tier: mode must be 0 (automatic) or 1 (wide only)");
  h->m.force_wide = mode;
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());   // queued launches read the old header
  return upload_header(h);
}

int aw_set_fault(aw_handle* h, int kind, int arg) {
  if (!h || kind < 0 || kind > 2) return fail(AW_EINVAL, "aw_set_fault: kind must be 0 (none), 1 (margin) or 2 (stick row)");
  if (kind == 2 && (arg < 0 || arg >= h->m.nfl)) return fail(AW_EINVAL, "aw_set_fault: no such frictionloss row");
  if (kind == 1 && (arg < -1000 || arg > 1000)) return fail(AW_EINVAL, "aw_set_fault: margin shift beyond 1 mm");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());   // queued launches read the old table / header
  MData* dm = (MData*)h->dmodel;
  const int np = h->m.npairall;
  if (h->fault_cls.empty()) {      // the table as built, saved once
    h->fault_margin0.resize(np); h->fault_rb0.resize(np); h->fault_margin64_0.resize(np); h->fault_cls.resize(np);
    HIPCHK(hipMemcpy(h->fault_margin0.data(), dm->cp_margin, np * sizeof(float), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(h->fault_rb0.data(), dm->cp_rb, np * sizeof(float), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(h->fault_margin64_0.data(), dm->cp_margin64, np * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(h->fault_cls.data(), dm->cp_class, np * sizeof(int), hipMemcpyDeviceToHost));
  }
  std::vector<float> mg = h->fault_margin0, rb = h->fault_rb0;
  std::vector<double> mg64 = h->fault_margin64_0;
  if (kind == 1) {
    // every sphere / capsule pair (collider class 1): activation, the fp64 decision, the rows'
    // includemargin and the broadphase radius all see the shifted margin
    const double dl = 1e-6 * arg;
    for (int p = 0; p < np; p++)
      if (h->fault_cls[p] == 1) {
        mg64[p] += dl;
        mg[p] = (float)mg64[p];
        rb[p] = (float)((double)rb[p] + dl);
      }
  }
  HIPCHK(hipMemcpy(dm->cp_margin, mg.data(), np * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dm->cp_rb, rb.data(), np * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dm->cp_margin64, mg64.data(), np * sizeof(double), hipMemcpyHostToDevice));
  h->m.fault_flrow = kind == 2 ? arg : -1;
  return upload_header(h);
}

int aw_reset(aw_handle* h, const uint8_t* mask, const float* params, uint64_t seed, float* obs, void* stream) {
  if (!h) return fail(AW_EINVAL, "aw_reset: null");
  HIPCHK(hipSetDevice(h->device));
#define CALL(TT) task_ops<TT>()->reset(h, mask, params, seed, obs, (hipStream_t)stream)
  DISPATCH_TASK(h->m.task_kind, CALL)
#undef CALL
  HIPCHK(hipGetLastError());
  return AW_OK;
}

int aw_step(aw_handle* h, const float* actions, float* obs, float* reward, uint8_t* done, uint8_t* goal,
            float* terminal_obs, int autoreset, uint64_t seed, void* stream) {
  if (!h || !actions || !obs || !reward || !done || !goal) return fail(AW_EINVAL, "aw_step: null buffer");
  HIPCHK(hipSetDevice(h->device));
#define CALL(TT) task_ops<TT>()->step(h, actions, obs, reward, done, goal, terminal_obs, autoreset, seed, (hipStream_t)stream)
  DISPATCH_TASK(h->m.task_kind, CALL)
#undef CALL
  HIPCHK(hipGetLastError());
  return AW_OK;
}

int aw_random_actions(aw_handle* h, uint64_t seed, uint64_t step, float* actions, void* stream) {
  if (!h || !actions) return fail(AW_EINVAL, "aw_random_actions: null");
  HIPCHK(hipSetDevice(h->device));
  int bs = 256, nb = (h->nenv + bs - 1) / bs;
  hipLaunchKernelGGL(k_random_actions, dim3(nb), dim3(bs), 0, (hipStream_t)stream, h->nenv, h->m.nu, seed, step,
                     (uint64_t)h->m.env_offset, actions);
  HIPCHK(hipGetLastError());
  return AW_OK;
}

int aw_get_state(aw_handle* h, float* qpos, float* qvel, float* warm, float* params, void* stream) {
  if (!h) return fail(AW_EINVAL, "aw_get_state: null");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  size_t N = h->nenv;
  if (qpos) HIPCHK(hipMemcpyAsync(qpos, h->st.qpos, N * h->m.nq * 4, hipMemcpyDeviceToDevice, st));
  if (qvel) HIPCHK(hipMemcpyAsync(qvel, h->st.qvel, N * h->m.nv * 4, hipMemcpyDeviceToDevice, st));
  if (warm) HIPCHK(hipMemcpyAsync(warm, h->st.warm, N * h->m.nv * 4, hipMemcpyDeviceToDevice, st));
  if (params && h->m.nparam)
    HIPCHK(hipMemcpyAsync(params, h->st.params, N * h->m.nparam * 4, hipMemcpyDeviceToDevice, st));
  return AW_OK;
}

int aw_set_state(aw_handle* h, const float* qpos, const float* qvel, const float* warm, const float* params,
                 float* obs, void* stream) {
  if (!h) return fail(AW_EINVAL, "aw_set_state: null");
  HIPCHK(hipSetDevice(h->device));
#define CALL(TT) task_ops<TT>()->set(h, qpos, qvel, warm, params, obs, (hipStream_t)stream)
  DISPATCH_TASK(h->m.task_kind, CALL)
#undef CALL
  HIPCHK(hipGetLastError());
  return AW_OK;
}

int aw_status(aw_handle* h, uint32_t* last, uint32_t* sticky, void* stream) {
  if (!h || (!last && !sticky)) return fail(AW_EINVAL, "aw_status: null");
  HIPCHK(hipSetDevice(h->device));
  const size_t b = (size_t)h->nenv * 4;
  if (last) HIPCHK(hipMemcpyAsync(last, h->st.status, b, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  if (sticky) HIPCHK(hipMemcpyAsync(sticky, h->st.status_acc, b, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return AW_OK;
}

int aw_clear_status(aw_handle* h, void* stream) {
  if (!h) return fail(AW_EINVAL, "aw_clear_status: null");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipMemsetAsync(h->st.status_acc, 0, (size_t)h->nenv * 4, (hipStream_t)stream));
  return AW_OK;
}

int aw_set_env_offset(aw_handle* h, uint64_t env_offset) {
  if (!h) return fail(AW_EINVAL, "aw_set_env_offset: null");
  h->m.env_offset = env_offset;
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());   // steps already queued read the old header
  return upload_header(h);
}

int aw_get_episode(aw_handle* h, int32_t* ep_len, float* ep_ret, int32_t* ep_goal, int32_t* episodes,
                   void* stream) {
  if (!h) return fail(AW_EINVAL, "aw_get_episode: null");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  const size_t b = (size_t)h->nenv * 4;
  if (ep_len) HIPCHK(hipMemcpyAsync(ep_len, h->st.ep_len, b, hipMemcpyDeviceToDevice, st));
  if (ep_ret) HIPCHK(hipMemcpyAsync(ep_ret, h->st.ep_ret, b, hipMemcpyDeviceToDevice, st));
  if (ep_goal) HIPCHK(hipMemcpyAsync(ep_goal, h->st.ep_goal, b, hipMemcpyDeviceToDevice, st));
  if (episodes) HIPCHK(hipMemcpyAsync(episodes, h->st.episode, b, hipMemcpyDeviceToDevice, st));
  return AW_OK;
}

int aw_set_episode(aw_handle* h, const int32_t* ep_len, const float* ep_ret, const int32_t* ep_goal,
                   const int32_t* episodes, void* stream) {
  if (!h) return fail(AW_EINVAL, "aw_set_episode: null");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  const size_t b = (size_t)h->nenv * 4;
  if (ep_len) HIPCHK(hipMemcpyAsync(h->st.ep_len, ep_len, b, hipMemcpyDeviceToDevice, st));
  if (ep_ret) HIPCHK(hipMemcpyAsync(h->st.ep_ret, ep_ret, b, hipMemcpyDeviceToDevice, st));
  if (ep_goal) HIPCHK(hipMemcpyAsync(h->st.ep_goal, ep_goal, b, hipMemcpyDeviceToDevice, st));
  if (episodes) HIPCHK(hipMemcpyAsync(h->st.episode, episodes, b, hipMemcpyDeviceToDevice, st));
  return AW_OK;
}

int aw_episode_totals(aw_handle* h, int32_t* episodes, float* sum_return, int32_t* successes, void* stream) {
  if (!h) return fail(AW_EINVAL, "aw_episode_totals: null");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  const size_t b = (size_t)h->nenv * 4;
  if (episodes) HIPCHK(hipMemcpyAsync(episodes, h->st.episode, b, hipMemcpyDeviceToDevice, st));
  if (sum_return) HIPCHK(hipMemcpyAsync(sum_return, h->st.sum_ret, b, hipMemcpyDeviceToDevice, st));
  if (successes) HIPCHK(hipMemcpyAsync(successes, h->st.n_success, b, hipMemcpyDeviceToDevice, st));
  return AW_OK;
}

int aw_set_episode_totals(aw_handle* h, const int32_t* episodes, const float* sum_return, const int32_t* successes,
                          void* stream) {
  if (!h) return fail(AW_EINVAL, "aw_set_episode_totals: null");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  const size_t b = (size_t)h->nenv * 4;
  if (episodes) HIPCHK(hipMemcpyAsync(h->st.episode, episodes, b, hipMemcpyDeviceToDevice, st));
  if (sum_return) HIPCHK(hipMemcpyAsync(h->st.sum_ret, sum_return, b, hipMemcpyDeviceToDevice, st));
  if (successes) HIPCHK(hipMemcpyAsync(h->st.n_success, successes, b, hipMemcpyDeviceToDevice, st));
  return AW_OK;
}

int aw_episode_stats(aw_handle* h, float* last_return, int32_t* last_goal, int32_t* last_len, int32_t* episodes,
                     void* stream) {
  if (!h) return fail(AW_EINVAL, "aw_episode_stats: null");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  size_t b = (size_t)h->nenv * 4;
  if (last_return) HIPCHK(hipMemcpyAsync(last_return, h->st.last_ret, b, hipMemcpyDeviceToDevice, st));
  if (last_goal) HIPCHK(hipMemcpyAsync(last_goal, h->st.last_goal, b, hipMemcpyDeviceToDevice, st));
  if (last_len) HIPCHK(hipMemcpyAsync(last_len, h->st.last_len, b, hipMemcpyDeviceToDevice, st));
  if (episodes) HIPCHK(hipMemcpyAsync(episodes, h->st.episode, b, hipMemcpyDeviceToDevice, st));
  return AW_OK;
}

int aw_task_eval(aw_handle* h, int n, const float* qpos, const float* qvel, const float* xpos, const float* xquat,
                 const float* sxpos, const float* touch, float* obs, float* reward, uint8_t* done, uint8_t* goal,
                 void* stream) {
  if (!h || n <= 0) return fail(AW_EINVAL, "aw_task_eval: bad arguments");
  HIPCHK(hipSetDevice(h->device));
  hipLaunchKernelGGL(k_task_eval, dim3(n), dim3(64), 0, (hipStream_t)stream, h->m, n, qpos, qvel, xpos, xquat,
                     sxpos, touch, obs, reward, done, goal);
  HIPCHK(hipGetLastError());
  return AW_OK;
}

int aw_forward_dump(aw_handle* h, int env, const float* ctrl, float* out, void* stream) {
  if (!h || !out || env < 0 || env >= h->nenv) return fail(AW_EINVAL, "aw_forward_dump: bad arguments");
  HIPCHK(hipSetDevice(h->device));
#define CALL(TT) task_ops<TT>()->dump(h, env, ctrl, out, (hipStream_t)stream)
  DISPATCH_TASK(h->m.task_kind, CALL)
#undef CALL
  HIPCHK(hipGetLastError());
  return AW_OK;
}

int aw_forward_dump_wide(aw_handle* h, int env, const float* ctrl, float* out, void* stream) {
  if (!h || !out || env < 0 || env >= h->nenv) return fail(AW_EINVAL, "aw_forward_dump_wide: bad arguments");
  HIPCHK(hipSetDevice(h->device));
#define CALL(TT) wide_ops<TT>()->dump(h, env, ctrl, out, (hipStream_t)stream)
  DISPATCH_TASK(h->m.task_kind, CALL)
#undef CALL
  HIPCHK(hipGetLastError());
  return AW_OK;
}

int aw_render_depth(aw_handle* h, const float* cam, int width, int height, float* out, void* stream) {
  if (!h || !cam || !out || width <= 0 || height <= 0 || width > 4096 || height > 4096)
    return fail(AW_EINVAL, "aw_render_depth: bad arguments");
  HIPCHK(hipSetDevice(h->device));
  CamRec c;
  memcpy(c.c, cam, sizeof(c.c));   // host array: the camera record travels as a kernel argument
#define CALL(TT) task_ops<TT>()->depth(h, c, width, height, out, (hipStream_t)stream)
  DISPATCH_TASK(h->m.task_kind, CALL)
#undef CALL
  HIPCHK(hipGetLastError());
  return AW_OK;
}

int aw_policy_mlp(int n, int in_dim, int hidden, int out_dim, const float* params, const float* obs, float* act,
                  int sample, uint64_t seed, uint64_t step, uint64_t env_offset, void* stream) {
  if (n <= 0 || !params || !obs || !act || in_dim <= 0 || in_dim > MLP_IMAX || out_dim <= 0 || out_dim > MLP_OMAX)
    return fail(AW_EINVAL, "aw_policy_mlp: bad arguments");
  const int bs = 256, nb = (n + bs - 1) / bs;
  hipStream_t st = (hipStream_t)stream;
  switch (hidden) {
    case 32: hipLaunchKernelGGL(k_mlp<32>, dim3(nb), dim3(bs), 0, st, n, in_dim, out_dim, params, obs, act, sample, seed, step, env_offset); break;
    case 64: hipLaunchKernelGGL(k_mlp<64>, dim3(nb), dim3(bs), 0, st, n, in_dim, out_dim, params, obs, act, sample, seed, step, env_offset); break;
    default: return fail(AW_EUNSUPPORTED, "aw_policy_mlp: hidden width must be 32 or 64 (two hidden layers)");
  }
  HIPCHK(hipGetLastError());
  return AW_OK;
}

int aw_collide_test(aw_handle* h, int n, const int32_t* types, const float* pos, const float* mat, const float* size,
                    const float* margin, float* out, int32_t* count, double* out64, void* stream) {
  if (!h || n <= 0 || !types || !pos || !mat || !size || !margin || !out || !count)
    return fail(AW_EINVAL, "aw_collide_test: bad arguments");
  HIPCHK(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_collide_test, dim3(n), dim3(64), 0, st, h->m, n, types, pos, mat, size, margin, out, count, out64);
  HIPCHK(hipGetLastError());
  return AW_OK;
}

int aw_stage_profile(unsigned long long* out, int reset) {
#ifdef AW_STAGE_PROF
  if (out) HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stage_prof), sizeof(unsigned long long) * AW_NPROF));
  if (reset) {
    unsigned long long z[AW_NPROF] = {};
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_stage_prof), z, sizeof(z)));
  }
  return AW_OK;
#else
  (void)out; (void)reset;
  return fail(AW_EUNSUPPORTED, "library built without -DAW_STAGE_PROF");
#endif
}

}  // extern "C"
#endif  // !AW_TASK_TU
