// aw_task.h -- per-task observation / reward / reset sampling on the wave (fp32).
//
// Restates the reference task layer:
//   hammer   hand_manipulation_suite/hammer_v0.py:54-104   (obs 46)
//   door     hand_manipulation_suite/door_v0.py:55-101     (obs 39)
//   pen      hand_manipulation_suite/pen_v0.py:65-113      (obs 45, done on drop)
//   relocate hand_manipulation_suite/relocate_v0.py:46-83  (obs 39)
//   quat2euler / euler2quat  utils/quatmath.py:60-164
// Obs/reward read the kinematics of the LAST substep's forward pass (pre-integration) and the
// post-integration qpos/qvel, exactly as the reference does after mj_step.
#pragma once
#include "aw_common.h"

namespace aw {

AW_DEV void quat2euler(const float* q, float* e) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  float Nq = w * w + x * x + y * y + z * z;
  float m[9];
  if (Nq > 2.220446049250313e-16f) {
    float s = 2.0f / Nq;
    float X = x * s, Y = y * s, Z = z * s;
    float wX = w * X, wY = w * Y, wZ = w * Z, xX = x * X, xY = x * Y, xZ = x * Z;
    float yY = y * Y, yZ = y * Z, zZ = z * Z;
    m[0] = 1.f - (yY + zZ); m[1] = xY - wZ; m[2] = xZ + wY;
    m[3] = xY + wZ; m[4] = 1.f - (xX + zZ); m[5] = yZ - wX;
    m[6] = xZ - wY; m[7] = yZ + wX; m[8] = 1.f - (xX + yY);
  } else {
    for (int k = 0; k < 9; k++) m[k] = (k % 4 == 0) ? 1.f : 0.f;
  }
  float cy = sqrtf(m[8] * m[8] + m[5] * m[5]);
  bool cond = cy > 8.881784197001252e-16f;
  e[2] = cond ? -atan2f(m[1], m[0]) : -atan2f(-m[3], m[4]);
  e[1] = -atan2f(-m[2], cy);
  e[0] = cond ? -atan2f(m[5], m[8]) : 0.f;
}

// utils/quatmath.py:60-76 (reference convention)
AW_DEV void euler2quat_ref(const float* eu, float* q) {
  float ai = eu[2] / 2, aj = -eu[1] / 2, ak = eu[0] / 2;
  float si = sinf(ai), sj = sinf(aj), sk = sinf(ak);
  float ci = cosf(ai), cj = cosf(aj), ck = cosf(ak);
  float cc = ci * ck, cs = ci * sk, sc = si * ck, ss = si * sk;
  q[0] = cj * cc + sj * ss;
  q[3] = cj * sc - sj * cs;
  q[2] = -(cj * ss + sj * cc);
  q[1] = cj * cs - sj * sc;
}

AW_DEV float dist3(const float* a, const float* b) {
  float d[3];
  sub3(d, a, b);
  return norm3(d);
}

// writes obs[0..obs_dim) into s.rowbuf (LDS); lane-parallel qpos copies
AW_DEV void task_obs(const DModel& m, Env& s, int lane, float* out) {
  const int* id = m.d->task_idx;
  const int nq = m.nq, nv = m.nv;
  switch (m.task_kind) {
    case 0: {  // hammer
      if (lane < nq - 6) out[lane] = s.qpos[lane];
      if (lane < 6) out[nq - 6 + lane] = clampf(s.qvel[nv - 6 + lane], -1.f, 1.f);
      int o = nq;
      if (lane < 3) {
        out[o + lane] = s.sxpos[id[0]][lane];
        out[o + 3 + lane] = s.xpos[id[1]][lane];
        out[o + 9 + lane] = s.sxpos[id[3]][lane];
      }
      if (lane == 0) {
        float e[3];
        quat2euler(s.xquat[id[1]], e);
        out[o + 6] = e[0]; out[o + 7] = e[1]; out[o + 8] = e[2];
        out[o + 12] = clampf(s.touch[0], -1.f, 1.f);
      }
      break;
    }
    case 1: {  // door
      if (lane >= 1 && lane < nq - 2) out[lane - 1] = s.qpos[lane];
      int o = nq - 3;
      if (lane == 0) {
        out[o] = s.qpos[nq - 1];
        float door = s.qpos[id[2]];
        out[o + 1] = door;
        out[o + 11] = door > 1.0f ? 1.f : -1.f;
      }
      if (lane < 3) {
        float p = s.sxpos[id[0]][lane], h = s.sxpos[id[1]][lane];
        out[o + 2 + lane] = p;
        out[o + 5 + lane] = h;
        out[o + 8 + lane] = p - h;
      }
      break;
    }
    case 2: {  // pen
      if (lane < nq - 6) out[lane] = s.qpos[lane];
      int o = nq - 6;
      if (lane < 3) {
        float ob = s.xpos[id[1]][lane];
        float oo = (s.sxpos[id[3]][lane] - s.sxpos[id[4]][lane]) / m.pen_length;
        float dd = (s.sxpos[id[5]][lane] - s.sxpos[id[6]][lane]) / m.tar_length;
        out[o + lane] = ob;
        out[o + 9 + lane] = oo;
        out[o + 12 + lane] = dd;
        out[o + 15 + lane] = ob - s.sxpos[id[2]][lane];
        out[o + 18 + lane] = oo - dd;
      }
      if (lane < 6) out[o + 3 + lane] = s.qvel[nv - 6 + lane];
      break;
    }
    case 3: {  // relocate
      if (lane < nq - 6) out[lane] = s.qpos[lane];
      int o = nq - 6;
      if (lane < 3) {
        float p = s.sxpos[id[0]][lane], ob = s.xpos[id[1]][lane], t = s.sxpos[id[2]][lane];
        out[o + lane] = p - ob;
        out[o + 3 + lane] = p - t;
        out[o + 6 + lane] = ob - t;
      }
      break;
    }
  }
}

// lane 0 computes reward / done / goal (fp32 restatement of the reference arithmetic)
AW_DEV void task_reward(const DModel& m, Env& s, float* reward, int* done, int* goal) {
  const int* id = m.d->task_idx;
  float r = 0.f;
  *done = 0;
  *goal = 0;
  switch (m.task_kind) {
    case 0: {
      const float* obj = s.xpos[id[1]];
      const float* palm = s.sxpos[id[0]];
      const float* tool = s.sxpos[id[2]];
      const float* target = s.sxpos[id[3]];
      const float* goalp = s.sxpos[id[4]];
      r = -0.1f * dist3(palm, obj);
      r -= dist3(tool, target);
      r -= 10.f * dist3(target, goalp);
      float qn = 0.f;
      for (int i = 0; i < m.nv; i++) qn += s.qvel[i] * s.qvel[i];
      r -= 1e-2f * sqrtf(qn);
      if (obj[2] > 0.04f && tool[2] > 0.04f) r += 2.f;
      float tg = dist3(target, goalp);
      if (tg < 0.020f) r += 25.f;
      if (tg < 0.010f) r += 75.f;
      *goal = tg < 0.010f;
      break;
    }
    case 1: {
      const float* handle = s.sxpos[id[1]];
      const float* palm = s.sxpos[id[0]];
      float door = s.qpos[id[2]];
      r = -0.1f * dist3(palm, handle);
      r += -0.1f * (door - 1.57f) * (door - 1.57f);
      float qs = 0.f;
      for (int i = 0; i < m.nv; i++) qs += s.qvel[i] * s.qvel[i];
      r += -1e-5f * qs;
      if (door > 0.2f) r += 2.f;
      if (door > 1.0f) r += 8.f;
      if (door > 1.35f) r += 10.f;
      *goal = door >= 1.35f;
      break;
    }
    case 2: {
      const float* obj = s.xpos[id[1]];
      const float* des = s.sxpos[id[2]];
      float oo[3], dd[3];
      for (int k = 0; k < 3; k++) {
        oo[k] = (s.sxpos[id[3]][k] - s.sxpos[id[4]][k]) / m.pen_length;
        dd[k] = (s.sxpos[id[5]][k] - s.sxpos[id[6]][k]) / m.tar_length;
      }
      float dist = dist3(obj, des);
      r = -dist;
      float sim = dot3(oo, dd);
      r += sim;
      if (dist < 0.075f && sim > 0.9f) r += 10.f;
      if (dist < 0.075f && sim > 0.95f) r += 50.f;
      if (obj[2] < 0.075f) { r -= 5.f; *done = 1; }
      *goal = dist < 0.075f && sim > 0.95f;
      break;
    }
    case 3: {
      const float* obj = s.xpos[id[1]];
      const float* palm = s.sxpos[id[0]];
      const float* tgt = s.sxpos[id[2]];
      r = -0.1f * dist3(palm, obj);
      if (obj[2] > 0.04f) {
        r += 1.0f;
        r += -0.5f * dist3(palm, tgt);
        r += -0.5f * dist3(obj, tgt);
      }
      float ot = dist3(obj, tgt);
      if (ot < 0.1f) r += 10.f;
      if (ot < 0.05f) r += 20.f;
      *goal = ot < 0.1f;
      break;
    }
  }
  *reward = r;
}

// ---------------------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG
AW_DEV void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}
AW_DEV float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// reset draws -> params (tasks.draws_to_params); counter = (global env id, episode, stream 0x5EED, block)
AW_DEV void sample_params(const DModel& m, uint64_t seed, uint32_t genv, uint32_t episode, float* params) {
  float u[8];
#pragma unroll
  for (int blk = 0; blk < 2; blk++) {
    uint32_t c[4] = {genv, episode, 0x5EEDu, (uint32_t)blk};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    for (int k = 0; k < 4; k++) u[4 * blk + k] = u01(c[k]);
  }
  float d[8];
#pragma unroll
  for (int k = 0; k < 8; k++) d[k] = k < m.ndraw ? MD(draw_lo, k) + (MD(draw_hi, k) - MD(draw_lo, k)) * u[k] : 0.f;
  if (m.task_kind == 2) {
    float eu[3] = {d[0], d[1], 0.f};
    euler2quat_ref(eu, params);
    return;
  }
  // tasks.param_draws: draw index, -1 keep (a field reset_model does not write keeps its last
  // value: the reference's model mutations persist across resets), -2 hammer
  // 'pos' neck x (hammer_v0.py:122).  params holds the env's current values on entry.
#pragma unroll
  for (int p = 0; p < MAXP; p++) {
    if (p >= m.nparam) break;
    const int c = MD(param_draw, p);
    float v = c == -2 ? -0.14f - (-0.24f - d[1]) : params[p];
#pragma unroll
    for (int k = 0; k < 8; k++) v = c == k ? d[k] : v;
    params[p] = v;
  }
}

}  // namespace aw
