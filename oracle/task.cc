/* task.cc -- fp64 restatement of the reference task layer (TEST INFRASTRUCTURE ONLY).
 * Exact restatement of:
 *   hammer   hand_manipulation_suite/hammer_v0.py:54-104
 *   door     hand_manipulation_suite/door_v0.py:55-101
 *   pen      hand_manipulation_suite/pen_v0.py:65-113
 *   relocate hand_manipulation_suite/relocate_v0.py:46-83
 *   quat2euler utils/quatmath.py:136-164 (+ mat2euler :79-96)
 * Pinned by tests/golden (vectors produced from the reference modules themselves).
 */
#include <cfloat>
#include <cmath>

#include "oracle.h"

namespace orc {

static const num FLOAT_EPS = DBL_EPSILON;
static const num EPS4 = DBL_EPSILON * 4.0;

void quat2euler(const num* q, num* e) {
  num w = q[0], x = q[1], y = q[2], z = q[3];
  num Nq = w * w + x * x + y * y + z * z;
  num m[9];
  if (Nq > FLOAT_EPS) {
    num s = 2.0 / Nq;
    num X = x * s, Y = y * s, Z = z * s;
    num wX = w * X, wY = w * Y, wZ = w * Z, xX = x * X, xY = x * Y, xZ = x * Z;
    num yY = y * Y, yZ = y * Z, zZ = z * Z;
    m[0] = 1.0 - (yY + zZ); m[1] = xY - wZ; m[2] = xZ + wY;
    m[3] = xY + wZ; m[4] = 1.0 - (xX + zZ); m[5] = yZ - wX;
    m[6] = xZ - wY; m[7] = yZ + wX; m[8] = 1.0 - (xX + yY);
  } else {
    m[0] = 1; m[1] = 0; m[2] = 0; m[3] = 0; m[4] = 1; m[5] = 0; m[6] = 0; m[7] = 0; m[8] = 1;
  }
  num cy = std::sqrt(m[8] * m[8] + m[5] * m[5]);
  bool cond = cy > EPS4;
  e[2] = cond ? -std::atan2(m[1], m[0]) : -std::atan2(-m[3], m[4]);
  e[1] = -std::atan2(-m[2], cy);
  e[0] = cond ? -std::atan2(m[5], m[8]) : 0.0;
}

static num dist3(const num* a, const num* b) {
  num d[3];
  sub3(d, a, b);
  return norm3(d);
}
static num clip(num x, num lo, num hi) { return x < lo ? lo : (x > hi ? hi : x); }

void task_obs(const Model* m, const Data* d, num* obs) {
  const int* id = m->task_idx.data();
  int nq = m->nq, nv = m->nv, o = 0;
  switch (m->task_kind) {
    case 0: { /* hammer */
      for (int i = 0; i < nq - 6; i++) obs[o++] = d->qpos[i];
      for (int i = nv - 6; i < nv; i++) obs[o++] = clip(d->qvel[i], -1, 1);
      for (int k = 0; k < 3; k++) obs[o++] = d->site_xpos[3 * id[0] + k];      /* palm */
      for (int k = 0; k < 3; k++) obs[o++] = d->xpos[3 * id[1] + k];           /* obj */
      num e[3];
      quat2euler(&d->xquat[4 * id[1]], e);
      for (int k = 0; k < 3; k++) obs[o++] = e[k];
      for (int k = 0; k < 3; k++) obs[o++] = d->site_xpos[3 * id[3] + k];      /* target */
      obs[o++] = clip(d->sensordata[id[5]], -1, 1);
      break;
    }
    case 1: { /* door */
      for (int i = 1; i < nq - 2; i++) obs[o++] = d->qpos[i];
      obs[o++] = d->qpos[nq - 1];                                              /* latch */
      num door = d->qpos[id[2]];
      obs[o++] = door;
      const num* palm = &d->site_xpos[3 * id[0]];
      const num* handle = &d->site_xpos[3 * id[1]];
      for (int k = 0; k < 3; k++) obs[o++] = palm[k];
      for (int k = 0; k < 3; k++) obs[o++] = handle[k];
      for (int k = 0; k < 3; k++) obs[o++] = palm[k] - handle[k];
      obs[o++] = door > 1.0 ? 1.0 : -1.0;
      break;
    }
    case 2: { /* pen */
      for (int i = 0; i < nq - 6; i++) obs[o++] = d->qpos[i];
      const num* obj = &d->xpos[3 * id[1]];
      const num* des = &d->site_xpos[3 * id[2]];
      num oo[3], dd[3];
      for (int k = 0; k < 3; k++) {
        oo[k] = (d->site_xpos[3 * id[3] + k] - d->site_xpos[3 * id[4] + k]) / m->pen_length;
        dd[k] = (d->site_xpos[3 * id[5] + k] - d->site_xpos[3 * id[6] + k]) / m->tar_length;
      }
      for (int k = 0; k < 3; k++) obs[o++] = obj[k];
      for (int i = nv - 6; i < nv; i++) obs[o++] = d->qvel[i];
      for (int k = 0; k < 3; k++) obs[o++] = oo[k];
      for (int k = 0; k < 3; k++) obs[o++] = dd[k];
      for (int k = 0; k < 3; k++) obs[o++] = obj[k] - des[k];
      for (int k = 0; k < 3; k++) obs[o++] = oo[k] - dd[k];
      break;
    }
    case 3: { /* relocate */
      for (int i = 0; i < nq - 6; i++) obs[o++] = d->qpos[i];
      const num* palm = &d->site_xpos[3 * id[0]];
      const num* obj = &d->xpos[3 * id[1]];
      const num* tgt = &d->site_xpos[3 * id[2]];
      for (int k = 0; k < 3; k++) obs[o++] = palm[k] - obj[k];
      for (int k = 0; k < 3; k++) obs[o++] = palm[k] - tgt[k];
      for (int k = 0; k < 3; k++) obs[o++] = obj[k] - tgt[k];
      break;
    }
  }
}

void task_reward(const Model* m, const Data* d, num* reward, uint8_t* done, uint8_t* goal, int starting_up) {
  const int* id = m->task_idx.data();
  num r = 0;
  *done = 0;
  *goal = 0;
  switch (m->task_kind) {
    case 0: { /* hammer_v0.py:62-90 */
      const num* obj = &d->xpos[3 * id[1]];
      const num* palm = &d->site_xpos[3 * id[0]];
      const num* tool = &d->site_xpos[3 * id[2]];
      const num* target = &d->site_xpos[3 * id[3]];
      const num* goalp = &d->site_xpos[3 * id[4]];
      r = -0.1 * dist3(palm, obj);
      r -= dist3(tool, target);
      r -= 10 * dist3(target, goalp);
      num qn = 0;
      for (int i = 0; i < m->nv; i++) qn += d->qvel[i] * d->qvel[i];
      r -= 1e-2 * std::sqrt(qn);
      if (obj[2] > 0.04 && tool[2] > 0.04) r += 2;
      num tg = dist3(target, goalp);
      if (tg < 0.020) r += 25;
      if (tg < 0.010) r += 75;
      *goal = tg < 0.010;
      break;
    }
    case 1: { /* door_v0.py:62-83 */
      const num* handle = &d->site_xpos[3 * id[1]];
      const num* palm = &d->site_xpos[3 * id[0]];
      num door = d->qpos[id[2]];
      r = -0.1 * dist3(palm, handle);
      r += -0.1 * (door - 1.57) * (door - 1.57);
      num qs = 0;
      for (int i = 0; i < m->nv; i++) qs += d->qvel[i] * d->qvel[i];
      r += -1e-5 * qs;
      if (door > 0.2) r += 2;
      if (door > 1.0) r += 8;
      if (door > 1.35) r += 10;
      *goal = door >= 1.35;
      break;
    }
    case 2: { /* pen_v0.py:73-100 */
      const num* obj = &d->xpos[3 * id[1]];
      const num* des = &d->site_xpos[3 * id[2]];
      num oo[3], dd[3];
      for (int k = 0; k < 3; k++) {
        oo[k] = (d->site_xpos[3 * id[3] + k] - d->site_xpos[3 * id[4] + k]) / m->pen_length;
        dd[k] = (d->site_xpos[3 * id[5] + k] - d->site_xpos[3 * id[6] + k]) / m->tar_length;
      }
      num dist = dist3(obj, des);
      r = -dist;
      num sim = dot3(oo, dd);
      r += sim;
      if (dist < 0.075 && sim > 0.9) r += 10;
      if (dist < 0.075 && sim > 0.95) r += 50;
      if (obj[2] < 0.075) {
        r -= 5;
        *done = starting_up ? 0 : 1;
      }
      *goal = dist < 0.075 && sim > 0.95;
      break;
    }
    case 3: { /* relocate_v0.py:53-70 */
      const num* obj = &d->xpos[3 * id[1]];
      const num* palm = &d->site_xpos[3 * id[0]];
      const num* tgt = &d->site_xpos[3 * id[2]];
      r = -0.1 * dist3(palm, obj);
      if (obj[2] > 0.04) {
        r += 1.0;
        r += -0.5 * dist3(palm, tgt);
        r += -0.5 * dist3(obj, tgt);
      }
      num ot = dist3(obj, tgt);
      if (ot < 0.1) r += 10.0;
      if (ot < 0.05) r += 20.0;
      *goal = ot < 0.1;
      break;
    }
  }
  *reward = r;
}

}  // namespace orc
