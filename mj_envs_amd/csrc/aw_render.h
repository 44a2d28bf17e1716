// aw_render.h -- depth ray casting against primitive geoms (fp32).
//
// Replaces the reference's OpenGL frame (hand_manipulation_suite/headless_observer.py:34-52)
// with metric z-depth; see mj_envs_amd/render.py for the camera construction.  numpy
// restatement for the tests: oracle/depth.py.
#pragma once
#include "aw_common.h"
#include "aw_solver.h"

namespace aw {

// first crossing t >= 0 of the ray o + t v (v unit, world frame) with a primitive geom, or -1;
// planes are finite where their size is positive (as MuJoCo draws them)
AW_DEV float ray_prim(const float* pos, const float* mat, const float* size, int type, const float* o,
                      const float* v) {
  if (type == GEOM_PLANE) {
    float dif[3], lp[3], lv[3];
    sub3(dif, o, pos);
    mulmtv3(lp, mat, dif);
    mulmtv3(lv, mat, v);
    if (fabsf(lv[2]) < MINVAL) return -1.f;
    const float t = -lp[2] / lv[2];
    if (t < 0.f) return -1.f;
    const float x = lp[0] + t * lv[0], y = lp[1] + t * lv[1];
    if ((size[0] > 0.f && fabsf(x) > size[0]) || (size[1] > 0.f && fabsf(y) > size[1])) return -1.f;
    return t;
  }
  return ray_geom(pos, mat, size, o, v, type);
}

// world poses of the rendered geoms of one env (s.xpos / s.xquat from stage_kinematics)
struct RGeoms {
  float pos[MAXRG][3], mat[MAXRG][9], size[MAXRG][3], rb[MAXRG];
  int type[MAXRG];
};

AW_DEV void render_geoms(const DModel& m, const Env& s, RGeoms& r, int tid, int nthreads) {
  for (int g = tid; g < m.nrgeom; g += nthreads) {
    const int b = MD(rg_body, g), cg = MD(rg_cgeom, g);
    float lp[3], lq[4], bq[4], v[3], q[4];
    for (int k = 0; k < 3; k++) lp[k] = MD(rg_pos, 3 * g + k);
    for (int k = 0; k < 4; k++) { lq[k] = MD(rg_quat, 4 * g + k); bq[k] = s.xquat[b][k]; }
    if (cg >= 0 && MD(geom_ovr, cg)) apply_ovr<3>(m, s, 4, cg, lp);
    rotvq(v, lp, bq);
    add3(r.pos[g], v, s.xpos[b]);
    mulq(q, bq, lq);
    q2m(r.mat[g], q);
    for (int k = 0; k < 3; k++) r.size[g][k] = cg >= 0 ? s.gsize[cg][k] : MD(rg_size, 3 * g + k);
    r.rb[g] = MD(rg_rbound, g);
    r.type[g] = MD(rg_type, g);
  }
}

// z-depth of one pixel: nearest hit over the geoms (bounding-sphere cull first)
AW_DEV float render_pixel(const RGeoms& r, int ng, const float* cam, int row, int col) {
  const float u = cam[12] + cam[13] * (float)col, w = cam[14] - cam[15] * (float)row;
  float d[3];
  for (int k = 0; k < 3; k++) d[k] = cam[3 + k] + u * cam[9 + k] + w * cam[6 + k];
  normalize3(d);
  const float* o = cam;
  float best = 3.0e38f;
  for (int g = 0; g < ng; g++) {
    const float rb = r.rb[g];
    if (rb > 0.f) {
      float oc[3];
      sub3(oc, r.pos[g], o);
      const float tc = dot3(oc, d);
      const float d2 = dot3(oc, oc) - tc * tc;
      if (d2 > rb * rb || tc + rb < 0.f || tc - rb > best) continue;
    }
    const float t = ray_prim(r.pos[g], r.mat[g], r.size[g], r.type[g], o, d);
    if (t >= 0.f && t < best) best = t;
  }
  return best < 1.0e38f ? best * dot3(d, cam + 3) : cam[16];
}

}  // namespace aw
