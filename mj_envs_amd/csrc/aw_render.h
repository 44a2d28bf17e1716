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
  float box[MAXRG][4];   // conservative pixel box of the bounding sphere: col min / max, row min / max
  int type[MAXRG];
};

AW_DEV void render_geoms(const DModel& m, const Env& s, RGeoms& r, const float* cam, int tid, int nthreads) {
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
    const float rb = MD(rg_rbound, g);
    r.rb[g] = rb;
    r.type[g] = MD(rg_type, g);
    // image-space box of the bounding sphere: x / z over the sphere's camera-frame bounding box
    // is extremal at its corners (conservative); behind / straddling the camera or unbounded
    // (planes: rbound 0) -> the whole image
    float c[3], x = 0.f, y = 0.f, z = 0.f;
    sub3(c, r.pos[g], cam);
    x = dot3(c, cam + 9); y = dot3(c, cam + 6); z = dot3(c, cam + 3);
    float b0 = -1e30f, b1 = 1e30f, b2 = -1e30f, b3 = 1e30f;
    if (rb > 0.f && z - rb > 1e-3f) {
      const float z0 = z - rb, z1 = z + rb;
      const float umin = fminf((x - rb) / z0, (x - rb) / z1), umax = fmaxf((x + rb) / z0, (x + rb) / z1);
      const float vmin = fminf((y - rb) / z0, (y - rb) / z1), vmax = fmaxf((y + rb) / z0, (y + rb) / z1);
      b0 = (umin - cam[12]) / cam[13] - 1.f;   // column range (one pixel of slack)
      b1 = (umax - cam[12]) / cam[13] + 1.f;
      b2 = (cam[14] - vmax) / cam[15] - 1.f;   // row range
      b3 = (cam[14] - vmin) / cam[15] + 1.f;
    }
    r.box[g][0] = b0; r.box[g][1] = b1; r.box[g][2] = b2; r.box[g][3] = b3;
  }
}

// z-depth of the 64 pixels [p0, p0 + 64) handled by one wave: the geoms whose pixel box meets
// the rows of this span are found once per wave (lane g tests geom g, ballot), then every lane
// runs only those: column box, bounding-sphere cull, exact ray-primitive test
AW_DEV void render_span(const RGeoms& r, int ng, const float* cam, int W, int H, int p0, int lane, float* out) {
  const int np = W * H;
  const int p = p0 + lane;
  const int rlo = p0 / W, rhi = min(p0 + 63, np - 1) / W;
  const bool on = lane < ng && r.box[lane][2] <= (float)rhi && r.box[lane][3] >= (float)rlo;
  unsigned long long mask = __ballot(on);
  const int row = p / W, col = p - row * W;
  const float u = cam[12] + cam[13] * (float)col, w = cam[14] - cam[15] * (float)row;
  float d[3];
  for (int k = 0; k < 3; k++) d[k] = cam[3 + k] + u * cam[9 + k] + w * cam[6 + k];
  normalize3(d);
  const float fc = (float)col, fr = (float)row;
  float best = 3.0e38f;
  while (mask) {
    const int g = __builtin_ctzll(mask);
    mask &= mask - 1ull;
    if (fc < r.box[g][0] || fc > r.box[g][1] || fr < r.box[g][2] || fr > r.box[g][3]) continue;
    const float rb = r.rb[g];
    if (rb > 0.f) {
      float oc[3];
      sub3(oc, r.pos[g], cam);
      const float tc = dot3(oc, d);
      const float d2 = dot3(oc, oc) - tc * tc;
      if (d2 > rb * rb || tc + rb < 0.f || tc - rb > best) continue;
    }
    const float t = ray_prim(r.pos[g], r.mat[g], r.size[g], r.type[g], cam, d);
    if (t >= 0.f && t < best) best = t;
  }
  if (p < np) out[p] = best < 1.0e38f ? best * dot3(d, cam + 3) : cam[16];
}

}  // namespace aw
