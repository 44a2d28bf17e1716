// fp64 sin / cos of a joint half-angle, shared by the kernel (aw_dynamics.h stage_kin64) and the
// host check (tests/sincos64_check.cc): one-pass Cody-Waite reduction by pi/2 -- a 33-bit head and
// its tail, carried as a double-double into the kernels -- and the classic minimax kernels of
// fdlibm's k_sin / k_cos (their published coefficients).  Accurate for |x| < 2^20 pi/2 (joint
// angles of fp32 state are far inside); <= 1 ulp against libm with fused multiply-adds, as the
// kernel is compiled.  The constants come in through K (AW_SINCOS64_K order) so the kernel can read
// them from constant memory instead of holding fifteen 64-bit literals in registers.
#pragma once
#ifdef __HIPCC__
#define AW_SC_HD __host__ __device__ inline
#else
#include <cmath>
#include <cstdint>
#include <cstring>
#define AW_SC_HD inline
#endif

// 2/pi; pi/2 head (33 bits) and tail; S1..S6 (k_sin); C1..C6 (k_cos)
#define AW_SINCOS64_K                                                                              \
  {6.36619772367581382433e-01,                                                                     \
   1.57079632673412561417e+00, 6.07710050650619224932e-11,                                         \
   -1.66666666666666324348e-01, 8.33333333332248946124e-03, -1.98412698298579493134e-04,           \
   2.75573137070700676789e-06, -2.50507602534068634195e-08, 1.58969099521155010221e-10,            \
   4.16666666666666019037e-02, -1.38888888888741095749e-03, 2.48015872894767294178e-05,            \
   -2.75573143513906633035e-07, 2.08757232129817482790e-09, -1.13596475577881948265e-11}

// |x| / 4 with the low 32 bits cleared (k_cos's qx: keeps 1 - qx exact)
AW_SC_HD double aw_quarter_hi(double ay) {
#ifdef __HIP_DEVICE_COMPILE__
  return __longlong_as_double((__double_as_longlong(ay) - (0x00200000ll << 32)) & ~0xffffffffll);
#else
  long long u;
  memcpy(&u, &ay, 8);
  u = (u - (0x00200000ll << 32)) & ~0xffffffffll;
  double r;
  memcpy(&r, &u, 8);
  return r;
#endif
}

AW_SC_HD void sincos64_k(double x, const double* K, double* sn, double* cs) {
  const double fn = rint(x * K[0]);
  const double r = x - fn * K[1], w = fn * K[2];
  const double y0 = r - w, y1 = (r - y0) - w;
  const double z = y0 * y0;
  const double v = z * y0, rs = K[4] + z * (K[5] + z * (K[6] + z * (K[7] + z * K[8])));
  const double ks = y0 - ((z * (0.5 * y1 - v * rs) - y1) - v * K[3]);
  const double rc = z * (K[9] + z * (K[10] + z * (K[11] + z * (K[12] + z * (K[13] + z * K[14])))));
  const double ay = fabs(y0);
  // |y0| >= 0.3: cos = (1 - qx) - ((z/2 - qx) - ...), 0.28125 past |y0| = 0.78125
  const double qx = ay < 0.3 ? 0.0 : ay > 0.78125 ? 0.28125 : aw_quarter_hi(ay);
  const double kc = (1.0 - qx) - ((0.5 * z - qx) - (z * rc - y0 * y1));
  const int n = (int)(long long)fn & 3;
  *sn = n == 0 ? ks : n == 1 ? kc : n == 2 ? -ks : -kc;
  *cs = n == 0 ? kc : n == 1 ? -ks : n == 2 ? -kc : ks;
}
