// Host check of the kernel's fp64 sin / cos restatement (mj_envs_amd/csrc/aw_sincos64.h) against
// libm: fp32 joint half-angles, small angles and |x| < 1e5.  Prints the largest error in ulps of
// libm's result for sin and cos (tests/test_sincos64.py runs it).
#include <cmath>
#include <cstdio>
#include <random>

#include "../mj_envs_amd/csrc/aw_sincos64.h"

static double ulps(double a, double b) {
  if (a == b) return 0;
  return std::fabs(a - b) / std::ldexp(1.0, std::ilogb(b) - 52);
}

int main() {
  static const double K[15] = AW_SINCOS64_K;
  std::mt19937_64 g(1);
  double ms = 0, mc = 0;
  const long N = 4000000;
  for (long i = 0; i < N; i++) {
    double x;
    switch (i % 4) {
      case 0: x = std::uniform_real_distribution<double>(-4, 4)(g); break;
      case 1: x = (double)(float)std::uniform_real_distribution<double>(-200, 200)(g) * 0.5; break;
      case 2: x = (double)(float)std::uniform_real_distribution<double>(-1e-3, 1e-3)(g) * 0.5; break;
      default: x = std::uniform_real_distribution<double>(-1e5, 1e5)(g);
    }
    double s, c;
    sincos64_k(x, K, &s, &c);
    ms = std::fmax(ms, ulps(s, std::sin(x)));
    mc = std::fmax(mc, ulps(c, std::cos(x)));
  }
  printf("%.3f %.3f\n", ms, mc);
  return 0;
}
