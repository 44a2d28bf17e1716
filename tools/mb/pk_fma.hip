#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
template <int PK>
__global__ void __launch_bounds__(64) kern(float* out, int iters, float s) {
  float a = threadIdx.x * 1e-3f;
  if (PK) {
    f2 acc[8];
    for (int i = 0; i < 8; i++) acc[i] = f2{a + i, a - i};
    f2 m = f2{s, s * 0.5f}, c = f2{1e-3f, 2e-3f};
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int r = 0; r < 16; r++)
#pragma unroll
        for (int i = 0; i < 8; i++) acc[i] = __builtin_elementwise_fma(acc[i], m, c);
    }
    float t = 0; for (int i = 0; i < 8; i++) t += acc[i].x + acc[i].y;
    out[blockIdx.x * 64 + threadIdx.x] = t;
  } else {
    float acc[16];
    for (int i = 0; i < 16; i++) acc[i] = a + i;
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int r = 0; r < 16; r++)
#pragma unroll
        for (int i = 0; i < 16; i++) asm("v_fma_f32 %0, %1, %2, %3" : "=v"(acc[i]) : "v"(acc[i]), "v"(s), "v"(1e-3f * (i & 1 ? 2 : 1)));
    }
    float t = 0; for (int i = 0; i < 16; i++) t += acc[i];
    out[blockIdx.x * 64 + threadIdx.x] = t;
  }
}
int main() {
  float* d; hipMalloc(&d, 64 * 8192 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int iters = 2000;
  for (int wps : {1, 2, 4}) {
    int blocks = 256 * 4 * wps;
    for (int pk = 0; pk < 2; pk++) {
      for (int rep = 0; rep < 2; rep++) {
        hipEventRecord(e0);
        if (pk) kern<1><<<blocks, 64>>>(d, iters, 0.999f); else kern<0><<<blocks, 64>>>(d, iters, 0.999f);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        double fma = (double)blocks * 64 * iters * 16 * 16;
        if (rep) printf("waves/SIMD %d %s: %.3f ms  %.1f TFLOP/s\n", wps, pk ? "v_pk_fma_f32" : "v_fma_f32", ms, 2 * fma / ms / 1e9);
      }
    }
  }
  return 0;
}
