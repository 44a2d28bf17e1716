// waitlvl.hip -- calibration of the SQ_INST_LEVEL_{LDS,SMEM,VMEM} counters (run under
// rocprofv3 --pmc on the GPU box; tools/gpu_waitlvl.sh).
//
// k_step's s_waitcnt time (SQ_WAIT_ANY) is split into LDS, scalar-memory and vector-memory classes
// with the INST_LEVEL counters (outstanding instructions of a class, accumulated per cycle).  Their
// normalisation is not documented for gfx950, so three kernels issue a DEPENDENT chain of one class
// each -- every instruction waits for the previous one -- one wave per CU, and time the chain with
// s_memtime.  For such a chain LEVEL / INSTS is the latency in the counter's unit and the measured
// cycles per instruction is the latency in shader cycles: their ratio is the scale that turns
// k_step's LEVEL counters into cycles of outstanding work per class.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;

__global__ void __launch_bounds__(64) k_lds_chain(int* out, int seed) {
  __shared__ int buf[256];
  for (int i = threadIdx.x; i < 256; i += 64) buf[i] = (i * 37 + seed) & 255;
  __syncthreads();
  int p = threadIdx.x;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; i++) p = buf[p];
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = p;
  if (threadIdx.x == 0) reinterpret_cast<long long*>(out + gridDim.x * 64)[blockIdx.x] = t1 - t0;
}

__global__ void __launch_bounds__(64) k_smem_chain(const int* __restrict__ tab, int* out) {
  int p = 0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; i++) p = __builtin_amdgcn_readfirstlane(tab[p]);
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = p;
  if (threadIdx.x == 0) reinterpret_cast<long long*>(out + gridDim.x * 64)[blockIdx.x] = t1 - t0;
}

__global__ void __launch_bounds__(64) k_vmem_chain(const int* tab, int* out) {
  int p = threadIdx.x;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; i++) p = tab[p];
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = p;
  if (threadIdx.x == 0) reinterpret_cast<long long*>(out + gridDim.x * 64)[blockIdx.x] = t1 - t0;
}

int main() {
  const int grid = 256;              // one wave per CU
  const int ntab = 1 << 12;          // 16 KB table: L2 / scalar-cache resident after the first pass
  int *tab, *out;
  (void)hipMalloc(&tab, ntab * 4);
  (void)hipMalloc(&out, grid * 64 * 4 + grid * 8);
  int h[1 << 12];
  for (int i = 0; i < ntab; i++) h[i] = (i * 613 + 64) & (ntab - 1) & ~63;   // a 64-aligned hop
  for (int i = 0; i < ntab; i++) h[i] += (i & 63);                           // + the lane offset
  (void)hipMemcpy(tab, h, ntab * 4, hipMemcpyHostToDevice);
  long long cyc[256];
  const char* names[3] = {"lds", "smem", "vmem"};
  for (int k = 0; k < 3; k++) {
    for (int rep = 0; rep < 2; rep++) {
      if (k == 0) hipLaunchKernelGGL(k_lds_chain, dim3(grid), dim3(64), 0, 0, out, rep);
      if (k == 1) hipLaunchKernelGGL(k_smem_chain, dim3(grid), dim3(64), 0, 0, tab, out);
      if (k == 2) hipLaunchKernelGGL(k_vmem_chain, dim3(grid), dim3(64), 0, 0, tab, out);
    }
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(cyc, out + grid * 64, grid * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int b = 0; b < grid; b++) s += (double)cyc[b];
    // s_memtime ticks are shader cycles (MI355X_MICROARCH.md PMC table)
    printf("{\"chain\": \"%s\", \"iters\": %d, \"cycles_per_inst\": %.3f}\n", names[k], ITERS, s / grid / ITERS);
  }
  (void)hipFree(tab);
  (void)hipFree(out);
  return 0;
}
