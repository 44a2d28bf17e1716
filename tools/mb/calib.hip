// calib.hip -- FETCH_SIZE / WRITE_SIZE calibration for k_step's access pattern (run under
// rocprofv3 --pmc FETCH_SIZE or --pmc WRITE_SIZE on the GPU box; tools/gpu_prof.sh).
//
// k_step moves each env's state as rows of 4-byte words, one word per lane (lane < row length):
// load_env / store_env / write_obs.  These kernels read / write exactly that pattern with known
// byte counts -- one wave per row, rows of 33 floats (hammer's qpos) at a row stride of 33 floats
// -- so the counters' ratio to the exact bytes calibrates the HBM traffic k_step reports.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int ROW = 33;

__global__ void __launch_bounds__(64) k_calib_read(int rows, const float* __restrict__ in, float* out) {
  float acc = 0.f;
  for (int r = blockIdx.x; r < rows; r += gridDim.x)
    if (threadIdx.x < ROW) acc += in[(size_t)r * ROW + threadIdx.x];
  // one word per workgroup leaves the kernel (negligible against the rows read)
  acc += __shfl_xor(acc, 1); acc += __shfl_xor(acc, 2); acc += __shfl_xor(acc, 4);
  acc += __shfl_xor(acc, 8); acc += __shfl_xor(acc, 16); acc += __shfl_xor(acc, 32);
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(64) k_calib_write(int rows, float* __restrict__ out) {
  for (int r = blockIdx.x; r < rows; r += gridDim.x)
    if (threadIdx.x < ROW) out[(size_t)r * ROW + threadIdx.x] = (float)(r + threadIdx.x);
}

int main() {
  const int rows = 1 << 20;             // 1 Mi rows x 132 B = 138 MB (far past the caches)
  const int grid = 2048;                // k_step's persistent grid on MI355X
  float *in, *out, *sums;
  (void)hipMalloc(&in, (size_t)rows * ROW * 4);
  (void)hipMalloc(&out, (size_t)rows * ROW * 4);
  (void)hipMalloc(&sums, grid * 4);
  (void)hipMemset(in, 0, (size_t)rows * ROW * 4);
  for (int it = 0; it < 3; it++) {
    hipLaunchKernelGGL(k_calib_read, dim3(grid), dim3(64), 0, 0, rows, in, sums);
    hipLaunchKernelGGL(k_calib_write, dim3(grid), dim3(64), 0, 0, rows, out);
  }
  (void)hipDeviceSynchronize();
  printf("{\"rows\": %d, \"row_floats\": %d, \"exact_read_bytes\": %zu, \"exact_write_bytes\": %zu, "
         "\"sums_bytes\": %d}\n", rows, ROW, (size_t)rows * ROW * 4, (size_t)rows * ROW * 4, grid * 4);
  (void)hipFree(in); (void)hipFree(out); (void)hipFree(sums);
  return 0;
}
