// aw_policy.h -- on-device Gaussian MLP policy.
//
// Restates mjrl's gaussian_mlp.MLP / FCNetwork (third-party, unpinned git master; used by the
// reference's DAPG baseline, mj_envs_vision/algos/baselines.py:67-86 with hidden_sizes=(32, 32)):
//   out = (obs - in_shift) / (in_scale + 1e-8); out = tanh(W0 out + b0); out = tanh(W1 out + b1);
//   mean = (W2 out + b2) * out_scale + out_shift;  action = mean [+ exp(log_std) * N(0, 1)].
// One thread per env; the parameters are staged in LDS per workgroup and read as uniform-address
// broadcasts, the activations stay in VGPRs.  Parameter block layout (fp32):
//   in_shift[in] in_scale[in] W0[H][in] b0[H] W1[H][H] b1[H] W2[out][H] b2[out]
//   out_scale[out] out_shift[out] log_std[out]
#pragma once
#include "aw_common.h"
#include "aw_task.h"

namespace aw {

constexpr int MLP_IMAX = 64;   // observation width cap
constexpr int MLP_OMAX = 32;   // action width cap

AW_DEV int mlp_param_count(int in, int h, int out) { return 2 * in + h * in + h + h * h + h + out * h + 4 * out; }

template <int H>
__global__ void __launch_bounds__(256) k_mlp(int n, int in, int out, const float* __restrict__ p,
                                             const float* __restrict__ obs, float* __restrict__ act, int sample,
                                             uint64_t seed, uint64_t step, uint64_t env_offset) {
  static_assert(H % 4 == 0 && MLP_IMAX % 4 == 0, "16-byte weight rows");
  const float* in_shift = p;
  const float* in_scale = p + in;
  const float* W0 = p + 2 * in;
  const float* b0 = W0 + H * in;
  const float* W1 = b0 + H;
  const float* b1 = W1 + H * H;
  const float* W2 = b1 + H;
  const float* b2 = W2 + out * H;
  const float* osc = b2 + out;
  const float* osh = osc + out;
  const float* lstd = osh + out;
  // the parameters staged in LDS once per workgroup, weight rows padded to 16 bytes (zeros past
  // `in`): every thread then reads them as uniform-address 16-byte broadcasts.  With a scalar load
  // per weight and one wave per SIMD (65 536 envs are 1 024 waves) the loads' latency was the
  // kernel's time (r05: 123 us per launch)
  __shared__ float4 sW0[H][MLP_IMAX / 4];
  __shared__ float4 sW1[H][H / 4];
  __shared__ float4 sW2[MLP_OMAX][H / 4];
  __shared__ float sb0[H], sb1[H], sb2[MLP_OMAX], sosc[MLP_OMAX], sosh[MLP_OMAX], slstd[MLP_OMAX];
  __shared__ float sish[MLP_IMAX], sisc[MLP_IMAX];
  for (int i = threadIdx.x; i < H * MLP_IMAX; i += blockDim.x) {
    const int j = i / MLP_IMAX, k = i % MLP_IMAX;
    reinterpret_cast<float*>(&sW0[0][0])[i] = k < in ? W0[j * in + k] : 0.f;
  }
  for (int i = threadIdx.x; i < H * H; i += blockDim.x) reinterpret_cast<float*>(&sW1[0][0])[i] = W1[i];
  for (int i = threadIdx.x; i < MLP_OMAX * H; i += blockDim.x)
    reinterpret_cast<float*>(&sW2[0][0])[i] = i / H < out ? W2[i] : 0.f;
  for (int i = threadIdx.x; i < H; i += blockDim.x) { sb0[i] = b0[i]; sb1[i] = b1[i]; }
  for (int i = threadIdx.x; i < MLP_OMAX; i += blockDim.x) {
    sb2[i] = i < out ? b2[i] : 0.f;
    sosc[i] = i < out ? osc[i] : 0.f;
    sosh[i] = i < out ? osh[i] : 0.f;
    slstd[i] = i < out ? lstd[i] : 0.f;
  }
  for (int i = threadIdx.x; i < MLP_IMAX; i += blockDim.x) {
    sish[i] = i < in ? in_shift[i] : 0.f;
    sisc[i] = i < in ? in_scale[i] : 1.f;
  }
  __syncthreads();
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  float x[MLP_IMAX];
#pragma unroll
  for (int k = 0; k < MLP_IMAX; k++)
    x[k] = k < in ? (obs[(size_t)e * in + k] - sish[k]) / (sisc[k] + 1e-8f) : 0.f;
  float h1[H], h2[H];
#pragma unroll
  for (int j = 0; j < H; j++) {
    float acc = sb0[j];
#pragma unroll
    for (int q = 0; q < MLP_IMAX / 4; q++) {
      if (4 * q >= in) break;   // uniform: the padded tail of the row is zeros
      const float4 w = sW0[j][q];
      acc = fmaf(w.x, x[4 * q], acc);
      if (4 * q + 1 < in) acc = fmaf(w.y, x[4 * q + 1], acc);
      if (4 * q + 2 < in) acc = fmaf(w.z, x[4 * q + 2], acc);
      if (4 * q + 3 < in) acc = fmaf(w.w, x[4 * q + 3], acc);
    }
    h1[j] = tanhf(acc);
  }
#pragma unroll
  for (int j = 0; j < H; j++) {
    float acc = sb1[j];
#pragma unroll
    for (int q = 0; q < H / 4; q++) {
      const float4 w = sW1[j][q];
      acc = fmaf(w.x, h1[4 * q], acc);
      acc = fmaf(w.y, h1[4 * q + 1], acc);
      acc = fmaf(w.z, h1[4 * q + 2], acc);
      acc = fmaf(w.w, h1[4 * q + 3], acc);
    }
    h2[j] = tanhf(acc);
  }
  float nz[MLP_OMAX];
#pragma unroll
  for (int o = 0; o < MLP_OMAX; o++) nz[o] = 0.f;
  if (sample) {
    // N(0, 1) by Box-Muller on Philox draws, counter = (global env id, step, 0x901C, block)
#pragma unroll
    for (int blk = 0; blk < MLP_OMAX / 4; blk++) {
      uint32_t c[4] = {(uint32_t)(env_offset + (uint64_t)e), (uint32_t)step, (uint32_t)(step >> 32) ^ 0x901Cu,
                       (uint32_t)blk};
      philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const float u1 = fmaxf(u01(c[2 * q]), 1.0f / 16777216.0f), u2 = u01(c[2 * q + 1]);
        const float r = sqrtf(-2.f * logf(u1));
        nz[4 * blk + 2 * q] = r * cosf(6.28318530717958647f * u2);
        nz[4 * blk + 2 * q + 1] = r * sinf(6.28318530717958647f * u2);
      }
    }
  }
#pragma unroll
  for (int o = 0; o < MLP_OMAX; o++) {
    if (o >= out) break;
    float acc = sb2[o];
#pragma unroll
    for (int q = 0; q < H / 4; q++) {
      const float4 w = sW2[o][q];
      acc = fmaf(w.x, h2[4 * q], acc);
      acc = fmaf(w.y, h2[4 * q + 1], acc);
      acc = fmaf(w.z, h2[4 * q + 2], acc);
      acc = fmaf(w.w, h2[4 * q + 3], acc);
    }
    float a = acc * sosc[o] + sosh[o];
    if (sample) a = fmaf(expf(slstd[o]), nz[o], a);
    act[(size_t)e * out + o] = a;
  }
}

}  // namespace aw
