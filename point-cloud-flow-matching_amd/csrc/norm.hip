// BatchNorm with batch statistics (training mode) fused with the activation
// that follows it everywhere on the PVConv path:
//   SharedMLP  (third_party/pvcnn/modules/shared_mlp.py:15-27): BN1d -> ReLU
//   PVConv     (third_party/pvcnn/modules/pvconv.py:20-30):     BN3d -> LeakyReLU(0.1)
// over (B, C, S) fp32 tensors (S = points or voxels), the layout the
// reference's Conv1d / Conv3d produce.  torch runs these as MIOpen BN + a
// separate (in-place) activation, and a threshold / leaky backward + MIOpen
// BN backward: ~12 full passes over the tensor per layer.  Here:
//   forward : stats pass (read x) -> per-channel finalize (mean, invstd,
//             running-stat update) -> apply pass (read x, write act(bn(x)))
//   backward: stats pass (read dz, x: sum g, sum g*xhat with g = dz * act')
//             -> finalize (dgamma, dbeta) -> apply pass (read dz, x, write dx)
// 8 passes.  Partial sums are per (channel, part) block and combined in a
// fixed order: deterministic.  The forward sums are shifted by the channel's
// first element (sum (x - K), sum (x - K)^2) against cancellation.
#include "pcfm_common.hpp"

namespace pcfm {
namespace {

constexpr int kBnParts = 16;  // target blocks per channel in the stats passes
inline int bn_parts(int b) { return b * ((kBnParts + b - 1) / b); }

__device__ __forceinline__ float act(float v, float slope) {
  return v > 0.0f ? v : (slope == 0.0f ? 0.0f : v * slope);
}

// Block-wide sum of two values (256 threads); result valid in thread 0.
__device__ __forceinline__ void block_sum2(float& a, float& b, float* sh) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off, 64);
    b += __shfl_xor(b, off, 64);
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    sh[2 * w] = a;
    sh[2 * w + 1] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    a = ((sh[0] + sh[2]) + sh[4]) + sh[6];
    b = ((sh[1] + sh[3]) + sh[5]) + sh[7];
  }
}

// Stats passes: part p = (b, ps) of channel c covers float4s
// [ps * chunk, (ps + 1) * chunk) of row (b, c), PS = P / B parts per row.
__device__ __forceinline__ void part_range(int S4, int ps, int PS, int& s0, int& s1) {
  const int chunk = (S4 + PS - 1) / PS;
  s0 = min(S4, chunk * ps);
  s1 = min(S4, chunk * (ps + 1));
}

// grid = (C, P), 256 threads.  part[c][p] = (sum (x-K), sum (x-K)^2), K = x[0][c][0].
__global__ void __launch_bounds__(256)
    bn_stats_kernel(const float* __restrict__ x, int B, int C, int S, float* __restrict__ part) {
  __shared__ float sh[8];
  const int c = blockIdx.x, p = blockIdx.y, P = gridDim.y;
  const int S4 = S / 4;
  const float K = x[(size_t)c * S];
  const int PS = P / B, b = p / PS;
  int s0, s1;
  part_range(S4, p - b * PS, PS, s0, s1);
  const float4* __restrict__ x4 = reinterpret_cast<const float4*>(x) + ((size_t)b * C + c) * S4;
  float s = 0.0f, q = 0.0f;
  for (int s4 = s0 + threadIdx.x; s4 < s1; s4 += 256) {
    const float4 v = x4[s4];
    const float d0 = v.x - K, d1 = v.y - K, d2 = v.z - K, d3 = v.w - K;
    s += (d0 + d1) + (d2 + d3);
    q += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
  }
  block_sum2(s, q, sh);
  if (threadIdx.x == 0) {
    part[((size_t)c * P + p) * 2] = s;
    part[((size_t)c * P + p) * 2 + 1] = q;
  }
}

// one thread per channel: mean, invstd (biased variance, as BN normalises) and
// the running-stat update with the unbiased variance (torch's batch_norm).
__global__ void __launch_bounds__(256)
    bn_finalize_kernel(const float* __restrict__ part, const float* __restrict__ x, int B, int C,
                       int S, int P, float eps, float momentum, float* __restrict__ rmean,
                       float* __restrict__ rvar, float* __restrict__ mean,
                       float* __restrict__ invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.0f, q = 0.0f;
  for (int p = 0; p < P; ++p) {
    s += part[((size_t)c * P + p) * 2];
    q += part[((size_t)c * P + p) * 2 + 1];
  }
  const double n = (double)B * S;
  const float K = x[(size_t)c * S];
  const float md = (float)(s / n);
  const float var = fmaxf((float)(q / n) - md * md, 0.0f);
  const float m = K + md;
  mean[c] = m;
  invstd[c] = rsqrtf(var + eps);
  if (rmean != nullptr) {
    rmean[c] = (1.0f - momentum) * rmean[c] + momentum * m;
    rvar[c] = (1.0f - momentum) * rvar[c] + momentum * (float)(var * n / (n - 1.0));
  }
}

// y = act((x - mean) * invstd * gamma + beta), float4 per thread;
// grid = (ceil(S4 / 256), B * C).
__global__ void __launch_bounds__(256)
    bn_act_apply_kernel(const float* __restrict__ x, const float* __restrict__ mean,
                        const float* __restrict__ invstd, const float* __restrict__ gamma,
                        const float* __restrict__ beta, int C, int S4, float slope,
                        float* __restrict__ y) {
  const int s4 = blockIdx.x * 256 + threadIdx.x;
  if (s4 >= S4) return;
  const int c = (int)(blockIdx.y % C);
  const size_t i = (size_t)blockIdx.y * S4 + s4;
  const float m = mean[c], is = invstd[c], g = gamma[c], bt = beta[c];
  const float4 v = reinterpret_cast<const float4*>(x)[i];
  float4 o;
  o.x = act(__builtin_fmaf((v.x - m) * is, g, bt), slope);
  o.y = act(__builtin_fmaf((v.y - m) * is, g, bt), slope);
  o.z = act(__builtin_fmaf((v.z - m) * is, g, bt), slope);
  o.w = act(__builtin_fmaf((v.w - m) * is, g, bt), slope);
  reinterpret_cast<float4*>(y)[i] = o;
}

// grid = (C, P): part[c][p] = (sum g, sum g * xhat), g = dz * act'(bn(x)).
__global__ void __launch_bounds__(256)
    bn_bwd_stats_kernel(const float* __restrict__ dz, const float* __restrict__ x,
                        const float* __restrict__ mean, const float* __restrict__ invstd,
                        const float* __restrict__ gamma, const float* __restrict__ beta, int B,
                        int C, int S, float slope, float* __restrict__ part) {
  __shared__ float sh[8];
  const int c = blockIdx.x, p = blockIdx.y, P = gridDim.y;
  const int S4 = S / 4;
  const float m = mean[c], is = invstd[c], gm = gamma[c], bt = beta[c];
  const int PS = P / B, b = p / PS;
  int s0, s1;
  part_range(S4, p - b * PS, PS, s0, s1);
  const size_t row = ((size_t)b * C + c) * S4;
  const float4* __restrict__ x4 = reinterpret_cast<const float4*>(x) + row;
  const float4* __restrict__ d4 = reinterpret_cast<const float4*>(dz) + row;
  float sg = 0.0f, sgx = 0.0f;
  for (int s4 = s0 + threadIdx.x; s4 < s1; s4 += 256) {
    const float4 v = x4[s4], d = d4[s4];
    const float xv[4] = {v.x, v.y, v.z, v.w}, dv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xh = (xv[e] - m) * is;
      const float g = __builtin_fmaf(xh, gm, bt) > 0.0f ? dv[e] : dv[e] * slope;
      sg += g;
      sgx += g * xh;
    }
  }
  block_sum2(sg, sgx, sh);
  if (threadIdx.x == 0) {
    part[((size_t)c * P + p) * 2] = sg;
    part[((size_t)c * P + p) * 2 + 1] = sgx;
  }
}

__global__ void __launch_bounds__(256)
    bn_bwd_finalize_kernel(const float* __restrict__ part, int C, int P, float* __restrict__ dgamma,
                           float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float sg = 0.0f, sgx = 0.0f;
  for (int p = 0; p < P; ++p) {
    sg += part[((size_t)c * P + p) * 2];
    sgx += part[((size_t)c * P + p) * 2 + 1];
  }
  dbeta[c] = sg;
  dgamma[c] = sgx;
}

// dx = gamma * invstd * (g - dbeta / n - xhat * dgamma / n)
__global__ void __launch_bounds__(256)
    bn_bwd_apply_kernel(const float* __restrict__ dz, const float* __restrict__ x,
                        const float* __restrict__ mean, const float* __restrict__ invstd,
                        const float* __restrict__ gamma, const float* __restrict__ beta,
                        const float* __restrict__ dgamma, const float* __restrict__ dbeta, int C,
                        int S4, float inv_n, float slope, float* __restrict__ dx) {
  const int s4 = blockIdx.x * 256 + threadIdx.x;
  if (s4 >= S4) return;
  const int c = (int)(blockIdx.y % C);
  const size_t i = (size_t)blockIdx.y * S4 + s4;
  const float m = mean[c], is = invstd[c], gm = gamma[c], bt = beta[c];
  const float mg = dbeta[c] * inv_n, mgx = dgamma[c] * inv_n, k = gm * is;
  const float4 v = reinterpret_cast<const float4*>(x)[i];
  const float4 d = reinterpret_cast<const float4*>(dz)[i];
  const float xv[4] = {v.x, v.y, v.z, v.w}, dv[4] = {d.x, d.y, d.z, d.w};
  float o[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float xh = (xv[e] - m) * is;
    const float g = __builtin_fmaf(xh, gm, bt) > 0.0f ? dv[e] : dv[e] * slope;
    o[e] = k * ((g - mg) - xh * mgx);
  }
  reinterpret_cast<float4*>(dx)[i] = make_float4(o[0], o[1], o[2], o[3]);
}

bool bn_ok(int b, int c, int s) {
  return b > 0 && c > 0 && s > 0 && s % 4 == 0 && (long long)b * c < 65536 &&
         (long long)b * c * s < (1LL << 40);
}

}  // namespace
}  // namespace pcfm

using namespace pcfm;

extern "C" size_t pcfm_bn_workspace_bytes(int b, int c, int s) {
  if (!bn_ok(b, c, s)) return 0;
  return (size_t)c * bn_parts(b) * 2 * sizeof(float);
}

extern "C" int pcfm_bn_act_fwd(const float* x, const float* gamma, const float* beta, int b, int c,
                               int s, float eps, float slope, float momentum, float* running_mean,
                               float* running_var, float* y, float* mean, float* invstd, void* ws,
                               size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(bn_ok(b, c, s), "bn_act_fwd: bad shape b=%d c=%d s=%d (s %% 4 == 0 needed)", b,
                 c, s);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_bn_workspace_bytes(b, c, s), "bn_act_fwd: workspace too small");
  PCFM_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr),
                 "bn_act_fwd: running_mean and running_var must both be given or both NULL");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(c, bn_parts(b)), dim3(256), 0, st, x, b, c, s, part);
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(ceil_div(c, 256)), dim3(256), 0, st,
                     (const float*)part, x, b, c, s, bn_parts(b), eps, momentum, running_mean,
                     running_var, mean, invstd);
  hipLaunchKernelGGL(bn_act_apply_kernel, dim3(ceil_div(s / 4, 256), b * c), dim3(256), 0, st, x,
                     (const float*)mean, (const float*)invstd, gamma, beta, c, s / 4, slope, y);
  return check_launch("bn_act_fwd");
}

extern "C" int pcfm_bn_act_bwd(const float* dz, const float* x, const float* gamma,
                               const float* beta, const float* mean, const float* invstd, int b,
                               int c, int s, float slope, float* dx, float* dgamma, float* dbeta,
                               void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(bn_ok(b, c, s), "bn_act_bwd: bad shape b=%d c=%d s=%d (s %% 4 == 0 needed)", b,
                 c, s);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_bn_workspace_bytes(b, c, s), "bn_act_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  hipLaunchKernelGGL(bn_bwd_stats_kernel, dim3(c, bn_parts(b)), dim3(256), 0, st, dz, x, mean,
                     invstd, gamma, beta, b, c, s, slope, part);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(ceil_div(c, 256)), dim3(256), 0, st,
                     (const float*)part, c, bn_parts(b), dgamma, dbeta);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(ceil_div(s / 4, 256), b * c), dim3(256), 0, st, dz,
                     x, mean, invstd, gamma, beta, (const float*)dgamma, (const float*)dbeta, c,
                     s / 4, (float)(1.0 / ((double)b * s)), slope, dx);
  return check_launch("bn_act_bwd");
}
