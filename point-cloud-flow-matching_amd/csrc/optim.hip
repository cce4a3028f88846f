// The train step's parameter update (reference train.py:652-661): GradScaler
// unscale -> clip_grad_norm_ over every parameter -> AdamW (torch.optim.AdamW,
// train.py:249-253, its foreach arithmetic) -> EMA of the updated parameters
// (util.py:17-21).  torch runs this as ~40 multi-tensor launches over ~9M
// parameters (several passes per tensor list); here it is three launches:
//   adamw_sumsq_kernel     one pass over the gradients: per-chunk fp64 sum of
//                          squares (order fixed: deterministic)
//   adamw_finalize_kernel  1 block: total norm, non-finite flag, the gradient
//                          multiplier inv_scale * clip_coef, the step counts
//   adamw_ema_step_kernel  one pass: read g, p, m, v, ema; write p, m, v, ema
// Every parameter is an entry of a device table (pcfm_adamw_tensor); blocks
// walk a chunk table (tensor, first element) of kAdamwChunk elements each.
#include <cmath>

#include "pcfm_common.hpp"

namespace pcfm {
namespace {

constexpr int kAdamwChunk = PCFM_ADAMW_CHUNK;
constexpr int kVec4 = 1, kSkip = 2, kEma = 4;

__device__ __forceinline__ double block_sum_d(double a, double* sh) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off, 64);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) sh[w] = a;
  __syncthreads();
  return ((sh[0] + sh[1]) + sh[2]) + sh[3];
}

__global__ void __launch_bounds__(256)
    adamw_sumsq_kernel(const pcfm_adamw_tensor* __restrict__ tab, const int* __restrict__ chunks,
                       double* __restrict__ part) {
  __shared__ double sh[4];
  const int ti = chunks[2 * blockIdx.x], s0 = chunks[2 * blockIdx.x + 1];
  const pcfm_adamw_tensor t = tab[ti];
  double acc = 0.0;
  if (!(t.flags & kSkip)) {
    const long long e1 = min((long long)s0 + kAdamwChunk, t.n);
    if (t.flags & kVec4) {
      for (long long e = s0 + 4 * threadIdx.x; e < e1; e += 1024) {
        const float4 g = *reinterpret_cast<const float4*>(t.g + e);
        acc += ((double)g.x * g.x + (double)g.y * g.y) + ((double)g.z * g.z + (double)g.w * g.w);
      }
    } else {
      for (long long e = s0 + threadIdx.x; e < e1; e += 256) acc += (double)t.g[e] * t.g[e];
    }
  }
  acc = block_sum_d(acc, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// state: [0] total norm, [1] gradient multiplier, [2] found_inf (0 / 1,
// GradScaler's flag); steps[t]: tensor t's AdamW step count (torch keeps one
// per parameter: a parameter without gradient does not advance)
__global__ void __launch_bounds__(256)
    adamw_finalize_kernel(const double* __restrict__ part, int nchunks,
                          const pcfm_adamw_tensor* __restrict__ tab, int ntensors,
                          const float* __restrict__ scale, float max_norm,
                          float* __restrict__ steps, float* __restrict__ state) {
  __shared__ double sh[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < nchunks; i += 256) s += part[i];
  s = block_sum_d(s, sh);
  // The inf check is GradScaler's (train.py:652-657 with amp on): only with a
  // scale does a non-finite gradient skip the update -- and, as in
  // AdamW(fused=True), the step count.  Without one (amp off) torch's AdamW
  // steps anyway and the non-finite values reach the parameters.
  const bool found = scale != nullptr && !isfinite(s);
  if (!found)
    for (int t = threadIdx.x; t < ntensors; t += 256)
      if (!(tab[t].flags & kSkip)) steps[t] += 1.0f;
  if (threadIdx.x != 0) return;
  // GradScaler._unscale_grads_: inv_scale = scale.double().reciprocal().float()
  const float inv = scale != nullptr ? (float)(1.0 / (double)scale[0]) : 1.0f;
  // clip_grad_norm_ over the unscaled gradients (g * inv is exact: the scale is
  // a power of two), fp32 coefficient arithmetic as torch; clamp(max=1) keeps
  // a NaN coefficient NaN (fminf would not)
  const float total = (float)(sqrt(s) * (double)inv);
  float coef = 1.0f;
  if (max_norm > 0.0f) {
    const float c = max_norm / (total + 1e-6f);
    coef = isnan(c) ? c : fminf(c, 1.0f);
  }
  state[0] = total;
  state[1] = inv * coef;
  state[2] = found ? 1.0f : 0.0f;
}

struct AdamwHyper {  // python floats (double), cast where torch casts its scalars
  double lr[PCFM_ADAMW_MAX_GROUPS];
  double wd[PCFM_ADAMW_MAX_GROUPS];
  double beta1, beta2, eps, ema_decay;
};

struct AdamwScalars {
  float mult, decay_mul, m_w, beta2, v_w, bc2_sqrt, step_size, eps, e_d, e_w;
  bool skip;
};

__device__ __forceinline__ void adamw_elem(const AdamwScalars& k, float g, float& p, float& m,
                                           float& v) {
  g *= k.mult;
  // torch.optim.AdamW foreach path (_multi_tensor_adamw): p *= 1 - lr * wd;
  // m.lerp_(g, 1 - beta1); v = v * beta2 + (1 - beta2) g g;
  // p += -(lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
  p = p * k.decay_mul;
  m = m + k.m_w * (g - m);
  v = v * k.beta2 + k.v_w * (g * g);
  const float den = sqrtf(v) / k.bc2_sqrt + k.eps;
  p = p + k.step_size * (m / den);
}

__global__ void __launch_bounds__(256)
    adamw_ema_step_kernel(const pcfm_adamw_tensor* __restrict__ tab,
                          const int* __restrict__ chunks, const float* __restrict__ steps,
                          const float* __restrict__ state, AdamwHyper hp) {
  const int ti = chunks[2 * blockIdx.x], s0 = chunks[2 * blockIdx.x + 1];
  const pcfm_adamw_tensor t = tab[ti];
  AdamwScalars k;
  {
    const double step = (double)steps[ti];
    const double lr = hp.lr[t.group], wd = hp.wd[t.group];
    const double bc1 = 1.0 - pow(hp.beta1, step);
    const double bc2 = 1.0 - pow(hp.beta2, step);
    k.mult = state[1];
    k.skip = state[2] != 0.0f || (t.flags & kSkip);
    k.decay_mul = (float)(1.0 - lr * wd);
    k.m_w = (float)(1.0 - hp.beta1);
    k.beta2 = (float)hp.beta2;
    k.v_w = (float)(1.0 - hp.beta2);
    k.bc2_sqrt = (float)sqrt(bc2);
    k.step_size = (float)(-(lr / bc1));
    k.eps = (float)hp.eps;
    k.e_d = (float)hp.ema_decay;
    k.e_w = (float)(1.0 - hp.ema_decay);
  }
  const bool ema = (t.flags & kEma) != 0;
  if (k.skip && !ema) return;
  const long long e1 = min((long long)s0 + kAdamwChunk, t.n);
  if (t.flags & kVec4) {
    for (long long e = s0 + 4 * threadIdx.x; e < e1; e += 1024) {
      float4 p = *reinterpret_cast<const float4*>(t.p + e);
      if (!k.skip) {
        const float4 g = *reinterpret_cast<const float4*>(t.g + e);
        float4 m = *reinterpret_cast<const float4*>(t.m + e);
        float4 v = *reinterpret_cast<const float4*>(t.v + e);
        adamw_elem(k, g.x, p.x, m.x, v.x);
        adamw_elem(k, g.y, p.y, m.y, v.y);
        adamw_elem(k, g.z, p.z, m.z, v.z);
        adamw_elem(k, g.w, p.w, m.w, v.w);
        *reinterpret_cast<float4*>(t.p + e) = p;
        *reinterpret_cast<float4*>(t.m + e) = m;
        *reinterpret_cast<float4*>(t.v + e) = v;
      }
      if (ema) {  // shadow.mul_(d).add_(p, alpha=1 - d)
        float4 s = *reinterpret_cast<const float4*>(t.ema + e);
        s.x = s.x * k.e_d + k.e_w * p.x;
        s.y = s.y * k.e_d + k.e_w * p.y;
        s.z = s.z * k.e_d + k.e_w * p.z;
        s.w = s.w * k.e_d + k.e_w * p.w;
        *reinterpret_cast<float4*>(t.ema + e) = s;
      }
    }
  } else {
    for (long long e = s0 + threadIdx.x; e < e1; e += 256) {
      float p = t.p[e];
      if (!k.skip) {
        float m = t.m[e], v = t.v[e];
        adamw_elem(k, t.g[e], p, m, v);
        t.p[e] = p;
        t.m[e] = m;
        t.v[e] = v;
      }
      if (ema) t.ema[e] = t.ema[e] * k.e_d + k.e_w * p;
    }
  }
}

}  // namespace
}  // namespace pcfm

using namespace pcfm;

extern "C" int pcfm_adamw_chunk_elems(void) { return kAdamwChunk; }

extern "C" size_t pcfm_adamw_workspace_bytes(int nchunks) {
  return (size_t)(nchunks > 0 ? nchunks : 1) * sizeof(double);
}

extern "C" int pcfm_adamw_grad_norm(const pcfm_adamw_tensor* tensors, int ntensors,
                                    const int* chunks, int nchunks, const float* scale,
                                    float max_norm, float* steps, float* state, void* ws,
                                    size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(nchunks >= 0 && ntensors >= 0 && tensors != nullptr && chunks != nullptr &&
                     steps != nullptr && state != nullptr,
                 "adamw_grad_norm: bad arguments");
  PCFM_CHECK_ARG(ws != nullptr && ws_bytes >= pcfm_adamw_workspace_bytes(nchunks),
                 "adamw_grad_norm: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  double* part = (double*)ws;
  if (nchunks > 0)
    hipLaunchKernelGGL(adamw_sumsq_kernel, dim3(nchunks), dim3(256), 0, st, tensors, chunks,
                       part);
  hipLaunchKernelGGL(adamw_finalize_kernel, dim3(1), dim3(256), 0, st, part, nchunks, tensors,
                     ntensors, scale, max_norm, steps, state);
  return check_launch("adamw_grad_norm");
}

extern "C" int pcfm_adamw_ema_step(const pcfm_adamw_tensor* tensors, const int* chunks,
                                   int nchunks, const float* steps, const float* state,
                                   int ngroups,
                                   const double* lr, const double* weight_decay, double beta1,
                                   double beta2, double eps, double ema_decay, void* stream) {
  PCFM_CHECK_ARG(nchunks >= 0 && tensors != nullptr && chunks != nullptr && steps != nullptr &&
                     state != nullptr,
                 "adamw_ema_step: bad arguments");
  PCFM_CHECK_ARG(ngroups >= 1 && ngroups <= PCFM_ADAMW_MAX_GROUPS && lr != nullptr &&
                     weight_decay != nullptr,
                 "adamw_ema_step: 1..%d parameter groups", PCFM_ADAMW_MAX_GROUPS);
  AdamwHyper hp{};
  for (int i = 0; i < ngroups; ++i) {
    hp.lr[i] = lr[i];
    hp.wd[i] = weight_decay[i];
  }
  hp.beta1 = beta1;
  hp.beta2 = beta2;
  hp.eps = eps;
  hp.ema_decay = ema_decay;
  if (nchunks > 0)
    hipLaunchKernelGGL(adamw_ema_step_kernel, dim3(nchunks), dim3(256), 0, (hipStream_t)stream,
                       tensors, chunks, steps, state, hp);
  return check_launch("adamw_ema_step");
}
