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
#include <algorithm>

#include "pcfm_common.hpp"

namespace pcfm {
namespace {

// streamed 16-B store (the output is next read by another kernel, > L2)
__device__ __forceinline__ void nt_store4(float4* p, float4 v) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  nt_st(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f*>(p));
}


constexpr int kBnParts = 16;  // target blocks per channel in the stats passes
constexpr int kBnUnroll = 4;  // float4 loads per thread issued together in the stats passes
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
  auto add = [&](const float4 v) {
    const float d0 = v.x - K, d1 = v.y - K, d2 = v.z - K, d3 = v.w - K;
    s += (d0 + d1) + (d2 + d3);
    q += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
  };
  int s4 = s0 + threadIdx.x;
  // kBnUnroll float4 loads in flight per thread before the first use
  for (; s4 + (kBnUnroll - 1) * 256 < s1; s4 += kBnUnroll * 256) {
    float4 v[kBnUnroll];
#pragma unroll
    for (int u = 0; u < kBnUnroll; ++u) v[u] = x4[s4 + u * 256];
#pragma unroll
    for (int u = 0; u < kBnUnroll; ++u) add(v[u]);
  }
  for (; s4 < s1; s4 += 256) add(x4[s4]);
  block_sum2(s, q, sh);
  if (threadIdx.x == 0) {
    part[((size_t)c * P + p) * 2] = s;
    part[((size_t)c * P + p) * 2 + 1] = q;
  }
}

// s = sum of part[2p], q = sum of part[2p + 1] over p < P, added in p order;
// 8 partials' loads in flight at a time (the serial form kept the thread that
// derives a block's statistics waiting on one load per partial)
__device__ __forceinline__ void sum_parts2(const float* __restrict__ part, int P, float& s,
                                           float& q) {
  const float2* __restrict__ p2 = reinterpret_cast<const float2*>(part);
  s = 0.0f;
  q = 0.0f;
  int p = 0;
  for (; p + 8 <= P; p += 8) {
    float2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p2[p + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      s += v[u].x;
      q += v[u].y;
    }
  }
  for (; p < P; ++p) {
    const float2 v = p2[p];
    s += v.x;
    q += v.y;
  }
}

// one thread per channel: mean, invstd (biased variance, as BN normalises) and
// the running-stat update with the unbiased variance (torch's batch_norm).
__global__ void __launch_bounds__(256)
    bn_finalize_kernel(const float* __restrict__ part, const float* __restrict__ x, int B, int C,
                       int S, int P, float eps, float momentum, float* __restrict__ rmean,
                       float* __restrict__ rvar, float* __restrict__ mean,
                       float* __restrict__ invstd, long long* __restrict__ nbt = nullptr) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s, q;
  sum_parts2(part + (size_t)c * P * 2, P, s, q);
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
  if (nbt != nullptr && c == 0) nbt[0] += 1;
}

// bn_finalize / bn_bwd_finalize folded into the apply passes (one launch
// less each): every apply block re-derives its channel's statistics from the
// P partials with exactly the finalize arithmetic, and one designated block
// per channel writes mean / invstd (+ running stats) or dgamma / dbeta.
struct BnFwdFin {
  const float* part;
  int B, S, P;
  float eps, momentum;
  float* rmean;
  float* rvar;
  long long* nbt;  // BatchNorm num_batches_tracked (+1 by channel 0's publisher), or NULL
  __device__ __forceinline__ void get(const float* x, int c, float& m, float& is, float& var,
                                      double& n) const {
    float s, q;
    sum_parts2(part + (size_t)c * P * 2, P, s, q);
    n = (double)B * S;
    const float K = x[(size_t)c * S];
    const float md = (float)(s / n);
    var = fmaxf((float)(q / n) - md * md, 0.0f);
    m = K + md;
    is = rsqrtf(var + eps);
  }
  __device__ __forceinline__ void publish(int c, float m, float is, float var, double n,
                                          float* mean, float* invstd) const {
    mean[c] = m;
    invstd[c] = is;
    if (rmean != nullptr) {
      rmean[c] = (1.0f - momentum) * rmean[c] + momentum * m;
      rvar[c] = (1.0f - momentum) * rvar[c] + momentum * (float)(var * n / (n - 1.0));
    }
    if (nbt != nullptr && c == 0) nbt[0] += 1;
  }
};
__device__ __forceinline__ void bn_bwd_fin(const float* part, int P, int c, float& sg,
                                           float& sgx) {
  sum_parts2(part + (size_t)c * P * 2, P, sg, sgx);
}

// Statistics from a producer's epilogue (pw_gemm256_kernel with stats): part
// float2 [C][P], the (mean, centred sum of squares) of P groups of up to 64
// values, group p holding min(gsz, S - (p % G) gsz) values (G = ceil(S / gsz);
// gsz 64 from the 256-row tiles, 32 from the 128-row streaming form).
// Four waves per channel: thread t combines groups t, t + 256, ... in order
// (Chan's update, fp64; 4 groups' loads in flight at a time), then a fixed xor
// tree per wave and the 4 wave results in wave order; thread 0 publishes mean /
// invstd and the running statistics exactly as BnFwdFin::publish.
// Deterministic.  (One wave per channel walked ~40 dependent loads per lane:
// 17 us per launch at P = 2504.)
__device__ __forceinline__ void chan_merge(double& n, double& mu, double& m2, double nb, double mb,
                                           double qb) {
  const double nn = n + nb;
  if (nn > 0.0) {
    const double d = mb - mu;
    mu += d * nb / nn;
    m2 += qb + d * d * n * nb / nn;
  }
  n = nn;
}

__global__ void __launch_bounds__(256)
    bn_fin_parts_kernel(const float2* __restrict__ part, int P, int S, float eps, float momentum,
                        float* __restrict__ rmean, float* __restrict__ rvar,
                        long long* __restrict__ nbt, float* __restrict__ mean,
                        float* __restrict__ invstd, int gsz = 64) {
  const int c = blockIdx.x, t = threadIdx.x, l = t & 63, w = t >> 6;
  const int G = (S + gsz - 1) / gsz;
  double n = 0.0, mu = 0.0, m2 = 0.0;
  const float2* __restrict__ pc = part + (size_t)c * P;
  int p = t;
  for (; p + 3 * 256 < P; p += 4 * 256) {
    float2 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = pc[p + u * 256];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double nb = (double)min(gsz, S - ((p + u * 256) % G) * gsz);
      const double nn = n + nb, d = (double)v[u].x - mu;
      mu += d * nb / nn;
      m2 += (double)v[u].y + d * d * n * nb / nn;
      n = nn;
    }
  }
  for (; p < P; p += 256) {
    const float2 v = pc[p];
    const double nb = (double)min(gsz, S - (p % G) * gsz);
    const double nn = n + nb, d = (double)v.x - mu;
    mu += d * nb / nn;
    m2 += (double)v.y + d * d * n * nb / nn;
    n = nn;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
    chan_merge(n, mu, m2, __shfl_xor(n, o, 64), __shfl_xor(mu, o, 64), __shfl_xor(m2, o, 64));
  __shared__ double wr[4][3];
  if (l == 0) {
    wr[w][0] = n;
    wr[w][1] = mu;
    wr[w][2] = m2;
  }
  __syncthreads();
  if (t == 0) {
    n = wr[0][0];
    mu = wr[0][1];
    m2 = wr[0][2];
    for (int k = 1; k < 4; ++k) chan_merge(n, mu, m2, wr[k][0], wr[k][1], wr[k][2]);
  }
  if (t == 0) {
    const float var = fmaxf((float)(m2 / n), 0.0f);
    const float m = (float)mu;
    mean[c] = m;
    invstd[c] = rsqrtf(var + eps);
    if (rmean != nullptr) {
      rmean[c] = (1.0f - momentum) * rmean[c] + momentum * m;
      rvar[c] = (1.0f - momentum) * rvar[c] + momentum * (float)(var * n / (n - 1.0));
    }
    if (nbt != nullptr && c == 0) nbt[0] += 1;
  }
}

// y = act((x - mean) * invstd * gamma + beta), kApplyU float4 per thread;
// grid = (bn_apply_blocks(S), B * C).  Thread 0 derives the channel's
// statistics from the P partials once per block (LDS broadcast).
// The backward apply passes walk their blocks in REVERSE of the statistics
// pass's order (which reads the last batch element last): the rows read most
// recently are the ones still in the 256 MiB Infinity Cache (A/B on MI355X,
// tools/bn_ab.py: 158 -> 147 us at B8 C256 S20000, 123 -> 112 us at C128
// S32768; the forward apply, at 6.4 TB/s already, does not gain).
__device__ __forceinline__ unsigned bn_rev(unsigned i, unsigned n) { return rev_order(i, n); }

#ifndef PCFM_BN_APPLY_U
#define PCFM_BN_APPLY_U 4
#endif
#ifndef PCFM_BN_BWD_U
#define PCFM_BN_BWD_U 2
#endif
constexpr int kApplyU = PCFM_BN_APPLY_U;
constexpr int kBwdU = PCFM_BN_BWD_U;
inline int bn_apply_blocks(int s) { return ceil_div(s / 4, 256 * kApplyU); }
inline int bn_bwd_blocks(int s) { return ceil_div(s / 4, 256 * kBwdU); }

__global__ void __launch_bounds__(256)
    bn_act_apply_kernel(const float* __restrict__ x, BnFwdFin fin, float* __restrict__ mean,
                        float* __restrict__ invstd, const float* __restrict__ gamma,
                        const float* __restrict__ beta, int C, int S4, float slope,
                        float* __restrict__ y) {
  __shared__ float st[2];
  const unsigned row = blockIdx.y, bx = blockIdx.x;
  const int c = (int)(row % C);
  if (threadIdx.x == 0) {
    float m, is, var;
    double n;
    if (fin.part != nullptr) {
      fin.get(x, c, m, is, var, n);
      if (bx == 0 && row < (unsigned)C) fin.publish(c, m, is, var, n, mean, invstd);
    } else {  // statistics already final (bn_fin_parts_kernel)
      m = mean[c];
      is = invstd[c];
    }
    st[0] = m;
    st[1] = is;
  }
  const float g = gamma[c], bt = beta[c];
  const float4* __restrict__ x4 = reinterpret_cast<const float4*>(x) + (size_t)row * S4;
  float4* __restrict__ y4 = reinterpret_cast<float4*>(y) + (size_t)row * S4;
  const int s0 = bx * 256 * kApplyU + threadIdx.x;
  float4 v[kApplyU];
#pragma unroll
  for (int u = 0; u < kApplyU; ++u)
    if (s0 + u * 256 < S4) v[u] = x4[s0 + u * 256];
  __syncthreads();
  const float m = st[0], is = st[1];
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    if (s0 + u * 256 >= S4) break;
    float4 o;
    o.x = act(__builtin_fmaf((v[u].x - m) * is, g, bt), slope);
    o.y = act(__builtin_fmaf((v[u].y - m) * is, g, bt), slope);
    o.z = act(__builtin_fmaf((v[u].z - m) * is, g, bt), slope);
    o.w = act(__builtin_fmaf((v[u].w - m) * is, g, bt), slope);
#ifndef PCFM_BN_CACHED_STORE  // streamed: bwd apply 148 -> 128 us at C256 N20000 (tools/bn_ab.py)
    nt_store4(y4 + s0 + u * 256, o);
#else
    y4[s0 + u * 256] = o;
#endif
  }
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
  auto add = [&](const float4 v, const float4 d) {
    const float xv[4] = {v.x, v.y, v.z, v.w}, dv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xh = (xv[e] - m) * is;
      const float g = __builtin_fmaf(xh, gm, bt) > 0.0f ? dv[e] : dv[e] * slope;
      sg += g;
      sgx += g * xh;
    }
  };
  int s4 = s0 + threadIdx.x;
  // same per-thread summation order as one-at-a-time; only the loads move up
  for (; s4 + (kBnUnroll - 1) * 256 < s1; s4 += kBnUnroll * 256) {
    float4 v[kBnUnroll], d[kBnUnroll];
#pragma unroll
    for (int u = 0; u < kBnUnroll; ++u) {
      v[u] = x4[s4 + u * 256];
      d[u] = d4[s4 + u * 256];
    }
#pragma unroll
    for (int u = 0; u < kBnUnroll; ++u) add(v[u], d[u]);
  }
  for (; s4 < s1; s4 += 256) add(x4[s4], d4[s4]);
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
  float sg, sgx;
  sum_parts2(part + (size_t)c * P * 2, P, sg, sgx);
  dbeta[c] = sg;
  dgamma[c] = sgx;
}

// dx = gamma * invstd * (g - dbeta / n - xhat * dgamma / n), kBwdU float4
// per thread; grid (bn_bwd_blocks(S), B*C).  With rowpart: the block's sum of
// dx -> rowpart[row][block] (producer bias grad).
__global__ void __launch_bounds__(256)
    bn_bwd_apply_kernel(const float* __restrict__ dz, const float* __restrict__ x,
                        const float* __restrict__ mean, const float* __restrict__ invstd,
                        const float* __restrict__ gamma, const float* __restrict__ beta,
                        const float* __restrict__ part, int P, float* __restrict__ dgamma,
                        float* __restrict__ dbeta, int C,
                        int S4, float inv_n, float slope, float* __restrict__ dx,
                        float* __restrict__ rowpart) {
  __shared__ float sh[8];
  __shared__ float st[2];
  const unsigned row = bn_rev(blockIdx.y, gridDim.y), bx = bn_rev(blockIdx.x, gridDim.x);
  const int c = (int)(row % C);
  if (threadIdx.x == 0) {
    float sg, sgx;
    bn_bwd_fin(part, P, c, sg, sgx);
    if (bx == 0 && row < (unsigned)C) {
      dbeta[c] = sg;
      dgamma[c] = sgx;
    }
    st[0] = sg;
    st[1] = sgx;
  }
  const float m = mean[c], is = invstd[c], gm = gamma[c], bt = beta[c];
  const size_t r0 = (size_t)row * S4;
  const float4* __restrict__ x4 = reinterpret_cast<const float4*>(x) + r0;
  const float4* __restrict__ d4 = reinterpret_cast<const float4*>(dz) + r0;
  float4* __restrict__ o4 = reinterpret_cast<float4*>(dx) + r0;
  const int s0 = bx * 256 * kBwdU + threadIdx.x;
  float4 v[kBwdU], d[kBwdU];
#pragma unroll
  for (int u = 0; u < kBwdU; ++u)
    if (s0 + u * 256 < S4) {
      v[u] = x4[s0 + u * 256];
      d[u] = d4[s0 + u * 256];
    }
  __syncthreads();
  const float mg = st[0] * inv_n, mgx = st[1] * inv_n, k = gm * is;
  float tsum = 0.0f;
#pragma unroll
  for (int u = 0; u < kBwdU; ++u) {
    if (s0 + u * 256 >= S4) break;
    const float xv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
    const float dv[4] = {d[u].x, d[u].y, d[u].z, d[u].w};
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xh = (xv[e] - m) * is;
      const float g = __builtin_fmaf(xh, gm, bt) > 0.0f ? dv[e] : dv[e] * slope;
      o[e] = k * ((g - mg) - xh * mgx);
    }
#ifndef PCFM_BN_CACHED_STORE
    nt_store4(o4 + s0 + u * 256, make_float4(o[0], o[1], o[2], o[3]));
#else
    o4[s0 + u * 256] = make_float4(o[0], o[1], o[2], o[3]);
#endif
    tsum += (o[0] + o[1]) + (o[2] + o[3]);
  }
  if (rowpart != nullptr) {  // block-uniform branch: every thread takes part
    float z = 0.0f;
    block_sum2(tsum, z, sh);
    if (threadIdx.x == 0) rowpart[(size_t)row * gridDim.x + bx] = tsum;
  }
}

// dbias[c] = sum over (b, k) of rowpart[(b * C + c) * nch + k]: one wave per
// channel, lane-strided in a fixed order, then a fixed xor tree (deterministic)
__global__ void __launch_bounds__(256)
    bn_bias_finalize_kernel(const float* __restrict__ rowpart, int B, int C, int nch,
                            float* __restrict__ dbias) {
  const int c = blockIdx.x * 4 + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= C) return;  // wave-uniform
  float s = 0.0f;
  const int tot = B * nch;
  for (int e = lane; e < tot; e += 64) {
    const int b = e / nch, k = e - b * nch;
    s += rowpart[((size_t)b * C + c) * nch + k];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) dbias[c] = s;
}

// dbias[c] = sum over (b, k) of rowpart[(b * C + c) * nch + k] for long rows:
// one block per channel, thread-strided in a fixed order, then a fixed tree.
__global__ void __launch_bounds__(256)
    bn_bias_finalize_block_kernel(const float* __restrict__ rowpart, int B, int C, int nch,
                                  float* __restrict__ dbias) {
  __shared__ float sh[8];
  const int c = blockIdx.x;
  float s = 0.0f;
  for (int bb = 0; bb < B; ++bb) {
    const float* __restrict__ rp = rowpart + ((size_t)bb * C + c) * nch;
    for (int k = threadIdx.x; k < nch; k += 256) s += rp[k];
  }
  float z = 0.0f;
  block_sum2(s, z, sh);
  if (threadIdx.x == 0) dbias[c] = s;
}

// BN backward apply for a voxel convolution's output, fused with the
// channels-last bf16 hi/lo split the convolution's backward reads
// (conv3_split_cl_kernel): dx is never written as fp32 [B][C][V].
// grid = (S / 64, C / 64, B), 256 threads; a 64 x 64 LDS tile.
// rowpart[(b * C + c) * (S / 64) + vb] = sum of dx over the tile's 64 voxels
// (fixed order: 16 sequential per thread, then a 4-lane xor tree).
typedef __bf16 bn_bf16x2 __attribute__((ext_vector_type(2)));

// A 64 (channel) x 64 (voxel) fp32 LDS tile -> channels-last bf16 hi / lo
// rows [b][v][c] interleaved per 32 channels (conv3_split_cl_kernel's layout,
// split_off, and rounding), 256 threads:
// thread t writes 16 channels of voxel t / 4.
__device__ __forceinline__ void tile_store_split(const float (&tile)[64][65], int b, int C, int S,
                                                 int v0, int c0, int t, uint16_t* __restrict__ h,
                                                 uint16_t* __restrict__ l) {
  const int v = t >> 2, cg = (t & 3) * 16;
  const size_t o = split_off((size_t)b * S + v0 + v, c0 + cg, C);  // l = h + kSplitLo
  uint32_t* h32 = reinterpret_cast<uint32_t*>(h + o);
  uint32_t* l32 = reinterpret_cast<uint32_t*>(l + o);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float f0 = tile[cg + 2 * q][v], f1 = tile[cg + 2 * q + 1][v];
    bn_bf16x2 hi, lo;
    hi.x = (__bf16)f0;
    hi.y = (__bf16)f1;
    lo.x = (__bf16)(f0 - (float)hi.x);
    lo.y = (__bf16)(f1 - (float)hi.y);
    h32[q] = __builtin_bit_cast(uint32_t, hi);
    l32[q] = __builtin_bit_cast(uint32_t, lo);
  }
}

// act(bn(x)) written directly as the next convolution's split input (the
// fp32 activation is never materialised); grid = (S / 64, C / 64, B).
__global__ void __launch_bounds__(256)
    bn_act_apply_split_kernel(const float* __restrict__ x, BnFwdFin fin,
                              float* __restrict__ mean, float* __restrict__ invstd,
                              const float* __restrict__ gamma,
                              const float* __restrict__ beta, int C, int S, float slope,
                              uint16_t* __restrict__ yh, uint16_t* __restrict__ yl) {
  __shared__ float tile[64][65];
  __shared__ float st_m[64], st_is[64];
  const unsigned bx = blockIdx.x;
  const int v0 = bx * 64, c0 = blockIdx.y * 64, b = blockIdx.z;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  if (t < 64) {
    float m, is, var;
    double n;
    fin.get(x, c0 + t, m, is, var, n);
    st_m[t] = m;
    st_is[t] = is;
    if (bx == 0 && b == 0) fin.publish(c0 + t, m, is, var, n, mean, invstd);
  }
  __syncthreads();
  const size_t rbase = ((size_t)b * C + c0) * S + v0;
  float xv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) xv[i] = x[rbase + (size_t)(4 * i + w) * S + lane];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = c0 + 4 * i + w;
    tile[4 * i + w][lane] =
        act(__builtin_fmaf((xv[i] - st_m[c - c0]) * st_is[c - c0], gamma[c], beta[c]), slope);
  }
  __syncthreads();
  tile_store_split(tile, b, C, S, v0, c0, t, yh, yl);
}
__global__ void __launch_bounds__(256)
    bn_bwd_apply_split_kernel(const float* __restrict__ dz, const float* __restrict__ x,
                              const float* __restrict__ mean, const float* __restrict__ invstd,
                              const float* __restrict__ gamma, const float* __restrict__ beta,
                              const float* __restrict__ part, int P, float* __restrict__ dgamma,
                              float* __restrict__ dbeta,
                              int C, int S, float inv_n, float slope, uint16_t* __restrict__ dxh,
                              uint16_t* __restrict__ dxl, float* __restrict__ rowpart) {
  __shared__ float tile[64][65];
  __shared__ float st_g[64], st_gx[64];
  const unsigned bx = bn_rev(blockIdx.x, gridDim.x);
  const int v0 = bx * 64, c0 = blockIdx.y * 64, b = bn_rev(blockIdx.z, gridDim.z);
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  if (t < 64) {
    float sg, sgx;
    bn_bwd_fin(part, P, c0 + t, sg, sgx);
    st_g[t] = sg;
    st_gx[t] = sgx;
    if (bx == 0 && b == 0) {
      dbeta[c0 + t] = sg;
      dgamma[c0 + t] = sgx;
    }
  }
  __syncthreads();
  const size_t rbase = ((size_t)b * C + c0) * S + v0;
  float xv[16], dv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const size_t o = rbase + (size_t)(4 * i + w) * S + lane;
    xv[i] = x[o];
    dv[i] = dz[o];
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = c0 + 4 * i + w;
    const float m = mean[c], is = invstd[c], gm = gamma[c], bt = beta[c];
    const float mg = st_g[c - c0] * inv_n, mgx = st_gx[c - c0] * inv_n, k = gm * is;
    const float xh = (xv[i] - m) * is;
    const float g = __builtin_fmaf(xh, gm, bt) > 0.0f ? dv[i] : dv[i] * slope;
    tile[4 * i + w][lane] = k * ((g - mg) - xh * mgx);
  }
  __syncthreads();
  tile_store_split(tile, b, C, S, v0, c0, t, dxh, dxl);
  if (rowpart != nullptr) {
    const int c = t >> 2, vq = (t & 3) * 16;
    float sum = 0.0f;
#pragma unroll
    for (int q = 0; q < 16; ++q) sum += tile[c][vq + q];
    sum += __shfl_xor(sum, 1, 64);
    sum += __shfl_xor(sum, 2, 64);
    if ((t & 3) == 0) rowpart[((size_t)b * C + c0 + c) * (S / 64) + bx] = sum;
  }
}

// ---------------------------------------------------------------------------
// PVConv's second voxel BatchNorm + LeakyReLU fused with SE3d and the
// devoxelization (pvconv.py:20-39, se.py:6-17): z = act(bn(x)) is never
// written.  Forward: the batch statistics, then ONE pass computing the SE
// pooling m[b][c] = mean_v z (bn_act_rowsum_kernel); the devoxelization
// gather applies bn + act to the rows while staging them (rows.hpp RowBn).
// Backward from g = devox_bwd(dout): dz = s[b][c] g + dmv[b][c] (SE's scale and
// the pooling's gradient dm / V), so every sum BatchNorm's backward needs is
// linear in (s, dmv) -- per (b, c) row, with a = act'(bn(x)), xh = xhat:
//   ds = sum z g,  A = sum a g,  N = sum a,  AX = sum a g xh,  NX = sum a xh
//   sum a dz = s A + dmv N,   sum a dz xh = s AX + dmv NX
// ONE pass over (g, x) gives all five (bn_se_bwd_stats_kernel); the SE MLP's
// backward turns ds into dmv; the apply pass writes dx as the conv's split
// operand (bn_se_bwd_apply_split_kernel).  The SE rows_dot passes, the
// rows_affine pass over g and the separate backward statistics pass are gone.
// ---------------------------------------------------------------------------

// grid (bn_apply_blocks(S), B * C): rowpart[row][bx] = sum over the block's
// elements of act(bn(x)); thread 0 derives the channel statistics from the
// partials (block bx == 0 of the first C rows publishes them, as the apply).
__global__ void __launch_bounds__(256)
    bn_act_rowsum_kernel(const float* __restrict__ x, BnFwdFin fin, float* __restrict__ mean,
                         float* __restrict__ invstd, const float* __restrict__ gamma,
                         const float* __restrict__ beta, int C, int S4, float slope,
                         float* __restrict__ rowpart) {
  __shared__ float sh[8];
  __shared__ float st[2];
  const unsigned row = blockIdx.y, bx = blockIdx.x;
  const int c = (int)(row % C);
  if (threadIdx.x == 0) {
    float m, is, var;
    double n;
    fin.get(x, c, m, is, var, n);
    if (bx == 0 && row < (unsigned)C) fin.publish(c, m, is, var, n, mean, invstd);
    st[0] = m;
    st[1] = is;
  }
  const float g = gamma[c], bt = beta[c];
  const float4* __restrict__ x4 = reinterpret_cast<const float4*>(x) + (size_t)row * S4;
  const int s0 = bx * 256 * kApplyU + threadIdx.x;
  float4 v[kApplyU];
#pragma unroll
  for (int u = 0; u < kApplyU; ++u)
    if (s0 + u * 256 < S4) v[u] = x4[s0 + u * 256];
  __syncthreads();
  const float m = st[0], is = st[1];
  float sum = 0.0f;
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    if (s0 + u * 256 >= S4) break;
    sum += (act(__builtin_fmaf((v[u].x - m) * is, g, bt), slope) +
            act(__builtin_fmaf((v[u].y - m) * is, g, bt), slope)) +
           (act(__builtin_fmaf((v[u].z - m) * is, g, bt), slope) +
            act(__builtin_fmaf((v[u].w - m) * is, g, bt), slope));
  }
  float z = 0.0f;
  block_sum2(sum, z, sh);
  if (threadIdx.x == 0) rowpart[(size_t)row * gridDim.x + bx] = sum;
}

// one thread per row: out[row] = scale * sum of its nblk partials, in order
__global__ void __launch_bounds__(256)
    rowpart_sum_kernel(const float* __restrict__ rowpart, int rows, int nblk, float scale,
                       float* __restrict__ out) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  const float* __restrict__ p = rowpart + (size_t)r * nblk;
  float s = 0.0f;
  for (int k = 0; k < nblk; ++k) s += p[k];
  out[r] = s * scale;
}

// grid (PS, B * C), PS = bn_parts(B) / B blocks per row:
// part[(row * PS + ps) * 5 + k] = the five sums above over the block's range.
constexpr int kSeSums = 5;
__global__ void __launch_bounds__(256)
    bn_se_bwd_stats_kernel(const float* __restrict__ g, const float* __restrict__ x,
                           const float* __restrict__ mean, const float* __restrict__ invstd,
                           const float* __restrict__ gamma, const float* __restrict__ beta, int C,
                           int S, float slope, float* __restrict__ part) {
  __shared__ float sh[8 * kSeSums];
  const unsigned row = blockIdx.y;
  const int c = (int)(row % C), ps = blockIdx.x, PS = gridDim.x;
  const int S4 = S / 4;
  int s0, s1;
  part_range(S4, ps, PS, s0, s1);
  const float m = mean[c], is = invstd[c], gm = gamma[c], bt = beta[c];
  const float4* __restrict__ x4 = reinterpret_cast<const float4*>(x) + (size_t)row * S4;
  const float4* __restrict__ g4 = reinterpret_cast<const float4*>(g) + (size_t)row * S4;
  float acc[kSeSums] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};  // ds, A, N, AX, NX
  auto add = [&](const float4 v, const float4 d) {
    const float xv[4] = {v.x, v.y, v.z, v.w}, dv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xh = (xv[e] - m) * is;
      const float t = __builtin_fmaf(xh, gm, bt);
      const float a = t > 0.0f ? 1.0f : slope;
      const float z = t > 0.0f ? t : (slope == 0.0f ? 0.0f : t * slope);
      const float ag = a * dv[e];
      acc[0] = __builtin_fmaf(z, dv[e], acc[0]);
      acc[1] += ag;
      acc[2] += a;
      acc[3] = __builtin_fmaf(ag, xh, acc[3]);
      acc[4] = __builtin_fmaf(a, xh, acc[4]);
    }
  };
  int s4 = s0 + threadIdx.x;
  for (; s4 + (kBnUnroll - 1) * 256 < s1; s4 += kBnUnroll * 256) {
    float4 v[kBnUnroll], d[kBnUnroll];
#pragma unroll
    for (int u = 0; u < kBnUnroll; ++u) {
      v[u] = x4[s4 + u * 256];
      d[u] = g4[s4 + u * 256];
    }
#pragma unroll
    for (int u = 0; u < kBnUnroll; ++u) add(v[u], d[u]);
  }
  for (; s4 < s1; s4 += 256) add(x4[s4], g4[s4]);
  // block sum of the five values: xor tree per wave, then the 4 waves in order
#pragma unroll
  for (int k = 0; k < kSeSums; ++k)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc[k] += __shfl_xor(acc[k], off, 64);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < kSeSums; ++k) sh[w * kSeSums + k] = acc[k];
  __syncthreads();
  if (threadIdx.x < kSeSums) {
    const int k = threadIdx.x;
    part[((size_t)row * PS + ps) * kSeSums + k] =
        ((sh[k] + sh[kSeSums + k]) + sh[2 * kSeSums + k]) + sh[3 * kSeSums + k];
  }
}

// one thread per (row, sum): rowstats[k][row] = sum over the row's PS parts, in order
__global__ void __launch_bounds__(256)
    bn_se_rowstats_kernel(const float* __restrict__ part, int rows, int PS,
                          float* __restrict__ rowstats) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * kSeSums) return;
  const int row = i / kSeSums, k = i - row * kSeSums;
  const float* __restrict__ p = part + (size_t)row * PS * kSeSums + k;
  float s = 0.0f;
  for (int q = 0; q < PS; ++q) s += p[(size_t)q * kSeSums];
  rowstats[(size_t)k * rows + row] = s;
}

// bn_bwd_apply_split_kernel for dz = s[b][c] g + dmv[b][c]; the per-channel
// sums from rowstats [5][B][C] (summed over b in order).
__global__ void __launch_bounds__(256)
    bn_se_bwd_apply_split_kernel(const float* __restrict__ g, const float* __restrict__ x,
                                 const float* __restrict__ mean, const float* __restrict__ invstd,
                                 const float* __restrict__ gamma, const float* __restrict__ beta,
                                 const float* __restrict__ se_s, const float* __restrict__ dmv,
                                 const float* __restrict__ rowstats, int B,
                                 float* __restrict__ dgamma, float* __restrict__ dbeta, int C,
                                 int S, float inv_n, float slope, uint16_t* __restrict__ dxh,
                                 uint16_t* __restrict__ dxl, float* __restrict__ rowpart) {
  __shared__ float tile[64][65];
  __shared__ float st_g[64], st_gx[64], st_s[64], st_t[64];
  const unsigned bx = bn_rev(blockIdx.x, gridDim.x);
  const int v0 = bx * 64, c0 = blockIdx.y * 64, b = bn_rev(blockIdx.z, gridDim.z);
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  if (t < 64) {
    const int c = c0 + t;
    const size_t BC = (size_t)B * C;
    float sg = 0.0f, sgx = 0.0f;
    for (int bb = 0; bb < B; ++bb) {
      const size_t r = (size_t)bb * C + c;
      const float sv = se_s[r], tv = dmv[r];
      sg += __builtin_fmaf(sv, rowstats[BC + r], tv * rowstats[2 * BC + r]);
      sgx += __builtin_fmaf(sv, rowstats[3 * BC + r], tv * rowstats[4 * BC + r]);
    }
    st_g[t] = sg;
    st_gx[t] = sgx;
    st_s[t] = se_s[(size_t)b * C + c];
    st_t[t] = dmv[(size_t)b * C + c];
    if (bx == 0 && b == 0) {
      dbeta[c] = sg;
      dgamma[c] = sgx;
    }
  }
  __syncthreads();
  const size_t rbase = ((size_t)b * C + c0) * S + v0;
  float xv[16], dv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const size_t o = rbase + (size_t)(4 * i + w) * S + lane;
    xv[i] = x[o];
    dv[i] = g[o];
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int cl = 4 * i + w, c = c0 + cl;
    const float m = mean[c], is = invstd[c], gm = gamma[c], bt = beta[c];
    const float mg = st_g[cl] * inv_n, mgx = st_gx[cl] * inv_n, k = gm * is;
    const float xh = (xv[i] - m) * is;
    const float dz = __builtin_fmaf(st_s[cl], dv[i], st_t[cl]);  // rows_affine's expression
    const float gg = __builtin_fmaf(xh, gm, bt) > 0.0f ? dz : dz * slope;
    tile[cl][lane] = k * ((gg - mg) - xh * mgx);
  }
  __syncthreads();
  tile_store_split(tile, b, C, S, v0, c0, t, dxh, dxl);
  if (rowpart != nullptr) {
    const int c = t >> 2, vq = (t & 3) * 16;
    float sum = 0.0f;
#pragma unroll
    for (int q = 0; q < 16; ++q) sum += tile[c][vq + q];
    sum += __shfl_xor(sum, 1, 64);
    sum += __shfl_xor(sum, 2, 64);
    if ((t & 3) == 0) rowpart[((size_t)b * C + c0 + c) * (S / 64) + bx] = sum;
  }
}

// ---------------------------------------------------------------------------
// GroupNorm + FiLM + residual of the hybrid backbone's PV blocks
// (reference models.py:322-346 _FiLM1d with GroupNorm, :349-368 _PVBlock):
//   out = x + (GN(x) * (1 + gamma[b]) + beta[b])
//   GN(x)[b, c, n] = (x - mean[b, g]) * rstd[b, g] * w[c] + bias[c],  g = c / (C / G)
// evaluated as torch does: y = x * a + s with a = rstd * w, s = bias - mean * a,
// then y * (1 + gamma) + beta, then + x.
// Backward with A2[b, c] = sum_n dout, A3[b, c] = sum_n dout * xhat:
//   d beta = A2, d gamma = w A3 + bias A2, d w = sum_b (1+gamma) A3,
//   d bias = sum_b (1+gamma) A2, and per group
//   dx = dout + rstd (dout (1+gamma) w - mean_g(dy w) - xhat mean_g(dy w xhat)).
// ---------------------------------------------------------------------------
constexpr int kGnParts = 4;  // blocks per (b, group) row set / per (b, c) row

// GroupNorm over the activation of a SharedMLP layer given as its pre-BatchNorm
// tensor y (the PV block's post layer, models.py:349-368): the GroupNorm reads
// z = act(bn(y)) = act(fma((y - m) * is, g, bt)) -- bn_act_apply_kernel's
// arithmetic, so z is bit-identical to the activation it no longer writes.
struct BnIn {
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  float slope;
};
struct BnInC {
  float m, is, g, bt, slope;
  __device__ __forceinline__ float xh(float v) const { return (v - m) * is; }
  __device__ __forceinline__ float z(float v) const {
    return act(__builtin_fmaf((v - m) * is, g, bt), slope);
  }
  // the BatchNorm backward's g = dz * act'(bn(y)) (bn_bwd_stats_kernel's form)
  __device__ __forceinline__ float grad(float v, float dz) const {
    return __builtin_fmaf(xh(v), g, bt) > 0.0f ? dz : dz * slope;
  }
};
__device__ __forceinline__ BnInC bnin_at(const BnIn& p, int c) {
  return BnInC{p.mean[c], p.invstd[c], p.gamma[c], p.beta[c], p.slope};
}

// fwd stats: grid (G * kGnParts, B); part[(b*G + g)*P + p] = (sum (x-K), sum (x-K)^2)
// IN: over z = act(bn(x)) (BnIn), K = z of the group's first element
template <bool IN>
__global__ void __launch_bounds__(256)
    gn_stats_kernel(const float* __restrict__ x, int C, int N, int G, float* __restrict__ part,
                    BnIn bn = {}) {
  __shared__ float sh[8];
  const int b = blockIdx.y, g = blockIdx.x / kGnParts, p = blockIdx.x % kGnParts;
  const int cpg = C / G, N4 = N / 4;
  const float* base = x + ((size_t)b * C + (size_t)g * cpg) * N;  // cpg rows of N, contiguous
  const float K = IN ? bnin_at(bn, g * cpg).z(base[0]) : base[0];
  const int tot = cpg * N4, chunk = (tot + kGnParts - 1) / kGnParts;
  const int f0 = min(tot, p * chunk), f1 = min(tot, f0 + chunk);
  const float4* x4 = reinterpret_cast<const float4*>(base);
  float s = 0.0f, q = 0.0f;
  // IN: the thread's current channel (its stride, 256 float4s, is below a row's N4)
  int f = f0 + threadIdx.x, bnd = 0;
  BnInC tc{};
  if (IN && f < f1) {
    const int cl = f / N4;
    bnd = (cl + 1) * N4;
    tc = bnin_at(bn, g * cpg + cl);
  }
  for (; f < f1; f += 256) {
    float4 v = x4[f];
    if (IN) {
      if (f >= bnd) {
        const int cl = f / N4;
        bnd = (cl + 1) * N4;
        tc = bnin_at(bn, g * cpg + cl);
      }
      v = make_float4(tc.z(v.x), tc.z(v.y), tc.z(v.z), tc.z(v.w));
    }
    const float d0 = v.x - K, d1 = v.y - K, d2 = v.z - K, d3 = v.w - K;
    s += (d0 + d1) + (d2 + d3);
    q += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
  }
  block_sum2(s, q, sh);
  if (threadIdx.x == 0) {
    part[(((size_t)b * G + g) * kGnParts + p) * 2] = s;
    part[(((size_t)b * G + g) * kGnParts + p) * 2 + 1] = q;
  }
}

// one thread per (b, c): group stats -> a = rstd*w, s = bias - mean*a, g1 = 1 + gamma
__global__ void __launch_bounds__(256)
    gn_finalize_kernel(const float* __restrict__ part, const float* __restrict__ x,
                       const float* __restrict__ w, const float* __restrict__ bias,
                       const float* __restrict__ gamma, int B, int C, int N, int G, float eps,
                       float* __restrict__ mean_o, float* __restrict__ rstd_o,
                       float* __restrict__ coef, BnIn bn = {}) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * C) return;
  const int b = i / C, c = i - b * C, cpg = C / G, g = c / cpg;
  float s = 0.0f, q = 0.0f;
  for (int p = 0; p < kGnParts; ++p) {
    s += part[(((size_t)b * G + g) * kGnParts + p) * 2];
    q += part[(((size_t)b * G + g) * kGnParts + p) * 2 + 1];
  }
  const double n = (double)cpg * N;
  float K = x[((size_t)b * C + (size_t)g * cpg) * N];
  if (bn.mean != nullptr) K = bnin_at(bn, g * cpg).z(K);
  const float md = (float)(s / n);
  const float var = fmaxf((float)(q / n) - md * md, 0.0f);
  const float mean = K + md, rstd = rsqrtf(var + eps);
  if (c % cpg == 0) {
    mean_o[b * G + g] = mean;
    rstd_o[b * G + g] = rstd;
  }
  const float a = rstd * w[c];
  coef[3 * (size_t)i] = a;
  coef[3 * (size_t)i + 1] = bias[c] - mean * a;
  coef[3 * (size_t)i + 2] = gamma != nullptr ? 1.0f + gamma[i] : 1.0f;
}

// torch's SiLU x / (1 + exp(-x)) and its derivative s (1 + x (1 - s))
__device__ __forceinline__ float gn_silu(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float gn_dsilu(float x) {
  const float sg = 1.0f / (1.0f + expf(-x));
  return sg * (1.0f + x * (1.0f - sg));
}

// ContextNet's head: out = SiLU(GN(x)) = SiLU(x * a + s); grid (ceil(N4 / 256), B * C)
__global__ void __launch_bounds__(256)
    gn_silu_apply_kernel(const float* __restrict__ x, const float* __restrict__ coef, int N4,
                         float* __restrict__ out) {
  const int n4 = blockIdx.x * 256 + threadIdx.x;
  if (n4 >= N4) return;
  const int row = blockIdx.y;
  const float a = coef[3 * (size_t)row], sh = coef[3 * (size_t)row + 1];
  const size_t i = (size_t)row * N4 + n4;
  const float4 v = reinterpret_cast<const float4*>(x)[i];
  float4 o;
  o.x = gn_silu(__builtin_fmaf(v.x, a, sh));
  o.y = gn_silu(__builtin_fmaf(v.y, a, sh));
  o.z = gn_silu(__builtin_fmaf(v.z, a, sh));
  o.w = gn_silu(__builtin_fmaf(v.w, a, sh));
  reinterpret_cast<float4*>(out)[i] = o;
}

// out = x + ((x * a + s) * g1 + beta); grid (ceil(N4 / 256), B * C)
// IN: x -> z = act(bn(x)) first (the residual is z too)
template <bool IN>
__global__ void __launch_bounds__(256)
    gn_film_apply_kernel(const float* __restrict__ x, const float* __restrict__ coef,
                         const float* __restrict__ beta, int N4, float* __restrict__ out,
                         int C = 1, BnIn bn = {}) {
  const int n4 = blockIdx.x * 256 + threadIdx.x;
  if (n4 >= N4) return;
  const int row = blockIdx.y;
  const float a = coef[3 * (size_t)row], s = coef[3 * (size_t)row + 1];
  const float g1 = coef[3 * (size_t)row + 2], bt = beta[row];
  const size_t i = (size_t)row * N4 + n4;
  float4 v = reinterpret_cast<const float4*>(x)[i];
  if (IN) {
    const BnInC tc = bnin_at(bn, row % C);
    v = make_float4(tc.z(v.x), tc.z(v.y), tc.z(v.z), tc.z(v.w));
  }
  float4 o;
  o.x = v.x + (__builtin_fmaf(v.x, a, s) * g1 + bt);
  o.y = v.y + (__builtin_fmaf(v.y, a, s) * g1 + bt);
  o.z = v.z + (__builtin_fmaf(v.z, a, s) * g1 + bt);
  o.w = v.w + (__builtin_fmaf(v.w, a, s) * g1 + bt);
#ifdef PCFM_GN_NT_STORE
  nt_store4(reinterpret_cast<float4*>(out) + i, o);
#else
  reinterpret_cast<float4*>(out)[i] = o;
#endif
}

// bwd row sums: grid (kGnParts, B * C); part[row * P + p] = (sum dout, sum dout * xhat)
// ACT (GN + SiLU): the gradient entering GN is dout * SiLU'(x * a + s), recomputed
// IN: over z = act(bn(x)) (BnIn)
template <bool ACT, bool IN = false>
__global__ void __launch_bounds__(256)
    gn_bwd_stats_kernel(const float* __restrict__ dout, const float* __restrict__ x,
                        const float* __restrict__ mean, const float* __restrict__ rstd,
                        const float* __restrict__ w, const float* __restrict__ bias, int C,
                        int N, int G, float* __restrict__ part, BnIn bn = {}) {
  __shared__ float sh[8];
  const int row = blockIdx.y, p = blockIdx.x;
  const int b = row / C, c = row - b * C, g = c / (C / G);
  const float m = mean[b * G + g], rs = rstd[b * G + g];
  const float ca = ACT ? rs * w[c] : 0.0f, cs = ACT ? bias[c] - m * ca : 0.0f;
  const int N4 = N / 4, chunk = (N4 + kGnParts - 1) / kGnParts;
  const int f0 = min(N4, p * chunk), f1 = min(N4, f0 + chunk);
  const float4* x4 = reinterpret_cast<const float4*>(x) + (size_t)row * N4;
  const float4* d4 = reinterpret_cast<const float4*>(dout) + (size_t)row * N4;
  float a2 = 0.0f, a3 = 0.0f;
  BnInC tc{};
  if (IN) tc = bnin_at(bn, c);
  for (int f = f0 + threadIdx.x; f < f1; f += 256) {
    float4 v = x4[f];
    if (IN) v = make_float4(tc.z(v.x), tc.z(v.y), tc.z(v.z), tc.z(v.w));
    float4 d = d4[f];
    if (ACT) {
      d.x *= gn_dsilu(__builtin_fmaf(v.x, ca, cs));
      d.y *= gn_dsilu(__builtin_fmaf(v.y, ca, cs));
      d.z *= gn_dsilu(__builtin_fmaf(v.z, ca, cs));
      d.w *= gn_dsilu(__builtin_fmaf(v.w, ca, cs));
    }
    a2 += (d.x + d.y) + (d.z + d.w);
    a3 += (d.x * ((v.x - m) * rs) + d.y * ((v.y - m) * rs)) +
          (d.z * ((v.z - m) * rs) + d.w * ((v.w - m) * rs));
  }
  block_sum2(a2, a3, sh);
  if (threadIdx.x == 0) {
    part[((size_t)row * kGnParts + p) * 2] = a2;
    part[((size_t)row * kGnParts + p) * 2 + 1] = a3;
  }
}

// one block, C threads (C <= 1024): per batch element the group coefficients
// k1 = mean_g(dy w), k2 = mean_g(dy w xhat) -> kc[b][c] = (rstd*g1*w, rstd*k1, rstd*k2)
// and d gamma / d beta [b][c]; summed over b: d w, d bias [c].
__global__ void __launch_bounds__(1024)
    gn_bwd_finalize_kernel(const float* __restrict__ part, const float* __restrict__ w,
                           const float* __restrict__ bias, const float* __restrict__ gamma,
                           const float* __restrict__ rstd, int B, int C, int N, int G,
                           float* __restrict__ kc, float* __restrict__ dgamma,
                           float* __restrict__ dbeta, float* __restrict__ dw,
                           float* __restrict__ dbias) {
  __shared__ float s1[1024], s2[1024];
  const int c = threadIdx.x, cpg = C / G;
  float dws = 0.0f, dbs = 0.0f;
  for (int b = 0; b < B; ++b) {
    float a2 = 0.0f, a3 = 0.0f, g1 = 0.0f, t1 = 0.0f, t2 = 0.0f;
    if (c < C) {
      const size_t row = (size_t)b * C + c;
      for (int p = 0; p < kGnParts; ++p) {
        a2 += part[(row * kGnParts + p) * 2];
        a3 += part[(row * kGnParts + p) * 2 + 1];
      }
      g1 = gamma != nullptr ? 1.0f + gamma[row] : 1.0f;
      if (dbeta != nullptr) dbeta[row] = a2;
      if (dgamma != nullptr) dgamma[row] = w[c] * a3 + bias[c] * a2;
      dws += g1 * a3;
      dbs += g1 * a2;
      t1 = w[c] * g1 * a2;  // sum_n dy w over this channel
      t2 = w[c] * g1 * a3;  // sum_n dy w xhat
    }
    s1[c] = t1;
    s2[c] = t2;
    __syncthreads();
    if (c < C) {
      const int g0 = (c / cpg) * cpg;
      float k1 = 0.0f, k2 = 0.0f;
      for (int j = 0; j < cpg; ++j) {
        k1 += s1[g0 + j];
        k2 += s2[g0 + j];
      }
      const float inv_d = (float)(1.0 / ((double)cpg * N));
      const float rs = rstd[b * G + c / cpg];
      const size_t row = (size_t)b * C + c;
      kc[3 * row] = rs * g1 * w[c];
      kc[3 * row + 1] = rs * k1 * inv_d;
      kc[3 * row + 2] = rs * k2 * inv_d;
    }
    __syncthreads();
  }
  if (c < C) {
    dw[c] = dws;
    dbias[c] = dbs;
  }
}

// dx = dout + dout * kc0 - kc1 - xhat * kc2; grid (ceil(N4 / 256), B * C)
// ACT: dx = dy * kc0 - kc1 - xhat * kc2 with dy = dout * SiLU'(x * a + s) (no residual)
// IN (GroupNorm over z = act(bn(x)), the residual z too): dx is dL/dz, and the
// block's BatchNorm backward sums of g = dx * act'(bn(x)) -- sum g and
// sum g * xhat_bn, bn_bwd_stats_kernel's terms -- go to bnpart[c][b * nbx + bx]
// (float2; nbx = gridDim.x): the separate BatchNorm statistics pass over
// (dL/dz, x) is not needed.
template <bool ACT, bool IN = false>
__global__ void __launch_bounds__(256)
    gn_film_bwd_apply_kernel(const float* __restrict__ dout, const float* __restrict__ x,
                             const float* __restrict__ mean, const float* __restrict__ rstd,
                             const float* __restrict__ kc, const float* __restrict__ w,
                             const float* __restrict__ bias, int C, int G, int N4,
                             float* __restrict__ dx, BnIn bn = {},
                             float* __restrict__ bnpart = nullptr) {
  // reverse of the statistics pass's row order (Infinity-cache reuse, as BN)
  const unsigned bx = bn_rev(blockIdx.x, gridDim.x);
  const int n4 = bx * 256 + threadIdx.x;
  if (!IN && n4 >= N4) return;  // IN: every thread reaches the block sum
  const int row = bn_rev(blockIdx.y, gridDim.y);
  const int b = row / C, c = row - b * C, g = c / (C / G);
  const float m = mean[b * G + g], rs = rstd[b * G + g];
  const float k0 = kc[3 * (size_t)row], k1 = kc[3 * (size_t)row + 1], k2 = kc[3 * (size_t)row + 2];
  const size_t i = (size_t)row * N4 + n4;
  float sg = 0.0f, sgx = 0.0f;
  if (n4 < N4) {
    const float4 y = reinterpret_cast<const float4*>(x)[i];
    float4 v = y;
    BnInC tc{};
    if (IN) {
      tc = bnin_at(bn, c);
      v = make_float4(tc.z(y.x), tc.z(y.y), tc.z(y.z), tc.z(y.w));
    }
    const float4 d = reinterpret_cast<const float4*>(dout)[i];
    float4 o;
    if (ACT) {
      const float ca = rs * w[c], cs = bias[c] - m * ca;
      const float dy0 = d.x * gn_dsilu(__builtin_fmaf(v.x, ca, cs));
      const float dy1 = d.y * gn_dsilu(__builtin_fmaf(v.y, ca, cs));
      const float dy2 = d.z * gn_dsilu(__builtin_fmaf(v.z, ca, cs));
      const float dy3 = d.w * gn_dsilu(__builtin_fmaf(v.w, ca, cs));
      o.x = (dy0 * k0 - k1) - ((v.x - m) * rs) * k2;
      o.y = (dy1 * k0 - k1) - ((v.y - m) * rs) * k2;
      o.z = (dy2 * k0 - k1) - ((v.z - m) * rs) * k2;
      o.w = (dy3 * k0 - k1) - ((v.w - m) * rs) * k2;
    } else {
      o.x = d.x + ((d.x * k0 - k1) - ((v.x - m) * rs) * k2);
      o.y = d.y + ((d.y * k0 - k1) - ((v.y - m) * rs) * k2);
      o.z = d.z + ((d.z * k0 - k1) - ((v.z - m) * rs) * k2);
      o.w = d.w + ((d.w * k0 - k1) - ((v.w - m) * rs) * k2);
    }
#ifdef PCFM_GN_NT_STORE
    nt_store4(reinterpret_cast<float4*>(dx) + i, o);
#else
    reinterpret_cast<float4*>(dx)[i] = o;
#endif
    if (IN) {
      const float yv[4] = {y.x, y.y, y.z, y.w}, ov[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float gg = tc.grad(yv[e], ov[e]);
        sg += gg;
        sgx += gg * tc.xh(yv[e]);
      }
    }
  }
  if (IN) {
    __shared__ float sh[8];
    block_sum2(sg, sgx, sh);
    if (threadIdx.x == 0) {
      const int nbx = (int)gridDim.x, P = (int)(gridDim.y / C) * nbx;
      float* pp = bnpart + ((size_t)c * P + (size_t)b * nbx + bx) * 2;
      pp[0] = sg;
      pp[1] = sgx;
    }
  }
}

bool gn_ok(int b, int c, int n, int g) {
  return b > 0 && c > 0 && c <= 1024 && g > 0 && c % g == 0 && n > 0 && n % 4 == 0 &&
         (long long)b * c < 65536 && (long long)(c / g) * n / 4 < (1LL << 31);
}

// group size of a producer's epilogue statistics: P = b * ceil(s / gsz) groups
// per channel, gsz 64 (256-row pointwise tiles) or 32 (128-row streaming form);
// 0 when P matches neither
int parts_gsz(int P, int b, int s) {
  if (P == b * ceil_div(s, 64)) return 64;
  if (P == b * ceil_div(s, 32)) return 32;
  return 0;
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
  const size_t rowpart = (size_t)b * c * bn_bwd_blocks(s);
  return ((size_t)c * bn_parts(b) * 2 + rowpart) * sizeof(float);
}

extern "C" int pcfm_bn_act_fwd(const float* x, const float* gamma, const float* beta, int b, int c,
                               int s, float eps, float slope, float momentum, float* running_mean,
                               float* running_var, long long* num_batches_tracked, float* y,
                               float* mean, float* invstd, void* ws, size_t ws_bytes,
                               void* stream) {
  PCFM_CHECK_ARG(bn_ok(b, c, s), "bn_act_fwd: bad shape b=%d c=%d s=%d (s %% 4 == 0 needed)", b,
                 c, s);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_bn_workspace_bytes(b, c, s), "bn_act_fwd: workspace too small");
  PCFM_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr),
                 "bn_act_fwd: running_mean and running_var must both be given or both NULL");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(c, bn_parts(b)), dim3(256), 0, st, x, b, c, s, part);
  const BnFwdFin fin{part,         b,           s,
                     bn_parts(b),  eps,         momentum,
                     running_mean, running_var, num_batches_tracked};
  hipLaunchKernelGGL(bn_act_apply_kernel, dim3(bn_apply_blocks(s), b * c), dim3(256), 0, st, x,
                     fin, mean, invstd, gamma, beta, c, s / 4, slope, y);
  return check_launch("bn_act_fwd");
}

// pcfm_bn_act_fwd with the statistics from the producer's epilogue (part float2
// [c][P], see bn_fin_parts_kernel): no statistics pass over x.
extern "C" int pcfm_bn_act_fwd_parts(const float* x, const float* part, int P, const float* gamma,
                                     const float* beta, int b, int c, int s, float eps,
                                     float slope, float momentum, float* running_mean,
                                     float* running_var, long long* num_batches_tracked, float* y,
                                     float* mean, float* invstd, void* stream) {
  PCFM_CHECK_ARG(bn_ok(b, c, s), "bn_act_fwd_parts: bad shape b=%d c=%d s=%d", b, c, s);
  const int gsz = parts_gsz(P, b, s);
  PCFM_CHECK_ARG(part != nullptr && gsz > 0,
                 "bn_act_fwd_parts: need b * ceil(s / 64) = %d or b * ceil(s / 32) = %d groups "
                 "per channel, got %d", b * ceil_div(s, 64), b * ceil_div(s, 32), P);
  PCFM_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr),
                 "bn_act_fwd_parts: running_mean and running_var must both be given or both NULL");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_fin_parts_kernel, dim3(c), dim3(256), 0, st,
                     reinterpret_cast<const float2*>(part), P, s, eps, momentum, running_mean,
                     running_var, num_batches_tracked, mean, invstd, gsz);
  const BnFwdFin fin{nullptr, b, s, 0, eps, momentum, running_mean, running_var, nullptr};
  hipLaunchKernelGGL(bn_act_apply_kernel, dim3(bn_apply_blocks(s), b * c), dim3(256), 0, st, x,
                     fin, mean, invstd, gamma, beta, c, s / 4, slope, y);
  return check_launch("bn_act_fwd_parts");
}

extern "C" int pcfm_bn_act_bwd(const float* dz, const float* x, const float* gamma,
                               const float* beta, const float* mean, const float* invstd, int b,
                               int c, int s, float slope, float* dx, float* dgamma, float* dbeta,
                               float* dbias_in, void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(bn_ok(b, c, s), "bn_act_bwd: bad shape b=%d c=%d s=%d (s %% 4 == 0 needed)", b,
                 c, s);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_bn_workspace_bytes(b, c, s), "bn_act_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  hipLaunchKernelGGL(bn_bwd_stats_kernel, dim3(c, bn_parts(b)), dim3(256), 0, st, dz, x, mean,
                     invstd, gamma, beta, b, c, s, slope, part);
  const int nch = bn_bwd_blocks(s);
  float* rowpart = dbias_in != nullptr ? part + (size_t)c * bn_parts(b) * 2 : nullptr;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(nch, b * c), dim3(256), 0, st, dz, x, mean, invstd,
                     gamma, beta, (const float*)part, bn_parts(b), dgamma, dbeta, c, s / 4,
                     (float)(1.0 / ((double)b * s)), slope, dx, rowpart);
  if (dbias_in != nullptr)
    hipLaunchKernelGGL(bn_bias_finalize_kernel, dim3(ceil_div(c, 4)), dim3(256), 0, st,
                       (const float*)rowpart, b, c, nch, dbias_in);
  return check_launch("bn_act_bwd");
}

extern "C" int pcfm_bn_act_fwd_split(const float* x, const float* gamma, const float* beta, int b,
                                     int c, int s, float eps, float slope, float momentum,
                                     float* running_mean, float* running_var,
                                     long long* num_batches_tracked, void* ys, float* mean,
                                     float* invstd, void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(bn_ok(b, c, s) && c % 64 == 0 && s % 64 == 0 && (long long)b < 65536,
                 "bn_act_fwd_split: bad shape b=%d c=%d s=%d (c, s multiples of 64)", b, c, s);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_bn_workspace_bytes(b, c, s), "bn_act_fwd_split: workspace too small");
  PCFM_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr),
                 "bn_act_fwd_split: running_mean and running_var must both be given or both NULL");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(c, bn_parts(b)), dim3(256), 0, st, x, b, c, s, part);
  const BnFwdFin fin{part,         b,           s,
                     bn_parts(b),  eps,         momentum,
                     running_mean, running_var, num_batches_tracked};
  uint16_t* yh = (uint16_t*)ys;
  hipLaunchKernelGGL(bn_act_apply_split_kernel, dim3(s / 64, c / 64, b), dim3(256), 0, st, x,
                     fin, mean, invstd, gamma, beta, c, s, slope, yh,
                     yh + kSplitLo);
  return check_launch("bn_act_fwd_split");
}

// --- PVConv's BN3d + LeakyReLU fused with SE3d and the devoxelization ------
static int se_stat_parts(int b, int c, int s) {  // blocks per (b, c) row of the statistics pass
  const long long rows = (long long)b * c;
  const int by_len = std::max(1, ceil_div(s / 4, 1024));
  const int by_grid = (int)std::max(1LL, (2048 + rows - 1) / rows);
  return std::min(by_len, by_grid);
}

extern "C" size_t pcfm_bn_act_fwd_rowmean_workspace_bytes(int b, int c, int s) {
  if (!bn_ok(b, c, s)) return 0;
  return pcfm_bn_workspace_bytes(b, c, s) + (size_t)b * c * bn_apply_blocks(s) * sizeof(float);
}

extern "C" int pcfm_bn_act_fwd_rowmean(const float* x, const float* gamma, const float* beta,
                                       int b, int c, int s, float eps, float slope,
                                       float momentum, float* running_mean, float* running_var,
                                       long long* num_batches_tracked, float* rowmean,
                                       float* mean, float* invstd, void* ws, size_t ws_bytes,
                                       void* stream) {
  PCFM_CHECK_ARG(bn_ok(b, c, s), "bn_act_fwd_rowmean: bad shape b=%d c=%d s=%d", b, c, s);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_bn_act_fwd_rowmean_workspace_bytes(b, c, s),
                 "bn_act_fwd_rowmean: workspace too small");
  PCFM_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr),
                 "bn_act_fwd_rowmean: running_mean and running_var must both be given or both NULL");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  float* rowpart = part + pcfm_bn_workspace_bytes(b, c, s) / sizeof(float);
  hipLaunchKernelGGL(bn_stats_kernel, dim3(c, bn_parts(b)), dim3(256), 0, st, x, b, c, s, part);
  const BnFwdFin fin{part,         b,           s,
                     bn_parts(b),  eps,         momentum,
                     running_mean, running_var, num_batches_tracked};
  const int nblk = bn_apply_blocks(s);
  hipLaunchKernelGGL(bn_act_rowsum_kernel, dim3(nblk, b * c), dim3(256), 0, st, x, fin, mean,
                     invstd, gamma, beta, c, s / 4, slope, rowpart);
  hipLaunchKernelGGL(rowpart_sum_kernel, dim3(ceil_div(b * c, 256)), dim3(256), 0, st,
                     (const float*)rowpart, b * c, nblk, (float)(1.0 / (double)s), rowmean);
  return check_launch("bn_act_fwd_rowmean");
}

extern "C" int pcfm_bn_fwd_stats(const float* x, const float* part, int P, int b, int c, int s,
                                 float eps, float momentum, float* running_mean,
                                 float* running_var, long long* num_batches_tracked, float* mean,
                                 float* invstd, void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(bn_ok(b, c, s), "bn_fwd_stats: bad shape b=%d c=%d s=%d", b, c, s);
  PCFM_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr),
                 "bn_fwd_stats: running_mean and running_var must both be given or both NULL");
  hipStream_t st = (hipStream_t)stream;
  if (part != nullptr) {  // the producer's epilogue statistics (pcfm_pointwise_gemm_bnstats)
    const int gsz = parts_gsz(P, b, s);
    PCFM_CHECK_ARG(gsz > 0,
                   "bn_fwd_stats: need b * ceil(s / 64) = %d or b * ceil(s / 32) = %d groups "
                   "per channel, got %d", b * ceil_div(s, 64), b * ceil_div(s, 32), P);
    hipLaunchKernelGGL(bn_fin_parts_kernel, dim3(c), dim3(256), 0, st,
                       reinterpret_cast<const float2*>(part), P, s, eps, momentum, running_mean,
                       running_var, num_batches_tracked, mean, invstd, gsz);
  } else {
    PCFM_CHECK_ARG(ws_bytes >= pcfm_bn_workspace_bytes(b, c, s), "bn_fwd_stats: workspace too small");
    float* wp = (float*)ws;
    hipLaunchKernelGGL(bn_stats_kernel, dim3(c, bn_parts(b)), dim3(256), 0, st, x, b, c, s, wp);
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(ceil_div(c, 256)), dim3(256), 0, st,
                       (const float*)wp, x, b, c, s, bn_parts(b), eps, momentum, running_mean,
                       running_var, mean, invstd, num_batches_tracked);
  }
  return check_launch("bn_fwd_stats");
}

extern "C" size_t pcfm_bn_se_bwd_workspace_bytes(int b, int c, int s) {
  if (!bn_ok(b, c, s) || c % 64 != 0 || s % 64 != 0) return 0;
  return ((size_t)b * c * se_stat_parts(b, c, s) * kSeSums + (size_t)b * c * (s / 64)) *
         sizeof(float);
}

extern "C" int pcfm_bn_se_bwd_stats(const float* g, const float* x, const float* mean,
                                    const float* invstd, const float* gamma, const float* beta,
                                    int b, int c, int s, float slope, float* rowstats, void* ws,
                                    size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(bn_ok(b, c, s) && c % 64 == 0 && s % 64 == 0,
                 "bn_se_bwd_stats: bad shape b=%d c=%d s=%d (c, s multiples of 64)", b, c, s);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_bn_se_bwd_workspace_bytes(b, c, s),
                 "bn_se_bwd_stats: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int PS = se_stat_parts(b, c, s);
  float* part = (float*)ws;
  hipLaunchKernelGGL(bn_se_bwd_stats_kernel, dim3(PS, b * c), dim3(256), 0, st, g, x, mean,
                     invstd, gamma, beta, c, s, slope, part);
  hipLaunchKernelGGL(bn_se_rowstats_kernel, dim3(ceil_div(b * c * kSeSums, 256)), dim3(256), 0,
                     st, (const float*)part, b * c, PS, rowstats);
  return check_launch("bn_se_bwd_stats");
}

extern "C" int pcfm_bn_se_bwd_apply_split(const float* g, const float* x, const float* mean,
                                          const float* invstd, const float* gamma,
                                          const float* beta, const float* se_scale,
                                          const float* dmv, const float* rowstats, int b, int c,
                                          int s, float slope, void* dxs, float* dgamma,
                                          float* dbeta, float* dbias_in, void* ws,
                                          size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(bn_ok(b, c, s) && c % 64 == 0 && s % 64 == 0 && (long long)b < 65536,
                 "bn_se_bwd_apply_split: bad shape b=%d c=%d s=%d (c, s multiples of 64)", b, c,
                 s);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_bn_se_bwd_workspace_bytes(b, c, s),
                 "bn_se_bwd_apply_split: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* rowpart = dbias_in != nullptr
                       ? (float*)ws + (size_t)b * c * se_stat_parts(b, c, s) * kSeSums
                       : nullptr;
  uint16_t* dxh = (uint16_t*)dxs;
  hipLaunchKernelGGL(bn_se_bwd_apply_split_kernel, dim3(s / 64, c / 64, b), dim3(256), 0, st, g,
                     x, mean, invstd, gamma, beta, se_scale, dmv, rowstats, b, dgamma, dbeta, c,
                     s, (float)(1.0 / ((double)b * s)), slope, dxh, dxh + kSplitLo, rowpart);
  if (dbias_in != nullptr)
    hipLaunchKernelGGL(bn_bias_finalize_block_kernel, dim3(c), dim3(256), 0, st,
                       (const float*)rowpart, b, c, s / 64, dbias_in);
  return check_launch("bn_se_bwd_apply_split");
}

extern "C" size_t pcfm_bn_act_bwd_split_workspace_bytes(int b, int c, int s) {
  if (!bn_ok(b, c, s) || c % 64 != 0 || s % 64 != 0) return 0;
  return ((size_t)c * bn_parts(b) * 2 + (size_t)b * c * (s / 64)) * sizeof(float);
}

extern "C" int pcfm_bn_act_bwd_split(const float* dz, const float* x, const float* gamma,
                                     const float* beta, const float* mean, const float* invstd,
                                     int b, int c, int s, float slope, void* dxs, float* dgamma,
                                     float* dbeta, float* dbias_in, void* ws, size_t ws_bytes,
                                     void* stream) {
  PCFM_CHECK_ARG(bn_ok(b, c, s) && c % 64 == 0 && s % 64 == 0 && (long long)b < 65536,
                 "bn_act_bwd_split: bad shape b=%d c=%d s=%d (c, s multiples of 64)", b, c, s);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_bn_act_bwd_split_workspace_bytes(b, c, s),
                 "bn_act_bwd_split: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  hipLaunchKernelGGL(bn_bwd_stats_kernel, dim3(c, bn_parts(b)), dim3(256), 0, st, dz, x, mean,
                     invstd, gamma, beta, b, c, s, slope, part);
  float* rowpart = dbias_in != nullptr ? part + (size_t)c * bn_parts(b) * 2 : nullptr;
  uint16_t* dxh = (uint16_t*)dxs;
  hipLaunchKernelGGL(bn_bwd_apply_split_kernel, dim3(s / 64, c / 64, b), dim3(256), 0, st, dz, x,
                     mean, invstd, gamma, beta, (const float*)part, bn_parts(b), dgamma, dbeta, c, s,
                     (float)(1.0 / ((double)b * s)), slope, dxh, dxh + kSplitLo, rowpart);
  if (dbias_in != nullptr)
    hipLaunchKernelGGL(bn_bias_finalize_block_kernel, dim3(c), dim3(256), 0, st,
                       (const float*)rowpart, b, c, s / 64, dbias_in);
  return check_launch("bn_act_bwd_split");
}

extern "C" size_t pcfm_gn_film_workspace_bytes(int b, int c, int n, int groups) {
  if (!gn_ok(b, c, n, groups)) return 0;
  const size_t fwd = ((size_t)b * groups * kGnParts * 2 + 3 * (size_t)b * c) * sizeof(float);
  const size_t bwd = ((size_t)b * c * kGnParts * 2 + 3 * (size_t)b * c) * sizeof(float);
  return fwd > bwd ? fwd : bwd;
}

extern "C" int pcfm_gn_film_res_fwd(const float* x, const float* w, const float* bias,
                                    const float* gamma, const float* beta, int b, int c, int n,
                                    int groups, float eps, float* out, float* mean, float* rstd,
                                    void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(gn_ok(b, c, n, groups), "gn_film_res_fwd: bad shape b=%d c=%d n=%d groups=%d",
                 b, c, n, groups);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_gn_film_workspace_bytes(b, c, n, groups),
                 "gn_film_res_fwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  float* coef = part + (size_t)b * groups * kGnParts * 2;
  hipLaunchKernelGGL(gn_stats_kernel<false>, dim3(groups * kGnParts, b), dim3(256), 0, st, x, c, n,
                     groups, part);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(ceil_div((long long)b * c, 256)), dim3(256), 0, st,
                     (const float*)part, x, w, bias, gamma, b, c, n, groups, eps, mean, rstd,
                     coef);
  hipLaunchKernelGGL(gn_film_apply_kernel<false>, dim3(ceil_div(n / 4, 256), b * c), dim3(256), 0, st,
                     x, (const float*)coef, beta, n / 4, out);
  return check_launch("gn_film_res_fwd");
}

extern "C" int pcfm_gn_film_res_bwd(const float* dout, const float* x, const float* w,
                                    const float* bias, const float* gamma, const float* mean,
                                    const float* rstd, int b, int c, int n, int groups, float* dx,
                                    float* dw, float* dbias, float* dgamma, float* dbeta,
                                    void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(gn_ok(b, c, n, groups), "gn_film_res_bwd: bad shape b=%d c=%d n=%d groups=%d",
                 b, c, n, groups);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_gn_film_workspace_bytes(b, c, n, groups),
                 "gn_film_res_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  float* kc = part + (size_t)b * c * kGnParts * 2;
  hipLaunchKernelGGL(gn_bwd_stats_kernel<false>, dim3(kGnParts, b * c), dim3(256), 0, st, dout, x,
                     mean, rstd, w, bias, c, n, groups, part);
  hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3(1), dim3(1024), 0, st, (const float*)part, w,
                     bias, gamma, rstd, b, c, n, groups, kc, dgamma, dbeta, dw, dbias);
  hipLaunchKernelGGL(gn_film_bwd_apply_kernel<false>, dim3(ceil_div(n / 4, 256), b * c), dim3(256),
                     0, st, dout, x, mean, rstd, (const float*)kc, w, bias, c, groups, n / 4, dx);
  return check_launch("gn_film_res_bwd");
}

// --- the PV block's post SharedMLP activation fused into its GroupNorm-FiLM
// residual (models.py:349-368: out = z + GN(z) (1 + gamma) + beta with
// z = ReLU(BN(y)), y = post's 1x1 conv output): z is never written, and the
// BatchNorm's backward statistics come out of the GroupNorm backward's apply.
static bool bnin_ok(const float* m, const float* is, const float* g, const float* bt) {
  return m != nullptr && is != nullptr && g != nullptr && bt != nullptr;
}

extern "C" int pcfm_gn_film_res_fwd_bnin(const float* y, const float* bn_mean,
                                         const float* bn_invstd, const float* bn_gamma,
                                         const float* bn_beta, float slope, const float* w,
                                         const float* bias, const float* gamma,
                                         const float* beta, int b, int c, int n, int groups,
                                         float eps, float* out, float* mean, float* rstd,
                                         void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(gn_ok(b, c, n, groups), "gn_film_res_fwd_bnin: bad shape b=%d c=%d n=%d groups=%d",
                 b, c, n, groups);
  PCFM_CHECK_ARG(bnin_ok(bn_mean, bn_invstd, bn_gamma, bn_beta),
                 "gn_film_res_fwd_bnin: BatchNorm operands missing");
  PCFM_CHECK_ARG(ws_bytes >= pcfm_gn_film_workspace_bytes(b, c, n, groups),
                 "gn_film_res_fwd_bnin: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const BnIn bn{bn_mean, bn_invstd, bn_gamma, bn_beta, slope};
  float* part = (float*)ws;
  float* coef = part + (size_t)b * groups * kGnParts * 2;
  hipLaunchKernelGGL(gn_stats_kernel<true>, dim3(groups * kGnParts, b), dim3(256), 0, st, y, c, n,
                     groups, part, bn);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(ceil_div((long long)b * c, 256)), dim3(256), 0, st,
                     (const float*)part, y, w, bias, gamma, b, c, n, groups, eps, mean, rstd,
                     coef, bn);
  hipLaunchKernelGGL(gn_film_apply_kernel<true>, dim3(ceil_div(n / 4, 256), b * c), dim3(256), 0,
                     st, y, (const float*)coef, beta, n / 4, out, c, bn);
  return check_launch("gn_film_res_fwd_bnin");
}

extern "C" int pcfm_gn_bnin_parts(int b, int n) {
  if (b <= 0 || n <= 0 || n % 4 != 0) return 0;
  return b * ceil_div(n / 4, 256);
}

extern "C" int pcfm_gn_film_res_bwd_bnin(const float* dout, const float* y, const float* bn_mean,
                                         const float* bn_invstd, const float* bn_gamma,
                                         const float* bn_beta, float slope, const float* w,
                                         const float* bias, const float* gamma, const float* mean,
                                         const float* rstd, int b, int c, int n, int groups,
                                         float* dz, float* dw, float* dbias, float* dgamma,
                                         float* dbeta, float* bnpart, void* ws, size_t ws_bytes,
                                         void* stream) {
  PCFM_CHECK_ARG(gn_ok(b, c, n, groups), "gn_film_res_bwd_bnin: bad shape b=%d c=%d n=%d groups=%d",
                 b, c, n, groups);
  PCFM_CHECK_ARG(bnin_ok(bn_mean, bn_invstd, bn_gamma, bn_beta) && bnpart != nullptr,
                 "gn_film_res_bwd_bnin: BatchNorm operands missing");
  PCFM_CHECK_ARG(ws_bytes >= pcfm_gn_film_workspace_bytes(b, c, n, groups),
                 "gn_film_res_bwd_bnin: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const BnIn bn{bn_mean, bn_invstd, bn_gamma, bn_beta, slope};
  float* part = (float*)ws;
  float* kc = part + (size_t)b * c * kGnParts * 2;
  hipLaunchKernelGGL((gn_bwd_stats_kernel<false, true>), dim3(kGnParts, b * c), dim3(256), 0, st,
                     dout, y, mean, rstd, w, bias, c, n, groups, part, bn);
  hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3(1), dim3(1024), 0, st, (const float*)part, w,
                     bias, gamma, rstd, b, c, n, groups, kc, dgamma, dbeta, dw, dbias);
  hipLaunchKernelGGL((gn_film_bwd_apply_kernel<false, true>), dim3(ceil_div(n / 4, 256), b * c),
                     dim3(256), 0, st, dout, y, mean, rstd, (const float*)kc, w, bias, c, groups,
                     n / 4, dz, bn, bnpart);
  return check_launch("gn_film_res_bwd_bnin");
}

// pcfm_bn_act_bwd's apply pass (+ the producer's bias gradient) on statistics
// a neighbouring kernel produced: part float2 [c][P] of (sum g, sum g xhat).
extern "C" int pcfm_bn_act_bwd_apply_parts(const float* dz, const float* x, const float* gamma,
                                           const float* beta, const float* mean,
                                           const float* invstd, const float* part, int P, int b,
                                           int c, int s, float slope, float* dx, float* dgamma,
                                           float* dbeta, float* dbias_in, void* ws,
                                           size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(bn_ok(b, c, s), "bn_act_bwd_apply_parts: bad shape b=%d c=%d s=%d", b, c, s);
  PCFM_CHECK_ARG(part != nullptr && P > 0, "bn_act_bwd_apply_parts: no statistics");
  const int nch = bn_bwd_blocks(s);
  PCFM_CHECK_ARG(dbias_in == nullptr || ws_bytes >= (size_t)b * c * nch * sizeof(float),
                 "bn_act_bwd_apply_parts: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* rowpart = dbias_in != nullptr ? (float*)ws : nullptr;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(nch, b * c), dim3(256), 0, st, dz, x, mean, invstd,
                     gamma, beta, part, P, dgamma, dbeta, c, s / 4,
                     (float)(1.0 / ((double)b * s)), slope, dx, rowpart);
  if (dbias_in != nullptr)
    hipLaunchKernelGGL(bn_bias_finalize_kernel, dim3(ceil_div(c, 4)), dim3(256), 0, st,
                       (const float*)rowpart, b, c, nch, dbias_in);
  return check_launch("bn_act_bwd_apply_parts");
}

// ContextNet head: SiLU(GroupNorm(x)) (models.py:460-466 head_norm + head_act)
extern "C" int pcfm_gn_silu_fwd(const float* x, const float* w, const float* bias, int b, int c,
                                int n, int groups, float eps, float* out, float* mean, float* rstd,
                                void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(gn_ok(b, c, n, groups), "gn_silu_fwd: bad shape b=%d c=%d n=%d groups=%d", b, c,
                 n, groups);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_gn_film_workspace_bytes(b, c, n, groups),
                 "gn_silu_fwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  float* coef = part + (size_t)b * groups * kGnParts * 2;
  hipLaunchKernelGGL(gn_stats_kernel<false>, dim3(groups * kGnParts, b), dim3(256), 0, st, x, c, n,
                     groups, part);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(ceil_div((long long)b * c, 256)), dim3(256), 0, st,
                     (const float*)part, x, w, bias, nullptr, b, c, n, groups, eps, mean, rstd,
                     coef);
  hipLaunchKernelGGL(gn_silu_apply_kernel, dim3(ceil_div(n / 4, 256), b * c), dim3(256), 0, st, x,
                     (const float*)coef, n / 4, out);
  return check_launch("gn_silu_fwd");
}

extern "C" int pcfm_gn_silu_bwd(const float* dout, const float* x, const float* w,
                                const float* bias, const float* mean, const float* rstd, int b,
                                int c, int n, int groups, float* dx, float* dw, float* dbias,
                                void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(gn_ok(b, c, n, groups), "gn_silu_bwd: bad shape b=%d c=%d n=%d groups=%d", b, c,
                 n, groups);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_gn_film_workspace_bytes(b, c, n, groups),
                 "gn_silu_bwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  float* kc = part + (size_t)b * c * kGnParts * 2;
  hipLaunchKernelGGL(gn_bwd_stats_kernel<true>, dim3(kGnParts, b * c), dim3(256), 0, st, dout, x,
                     mean, rstd, w, bias, c, n, groups, part);
  hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3(1), dim3(1024), 0, st, (const float*)part, w,
                     bias, nullptr, rstd, b, c, n, groups, kc, nullptr, nullptr, dw, dbias);
  hipLaunchKernelGGL(gn_film_bwd_apply_kernel<true>, dim3(ceil_div(n / 4, 256), b * c), dim3(256),
                     0, st, dout, x, mean, rstd, (const float*)kc, w, bias, c, groups, n / 4, dx);
  return check_launch("gn_silu_bwd");
}
