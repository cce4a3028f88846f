// Row gather engine shared by the voxel ops and grouping.
//
// Every PVConv scatter/gather in the reference is, for one (batch, channel),
// a 1-D problem between a "row" of V cells (voxels r^3, or points n) and a list
// of NI items (points, or grouped neighbours) with TAPS (index, weight) pairs
// per item:
//
//   gather : out[b, c, i]  = sum_k w_k(i) * row[b, c, idx_k(i)]       (devox fwd, vox bwd, grouping fwd)
//   scatter: row[b, c, v] += sum_{(i,k): idx_k(i)=v} w_k(i) * in[b, c, i]  (vox fwd, devox bwd, grouping bwd)
//
// The reference launches one block per batch element and walks points with a
// channel loop inside (vox.cu:48-72, trilinear_devox.cu:21-162,
// grouping.cu:18-77): 8 blocks on a 256-CU part, random 4-byte global gathers
// and float atomics into HBM.  Gathers here: one block owns (batch, channel
// group), its row lives in LDS (<= 128 KiB per block), so every random access
// is an LDS read while HBM only sees coalesced streams.  Scatters run on the
// sorted segment engine (segsum.hpp: fixed summation order, no float atomics).
#pragma once

#include <algorithm>
#include <cstdlib>

#include "pcfm_common.hpp"

namespace pcfm {

// ---------------------------------------------------------------------------
// Index providers.  get(b, i, primary, id, w) fills TAPS (index, weight) pairs
// for item i of batch b.  Out-of-range indices come back as (0, 0) so no
// kernel can address outside its row; `primary` is true for exactly one block
// column so providers with side outputs write them once.
// ---------------------------------------------------------------------------

// idx [b, ni] (+ optional weights [b, ni]); rows of length `nrows`.
struct ProvIdx1 {
  static constexpr int TAPS = 1;
  const int* idx;
  const float* w;  // nullptr -> weight 1
  int ni;
  int nrows;
  __device__ __forceinline__ void get(int b, int i, bool, int (&id)[1], float (&wt)[1]) const {
    const size_t o = (size_t)b * ni + i;
    const int v = idx[o];
    const bool ok = (unsigned)v < (unsigned)nrows;
    id[0] = ok ? v : 0;
    wt[0] = ok ? (w ? w[o] : 1.0f) : 0.0f;
  }
};

// inds [b, 8, ni], wgts [b, 8, ni] as saved by the devoxelization forward.
struct ProvIdx8 {
  static constexpr int TAPS = 8;
  const int* inds;
  const float* wgts;
  int ni;
  int nrows;
  __device__ __forceinline__ void get(int b, int i, bool, int (&id)[8], float (&wt)[8]) const {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const size_t o = ((size_t)b * 8 + k) * ni + i;
      const int v = inds[o];
      const bool ok = (unsigned)v < (unsigned)nrows;
      id[k] = ok ? v : 0;
      wt[k] = ok ? wgts[o] : 0.0f;
    }
  }
};

// Trilinear corners straight from float coords [b, 3, n] (values in [0, r-1]),
// exactly as trilinear_devox.cu:37-75 computes them: weights are the products
// dX*dY*dZ in that order, the hi offsets are added only when the fraction is
// non-zero.  Optionally writes inds/wgts [b, 8, n] (training mode).
struct ProvDevox {
  static constexpr int TAPS = 8;
  const float* coords;
  int n, r, r2, r3;
  int* inds_out;    // nullptr in eval mode
  float* wgts_out;  // nullptr in eval mode
  __device__ __forceinline__ void get(int b, int i, bool primary, int (&id)[8],
                                      float (&wt)[8]) const {
    const float* cb = coords + (size_t)b * 3 * n;
    const float x = cb[i], y = cb[i + n], z = cb[i + 2 * n];
    const float xl = floorf(x), yl = floorf(y), zl = floorf(z);
    const float x1 = x - xl, y1 = y - yl, z1 = z - zl;
    const float x0 = 1.0f - x1, y0 = 1.0f - y1, z0 = 1.0f - z1;
    wt[0] = x0 * y0 * z0;
    wt[1] = x0 * y0 * z1;
    wt[2] = x0 * y1 * z0;
    wt[3] = x0 * y1 * z1;
    wt[4] = x1 * y0 * z0;
    wt[5] = x1 * y0 * z1;
    wt[6] = x1 * y1 * z0;
    wt[7] = x1 * y1 * z1;
    const int xh = (x1 > 0.0f) ? r2 : 0;
    const int yh = (y1 > 0.0f) ? r : 0;
    const int zh = (z1 > 0.0f) ? 1 : 0;
    const int base = (int)xl * r2 + (int)yl * r + (int)zl;
    id[0] = base;
    id[1] = base + zh;
    id[2] = base + yh;
    id[3] = base + yh + zh;
    id[4] = base + xh;
    id[5] = base + xh + zh;
    id[6] = base + xh + yh;
    id[7] = base + xh + yh + zh;
    if (primary && inds_out != nullptr) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const size_t o = ((size_t)b * 8 + k) * n + i;
        inds_out[o] = id[k];
        wgts_out[o] = wt[k];
      }
    }
    // A corner whose linear index leaves [0, r^3) (coordinates outside [0, r-1])
    // contributes nothing: (0, 0), as the oracle and the backward's ProvIdx8
    // treat the stored pair, so forward and backward agree on every point.
#ifndef PCFM_DEVOX_CHECK_EACH
    // every corner is inside the volume when the low cell and the high offsets
    // are (the usual case: coords in [0, r-1]); only then are the 8 checks skipped
    const int xi = (int)xl, yi = (int)yl, zi = (int)zl;
    const bool inside = (unsigned)xi < (unsigned)r && (unsigned)yi < (unsigned)r &&
                        (unsigned)zi < (unsigned)r && (unsigned)(xi + (xh != 0)) < (unsigned)r &&
                        (unsigned)(yi + (yh != 0)) < (unsigned)r &&
                        (unsigned)(zi + zh) < (unsigned)r;
    if (!inside)
#endif
    {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const bool ok = (unsigned)id[k] < (unsigned)r3;
        wt[k] = ok ? wt[k] : 0.0f;
        id[k] = ok ? id[k] : 0;
      }
    }
  }
};

// Voxelization backward: one tap, weight (float)(1.0 / (double)cnt[v]) exactly
// as vox.cu:104 (the reference divides in double, then rounds to float).
struct ProvVoxBwd {
  static constexpr int TAPS = 1;
  const int* ind;  // [b, n]
  const int* cnt;  // [b, s]
  int n, s;
  __device__ __forceinline__ void get(int b, int i, bool, int (&id)[1], float (&wt)[1]) const {
    const int v = ind[(size_t)b * n + i];
    const int c = ((unsigned)v < (unsigned)s) ? cnt[(size_t)b * s + v] : 0;
    id[0] = c > 0 ? v : 0;
    wt[0] = c > 0 ? (float)(1.0 / (double)c) : 0.0f;
  }
};

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------

// Sum of TAPS weighted row reads in the reference's contraction order:
// a = w1*f1; a = fma(w0, f0, a); a = fma(wk, fk, a) for k = 2..TAPS-1.
template <int T>
__device__ __forceinline__ float tap_sum(const float* __restrict__ s, const int (&id)[T],
                                         const float (&w)[T]) {
  if constexpr (T == 1) {
    return s[id[0]] * w[0];
  } else {
    float a = w[1] * s[id[1]];
    a = __builtin_fmaf(w[0], s[id[0]], a);
#pragma unroll
    for (int k = 2; k < T; ++k) a = __builtin_fmaf(w[k], s[id[k]], a);
    return a;
  }
}

// Optional epilogue of a gather: out = scale[b, c] * sum + add[b, c, i]
// (either pointer may be null).  Used to fold a squeeze-excitation channel
// scale of the rows and the residual point branch into the devoxelization.
struct RowBn;
struct GatherEpi {
  const float* scale = nullptr;  // [B][C]
  const float* add = nullptr;    // [B][C][NI]
  // optional act(bn(.)) of the add operand (PVConv's point-branch BatchNorm1d +
  // ReLU: SharedMLP's activation is never written); mean == nullptr: plain add
  const float* add_mean = nullptr;
  const float* add_invstd = nullptr;
  const float* add_gamma = nullptr;
  const float* add_beta = nullptr;
  float add_slope = 0.0f;
};

// Optional transform of the rows as they are staged: row value v of channel c
// becomes act(fma((v - mean[c]) * invstd[c], gamma[c], beta[c])) with act(t) =
// t > 0 ? t : slope * t -- PVConv's BatchNorm3d + LeakyReLU applied to the conv
// output while the devoxelization stages it, exactly as bn_act_apply_kernel
// computes it (norm.hip), so the activation is never written.
struct RowBn {
  const float* mean = nullptr;  // nullptr: rows staged as they are
  const float* invstd = nullptr;
  const float* gamma = nullptr;
  const float* beta = nullptr;
  float slope = 0.0f;
};
struct RowBnC {  // one channel's constants
  float m, is, g, bt, slope;
  __device__ __forceinline__ float operator()(float v) const {
    const float t = __builtin_fmaf((v - m) * is, g, bt);
    return t > 0.0f ? t : (slope == 0.0f ? 0.0f : t * slope);
  }
  __device__ __forceinline__ float4 operator()(float4 v) const {
    return make_float4((*this)(v.x), (*this)(v.y), (*this)(v.z), (*this)(v.w));
  }
};
__device__ __forceinline__ RowBnC row_bn_at(const RowBn& bn, int c) {
  return RowBnC{bn.mean[c], bn.invstd[c], bn.gamma[c], bn.beta[c], bn.slope};
}
// the add operand's transform for channel c (identity when epi.add_mean == nullptr)
__device__ __forceinline__ RowBnC add_bn_at(const GatherEpi& epi, int c) {
  if (epi.add_mean == nullptr) return RowBnC{0.0f, 1.0f, 1.0f, 0.0f, 1.0f};
  return RowBnC{epi.add_mean[c], epi.add_invstd[c], epi.add_gamma[c], epi.add_beta[c],
                epi.add_slope};
}

// grid = (item splits, channel groups, b).  USE_LDS stages the block's
// `cpb` rows (cpb * V floats) in LDS first.
template <class Prov, bool USE_LDS>
__global__ void __launch_bounds__(1024)
    gather_rows_kernel(const float* __restrict__ rows, float* __restrict__ out, int C, int V,
                       int NI, int cpb, Prov prov, GatherEpi epi, RowBn bn) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int T = Prov::TAPS;
  const int b = blockIdx.z;
  const int c0 = blockIdx.y * cpb;
  const int nc = min(cpb, C - c0);
  const float* __restrict__ rb = rows + ((size_t)b * C + c0) * V;
  if constexpr (USE_LDS) {
    const int total = nc * V;
    if (bn.mean != nullptr) {  // block-uniform
      for (int e = threadIdx.x; e < total; e += blockDim.x)
        lds[e] = row_bn_at(bn, c0 + e / V)(rb[e]);
    } else if ((((uintptr_t)rb) & 15) == 0 && (total & 3) == 0) {
      const float4* __restrict__ s4 = reinterpret_cast<const float4*>(rb);
      float4* d4 = reinterpret_cast<float4*>(lds);
      for (int e = threadIdx.x; e < (total >> 2); e += blockDim.x) d4[e] = s4[e];
    } else {
      for (int e = threadIdx.x; e < total; e += blockDim.x) lds[e] = rb[e];
    }
    __syncthreads();
  }
  float* __restrict__ ob = out + ((size_t)b * C + c0) * NI;
  const bool primary = blockIdx.y == 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < NI; i += gridDim.x * blockDim.x) {
    int id[T];
    float w[T];
    if (epi.scale == nullptr && epi.add == nullptr) {
      prov.get(b, i, primary, id, w);
      for (int cc = 0; cc < nc; ++cc) {
        float acc;
        if constexpr (USE_LDS) {
          acc = tap_sum<T>(lds + (size_t)cc * V, id, w);
        } else {
          acc = tap_sum<T>(rb + (size_t)cc * V, id, w);
        }
        ob[(size_t)cc * NI + i] = acc;
      }
    } else {
      // epilogue operands of 4 channels at a time, the first 4 fetched before
      // the taps so their latency overlaps the index computation (the plain
      // per-channel form: devox forward 0.71 -> 1.14 ms/step, vox backward
      // 0.55 -> 0.88 ms/step, profiles/r03_bench_step_breakdown.txt notes)
      const float* __restrict__ ab =
          epi.add != nullptr ? epi.add + ((size_t)b * C + c0) * NI + i : nullptr;
      const float* __restrict__ sb = epi.scale != nullptr ? epi.scale + (size_t)b * C + c0 : nullptr;
      float ad[4], sc[4];
      const bool abn = epi.add_mean != nullptr;  // block-uniform
      auto fetch = [&](int cq) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int cc = min(cq + k, nc - 1);
          ad[k] = ab != nullptr ? nt_ld(ab + (size_t)cc * NI) : 0.0f;
          if (abn) ad[k] = add_bn_at(epi, c0 + cc)(ad[k]);
          sc[k] = sb != nullptr ? sb[cc] : 1.0f;
        }
      };
      fetch(0);
      prov.get(b, i, primary, id, w);
      for (int cq = 0; cq < nc; cq += 4) {
        if (cq > 0) fetch(cq);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int cc = cq + k;
          if (cc < nc) {
            float acc;
            if constexpr (USE_LDS) {
              acc = tap_sum<T>(lds + (size_t)cc * V, id, w);
            } else {
              acc = tap_sum<T>(rb + (size_t)cc * V, id, w);
            }
            if (sb != nullptr) acc *= sc[k];
            if (ab != nullptr) acc += ad[k];
            ob[(size_t)cc * NI + i] = acc;
          }
        }
      }
    }
  }
}

// The one-channel form (cpb == 1: the r = 32 rows of 32768 voxels, 128 KiB, one
// 1024-thread block per CU): IPT items per thread per round, every item's
// loads (coordinates / indices, the epilogue's add) issued before any of them
// is used -- the plain loop had one item's load chain in flight per thread
// (its store may alias the next item's loads as far as the compiler knows),
// which held the gather to ~2 TB/s.  Same expressions: bit-identical.
template <class Prov, int IPT>
__global__ void __launch_bounds__(1024)
    gather_rows1_kernel(const float* __restrict__ rows, float* __restrict__ out, int C, int V,
                        int NI, Prov prov, GatherEpi epi, RowBn bn) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int T = Prov::TAPS;
  const int b = blockIdx.z;
  const int c0 = blockIdx.y;
  const float* __restrict__ rb = rows + ((size_t)b * C + c0) * V;
  if ((((uintptr_t)rb) & 15) == 0 && (V & 3) == 0) {
    const float4* __restrict__ s4 = reinterpret_cast<const float4*>(rb);
    float4* d4 = reinterpret_cast<float4*>(lds);
    if (bn.mean != nullptr) {  // block-uniform
      const RowBnC f = row_bn_at(bn, c0);
      for (int e = threadIdx.x; e < (V >> 2); e += blockDim.x) d4[e] = f(s4[e]);
    } else {
      for (int e = threadIdx.x; e < (V >> 2); e += blockDim.x) d4[e] = s4[e];
    }
  } else if (bn.mean != nullptr) {
    const RowBnC f = row_bn_at(bn, c0);
    for (int e = threadIdx.x; e < V; e += blockDim.x) lds[e] = f(rb[e]);
  } else {
    for (int e = threadIdx.x; e < V; e += blockDim.x) lds[e] = rb[e];
  }
  __syncthreads();
  float* __restrict__ ob = out + ((size_t)b * C + c0) * NI;
  const float* __restrict__ ab = epi.add != nullptr ? epi.add + ((size_t)b * C + c0) * NI : nullptr;
  const float sc = epi.scale != nullptr ? epi.scale[(size_t)b * C + c0] : 1.0f;
  const bool abn = epi.add_mean != nullptr;  // block-uniform
  const RowBnC fa = add_bn_at(epi, c0);
  const bool primary = blockIdx.y == 0;
  const int stride = gridDim.x * blockDim.x;
  for (int i0 = blockIdx.x * blockDim.x + threadIdx.x; i0 < NI; i0 += IPT * stride) {
    int id[IPT][T];
    float w[IPT][T], ad[IPT];
#pragma unroll
    for (int u = 0; u < IPT; ++u) {
      const int i = i0 + u * stride;
      const bool ok = i < NI;
      const int iu = ok ? i : i0;
      ad[u] = ab != nullptr ? nt_ld(ab + iu) : 0.0f;
      prov.get(b, iu, primary && ok, id[u], w[u]);
    }
#pragma unroll
    for (int u = 0; u < IPT; ++u) {
      const int i = i0 + u * stride;
      if (i < NI) {
        float acc = tap_sum<T>(lds, id[u], w[u]);
        if (epi.scale != nullptr) acc *= sc;
        if (ab != nullptr) acc += abn ? fa(ad[u]) : ad[u];
        ob[i] = acc;
      }
    }
  }
}

// The 4-channel form of gather_rows_kernel (cpb == 4, the r = 16 / 8 devox
// forward and voxelization backward): the four rows are staged interleaved,
// lds4[v] = (row c0 .. c0+3 at v), so a tap of an item reads its four channels
// with one ds_read_b128 instead of four ds_read_b32 (the random corner reads
// are what the gather waits on: LDS bank conflicts were 0.7 of its LDS cycles).
// Per channel the same products and fma order: bit-identical.
template <int T>
__device__ __forceinline__ float4 tap_sum4(const float4* __restrict__ s, const int (&id)[T],
                                           const float (&w)[T]) {
  if constexpr (T == 1) {
    const float4 v = s[id[0]];
    return make_float4(v.x * w[0], v.y * w[0], v.z * w[0], v.w * w[0]);
  } else {
    const float4 v1 = s[id[1]], v0 = s[id[0]];
    float4 a = make_float4(w[1] * v1.x, w[1] * v1.y, w[1] * v1.z, w[1] * v1.w);
    a.x = __builtin_fmaf(w[0], v0.x, a.x);
    a.y = __builtin_fmaf(w[0], v0.y, a.y);
    a.z = __builtin_fmaf(w[0], v0.z, a.z);
    a.w = __builtin_fmaf(w[0], v0.w, a.w);
#pragma unroll
    for (int k = 2; k < T; ++k) {
      const float4 v = s[id[k]];
      a.x = __builtin_fmaf(w[k], v.x, a.x);
      a.y = __builtin_fmaf(w[k], v.y, a.y);
      a.z = __builtin_fmaf(w[k], v.z, a.z);
      a.w = __builtin_fmaf(w[k], v.w, a.w);
    }
    return a;
  }
}

// grid = (item splits, C / 4, b); C % 4 == 0.
template <class Prov>
__global__ void __launch_bounds__(512)
    gather_rows4_kernel(const float* __restrict__ rows, float* __restrict__ out, int C, int V,
                        int NI, Prov prov, GatherEpi epi, RowBn bn) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float4* lds4 = reinterpret_cast<float4*>(lds);
  constexpr int T = Prov::TAPS;
  const int b = blockIdx.z;
  const int c0 = blockIdx.y * 4;
  const float* __restrict__ rb = rows + ((size_t)b * C + c0) * V;
  if (bn.mean != nullptr) {  // block-uniform
    const RowBnC f0 = row_bn_at(bn, c0), f1 = row_bn_at(bn, c0 + 1), f2 = row_bn_at(bn, c0 + 2),
                 f3 = row_bn_at(bn, c0 + 3);
    for (int v = threadIdx.x; v < V; v += blockDim.x)
      lds4[v] = make_float4(f0(rb[v]), f1(rb[(size_t)V + v]), f2(rb[2 * (size_t)V + v]),
                            f3(rb[3 * (size_t)V + v]));
  } else {
    for (int v = threadIdx.x; v < V; v += blockDim.x)
      lds4[v] =
          make_float4(rb[v], rb[(size_t)V + v], rb[2 * (size_t)V + v], rb[3 * (size_t)V + v]);
  }
  __syncthreads();
  float* __restrict__ ob = out + ((size_t)b * C + c0) * NI;
  const float* __restrict__ ab = epi.add != nullptr ? epi.add + ((size_t)b * C + c0) * NI : nullptr;
  float sc[4] = {1.0f, 1.0f, 1.0f, 1.0f};
  if (epi.scale != nullptr) {
#pragma unroll
    for (int k = 0; k < 4; ++k) sc[k] = epi.scale[(size_t)b * C + c0 + k];
  }
  const bool abn = epi.add_mean != nullptr;  // block-uniform
  const RowBnC fa[4] = {add_bn_at(epi, c0), add_bn_at(epi, c0 + 1), add_bn_at(epi, c0 + 2),
                        add_bn_at(epi, c0 + 3)};
  const bool primary = blockIdx.y == 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < NI; i += gridDim.x * blockDim.x) {
    float ad[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (ab != nullptr) {  // issued before the taps: their latency overlaps the index math
#pragma unroll
      for (int k = 0; k < 4; ++k) ad[k] = nt_ld(ab + (size_t)k * NI + i);
    }
    int id[T];
    float w[T];
    prov.get(b, i, primary, id, w);
    const float4 a = tap_sum4<T>(lds4, id, w);
    const float r[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float acc = r[k];
      if (epi.scale != nullptr) acc *= sc[k];
      if (ab != nullptr) acc += abn ? fa[k](ad[k]) : ad[k];
      ob[(size_t)k * NI + i] = acc;
    }
  }
}

// ---------------------------------------------------------------------------
// Launch planning
// ---------------------------------------------------------------------------

struct RowPlan {
  int threads = 512;
  int cpb = 1;       // channels per block
  int groups = 1;    // ceil(C / cpb), at least 1
  int psplit = 1;    // item splits (grid.x multiplier)
  bool use_lds = true;
  size_t lds_bytes = 0;
};

constexpr int kLdsFloatsSmall = 16 * 1024;  // 64 KiB: 2 blocks of 512 threads per CU
constexpr int kLdsFloatsBig = 32 * 1024;    // 128 KiB: 1 block of 1024 threads per CU

inline long long gather_target_blocks() {
  static const long long t = [] {
    const char* e = std::getenv("PCFM_GATHER_BLOCKS");  // dev knob (measurement)
    // 2 per CU: more channels per block amortise the per-item index work
    // (measured 0.6-0.8x the time of 4 per CU at r = 16 and 8, equal at r = 32)
    return e != nullptr ? std::max(1LL, std::atoll(e)) : 512LL;
  }();
  return t;
}

// PCFM_GATHER4=0: the per-channel form for cpb == 4 too (A/B knob)
inline bool gather4_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("PCFM_GATHER4");
    return !(e != nullptr && e[0] == '0');
  }();
  return on;
}

// items per thread per round of the one-channel gather (PCFM_GATHER1_IPT: 1 =
// the generic loop; A/B knob)
inline int gather1_ipt() {
  static const int v = [] {
    const char* e = std::getenv("PCFM_GATHER1_IPT");
    return e != nullptr ? std::max(1, std::atoi(e)) : 2;
  }();
  return v;
}

inline RowPlan plan_gather(int B, int C, int V, int NI) {
  RowPlan p;
  const long long target = gather_target_blocks();
  if ((long long)V <= kLdsFloatsSmall) {
    p.threads = 512;
    p.cpb = std::max(1, std::min(C, kLdsFloatsSmall / std::max(V, 1)));
  } else if ((long long)V <= kLdsFloatsBig) {
    p.threads = 1024;
    p.cpb = 1;
  } else {
    p.use_lds = false;
    p.threads = 256;
    p.cpb = std::max(1, std::min(C, 4));
  }
  auto groups = [&](int cpb) { return std::max(1, ceil_div(C, cpb)); };
  while (p.cpb > 1 && (long long)groups(p.cpb) * B < target) p.cpb = (p.cpb + 1) / 2;
  p.groups = groups(p.cpb);
  const long long blocks = (long long)p.groups * B;
  if (blocks < target) {
    const int want = ceil_div(target, blocks);
    const int cap = std::max(1, ceil_div(NI, p.threads));
    p.psplit = std::min(want, cap);
  }
  p.lds_bytes = p.use_lds ? (size_t)p.cpb * V * sizeof(float) : 0;
  return p;
}

template <class Prov>
inline bool prov_has_side_outputs(const Prov&) { return false; }
inline bool prov_has_side_outputs(const ProvDevox& p) { return p.inds_out != nullptr; }

template <class Prov>
inline int launch_gather(const float* rows, float* out, int B, int C, int V, int NI, Prov prov,
                         hipStream_t st, const char* what, GatherEpi epi = GatherEpi{},
                         RowBn bn = RowBn{}) {
  if (B == 0 || NI == 0) return PCFM_OK;
  if (V == 0 && C > 0 && epi.add == nullptr) {  // empty rows: every tap is out of range -> zeros
    hipError_t e = hipMemsetAsync(out, 0, (size_t)B * C * NI * sizeof(float), st);
    if (e != hipSuccess) {
      set_error("%s: hipMemsetAsync: %s", what, hipGetErrorString(e));
      return (int)e;
    }
    if (!prov_has_side_outputs(prov)) return PCFM_OK;
  }
  RowPlan p = plan_gather(B, C, V, NI);
  dim3 grid(p.psplit, p.groups, B);
  if (p.use_lds && p.cpb == 4 && C % 4 == 0 && p.threads == 512 && gather4_enabled()) {
    int e = allow_big_lds((const void*)gather_rows4_kernel<Prov>);
    if (e) return e;
    hipLaunchKernelGGL((gather_rows4_kernel<Prov>), grid, dim3(512), p.lds_bytes, st, rows, out, C,
                       V, NI, prov, epi, bn);
  } else if (p.use_lds && p.cpb == 1 && p.threads == 1024 && gather1_ipt() > 1) {
    int e = allow_big_lds((const void*)gather_rows1_kernel<Prov, 2>);
    if (e) return e;
    e = allow_big_lds((const void*)gather_rows1_kernel<Prov, 4>);
    if (e) return e;
    if (gather1_ipt() >= 4)
      hipLaunchKernelGGL((gather_rows1_kernel<Prov, 4>), grid, dim3(1024), p.lds_bytes, st, rows,
                         out, C, V, NI, prov, epi, bn);
    else
      hipLaunchKernelGGL((gather_rows1_kernel<Prov, 2>), grid, dim3(1024), p.lds_bytes, st, rows,
                         out, C, V, NI, prov, epi, bn);
  } else if (p.use_lds) {
    int e = allow_big_lds((const void*)gather_rows_kernel<Prov, true>);
    if (e) return e;
    hipLaunchKernelGGL((gather_rows_kernel<Prov, true>), grid, dim3(p.threads), p.lds_bytes, st,
                       rows, out, C, V, NI, p.cpb, prov, epi, bn);
  } else {
    if (bn.mean != nullptr) {  // the row transform needs the staged rows
      set_error("%s: a row transform needs rows that fit LDS (V = %d)", what, V);
      return PCFM_EINVAL;
    }
    hipLaunchKernelGGL((gather_rows_kernel<Prov, false>), grid, dim3(p.threads), 0, st, rows,
                       out, C, V, NI, p.cpb, prov, epi, bn);
  }
  return check_launch(what);
}

}  // namespace pcfm
