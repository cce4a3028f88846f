// Approximate EMD: approxmatch, matchcost and its gradient (include/pcfm.h).
//
// Reference: third_party/PyTorchEMD/cuda/emd_kernel.cu.  The reference runs
// the whole 10-level x 3-pass auction inside one block per batch element
// (<<<32,512>>>, emd_kernel.cu:186) and read-modify-writes the dense
// match[b, m, n] matrix once per level (:144).
//
// MI355X design:
//   * every pass of every level is a full-chip launch with its finalize
//     included: a block owns 64 rows (lanes), its 16 waves split the column
//     range (wave-uniform, so the column points arrive through scalar loads),
//     the wave sums of a row are added in a fixed order in LDS and the row's
//     finalize runs in the same block; a level's third pass and the next
//     level's first share one launch (21 launches per approxmatch);
//   * match is NOT accumulated level by level.  Each level only needs the
//     vectors ratioL (n) and ratioR (m), which are kept per level (10 x (n+m));
//     match is written once at the end as
//         match[l, k] = sum_j (exp(level_j * d2) * ratioL_j[k]) * ratioR_j[l]
//     summed in the reference's level order -- the same per-entry expression
//     and order as the reference's `match += w` (:143-144), with 1/10th of the
//     HBM traffic.
//   * exp is the hardware exp2 on x*log2(e): the reference is built with
//     --use_fast_math (__expf, backend.py:20), so EMD parity is tolerance-based.
#include "pcfm_common.hpp"

#include <algorithm>
#include <cstdlib>

namespace pcfm {
namespace {

constexpr int kLevels = 10;
// level_j = -4^j for j = 7 .. -1, then 0 (emd_kernel.cu:44-48).
__constant__ float c_levels[kLevels] = {-16384.0f, -4096.0f, -1024.0f, -256.0f, -64.0f,
                                        -16.0f,    -4.0f,    -1.0f,    -0.25f,  0.0f};
constexpr float h_levels[kLevels] = {-16384.0f, -4096.0f, -1024.0f, -256.0f, -64.0f,
                                     -16.0f,    -4.0f,    -1.0f,    -0.25f,  0.0f};

__device__ __forceinline__ float fast_expf(float x) {
  return __builtin_amdgcn_exp2f(x * 1.4426950408889634f);
}
template <typename T>
__device__ __forceinline__ T emd_exp(T x) {
  return (T)fast_expf((float)x);
}

template <typename T>
__device__ __forceinline__ T fmaT(T a, T b, T c);
template <>
__device__ __forceinline__ float fmaT<float>(float a, float b, float c) {
  return __builtin_fmaf(a, b, c);
}
template <>
__device__ __forceinline__ double fmaT<double>(double a, double b, double c) {
  return __builtin_fma(a, b, c);
}

constexpr int kThreads = 256;

// MODE 0: acc += e * coef[c]            (pass 1: coef = remainR, :70-76)
// MODE 1: acc += e * coef[c]            (pass 2: coef = ratioL,  :102-107)
// MODE 2: acc += (e * rowscale[i]) * coef[c]  (pass 3: ratioL[k] * ratioR[l], :139-146)
// grid = (row blocks, S, b); part[s][b*nr + i].
template <typename T, int MODE>
__global__ void __launch_bounds__(kThreads)
    emd_pass_kernel(const T* __restrict__ rows, int nr, const T* __restrict__ cols, int ncol,
                    int b, T level, const T* __restrict__ coef, const T* __restrict__ rowscale,
                    int S, T* __restrict__ part) {
  const int bb = blockIdx.z;
  const int s = blockIdx.y;
  const int i = blockIdx.x * kThreads + threadIdx.x;
  const int ii = i < nr ? i : nr - 1;
  const T* rp = rows + ((size_t)bb * nr + ii) * 3;
  const T x1 = rp[0], y1 = rp[1], z1 = rp[2];
  T rl = (T)0;
  if constexpr (MODE == 2) rl = rowscale[(size_t)bb * nr + ii];
  const int c0 = (int)(((long long)ncol * s) / S);
  const int c1 = (int)(((long long)ncol * (s + 1)) / S);
  const T* __restrict__ cb = cols + (size_t)bb * ncol * 3;
  const T* __restrict__ kb = coef + (size_t)bb * ncol;
  T acc = 0;
#pragma unroll 4
  for (int c = c0; c < c1; ++c) {
    const T d2 = sqdist3(cb[3 * c] - x1, cb[3 * c + 1] - y1, cb[3 * c + 2] - z1);
    const T e = emd_exp<T>(level * d2);
    if constexpr (MODE == 2) {
      acc = fmaT<T>(e * rl, kb[c], acc);
    } else {
      acc = fmaT<T>(e, kb[c], acc);
    }
  }
  if (i < nr) part[(size_t)s * b * nr + (size_t)bb * nr + i] = acc;
}

template <typename T>
__device__ __forceinline__ T sum_parts(const T* part, int S, size_t stride, size_t i) {
  T v = 0;
  for (int s = 0; s < S; ++s) v += part[(size_t)s * stride + i];
  return v;
}

template <typename T>
__global__ void emd_init_kernel(T* remL, size_t nl, T multiL, T* remR, size_t nr, T multiR) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nl) remL[i] = multiL;
  if (i < nr) remR[i] = multiR;
}

// ratioL = remainL / (1e-9 + suml)    (:57, :81)
template <typename T>
__global__ void emd_fin1_kernel(const T* __restrict__ part, int S, size_t total,
                                const T* __restrict__ remL, T* __restrict__ ratL) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  ratL[i] = remL[i] / ((T)1e-9f + sum_parts(part, S, total, i));
}

// sumr *= remainR; consumption = min(remainR / (sumr + 1e-9), 1);
// ratioR = consumption * remainR; remainR = max(0, remainR - sumr)   (:111-116)
// fminf/fmaxf take float arguments in the reference for both dtypes.
template <typename T>
__global__ void emd_fin2_kernel(const T* __restrict__ part, int S, size_t total,
                                T* __restrict__ remR, T* __restrict__ ratR,
                                T* __restrict__ levR) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const T r = remR[i];
  T sumr = sum_parts(part, S, total, i);
  sumr *= r;
  const T cons = (T)fminf((float)(r / (sumr + (T)1e-9f)), 1.0f);
  const T rat = cons * r;
  ratR[i] = rat;
  levR[i] = rat;
  remR[i] = (T)fmaxf(0.0f, (float)(r - sumr));
}

// remainL = max(0, remainL - suml); keep this level's ratioL   (:150-151)
template <typename T>
__global__ void emd_fin3_kernel(const T* __restrict__ part, int S, size_t total,
                                T* __restrict__ remL, const T* __restrict__ ratL,
                                T* __restrict__ levL) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  remL[i] = (T)fmaxf(0.0f, (float)(remL[i] - sum_parts(part, S, total, i)));
  levL[i] = ratL[i];
}

// match[b, l, k] = sum_j (exp(level_j * d2(k,l)) * ratioL_j[k]) * ratioR_j[l].
// grid = (k blocks, l blocks of kLPer, b); lanes over k -> coalesced rows.
constexpr int kLPer = 8;
template <typename T>
__global__ void __launch_bounds__(kThreads)
    emd_match_kernel(const T* __restrict__ xyz1, const T* __restrict__ xyz2, int b, int n, int m,
                     const T* __restrict__ levL, const T* __restrict__ levR,
                     T* __restrict__ match) {
  const int bb = blockIdx.z;
  const int k = blockIdx.x * kThreads + threadIdx.x;
  if (blockIdx.x * kThreads >= n) return;
  const int kk = k < n ? k : n - 1;
  const T* p1 = xyz1 + ((size_t)bb * n + kk) * 3;
  const T x1 = p1[0], y1 = p1[1], z1 = p1[2];
  T rl[kLevels];
#pragma unroll
  for (int j = 0; j < kLevels; ++j) rl[j] = levL[(size_t)j * b * n + (size_t)bb * n + kk];
  const int l0 = blockIdx.y * kLPer;
  const int l1 = min(m, l0 + kLPer);
  for (int l = l0; l < l1; ++l) {
    const T* p2 = xyz2 + ((size_t)bb * m + l) * 3;
    const T d2 = sqdist3(p2[0] - x1, p2[1] - y1, p2[2] - z1);
    T acc = 0;
#pragma unroll
    for (int j = 0; j < kLevels; ++j) {
      const T rr = levR[(size_t)j * b * m + (size_t)bb * m + l];
      const T e = emd_exp<T>((T)c_levels[j] * d2);
      acc += (e * rl[j]) * rr;
    }
    if (k < n) match[((size_t)bb * m + l) * n + k] = acc;
  }
}

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  T t = 0;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;  // valid in thread 0
}

// cost partials: grid = (k blocks, S, b); part[(bb*S + s)*kblocks + kb].
template <typename T>
__global__ void __launch_bounds__(kThreads)
    emd_cost_kernel(const T* __restrict__ xyz1, const T* __restrict__ xyz2,
                    const T* __restrict__ match, int b, int n, int m, int S,
                    T* __restrict__ part) {
  __shared__ T red[kThreads / 64];
  const int bb = blockIdx.z, s = blockIdx.y;
  const int k = blockIdx.x * kThreads + threadIdx.x;
  const int kk = k < n ? k : n - 1;
  const T* p1 = xyz1 + ((size_t)bb * n + kk) * 3;
  const T x1 = p1[0], y1 = p1[1], z1 = p1[2];
  const int l0 = (int)(((long long)m * s) / S), l1 = (int)(((long long)m * (s + 1)) / S);
  const T* __restrict__ cb = xyz2 + (size_t)bb * m * 3;
  T sub = 0;
  if (k < n) {
    for (int l = l0; l < l1; ++l) {
      const T d = sqdist3(cb[3 * l] - x1, cb[3 * l + 1] - y1, cb[3 * l + 2] - z1);
      sub = fmaT<T>(d, match[((size_t)bb * m + l) * n + k], sub);
    }
  }
  const T t = block_sum(sub, red);
  if (threadIdx.x == 0) part[((size_t)bb * S + s) * gridDim.x + blockIdx.x] = t;
}

// cost[bb] = sum of the batch element's per_b block partials: one wave per
// batch element, lanes over strided partials, then a fixed xor tree
// (deterministic; the serial form was 9 us at 512 partials).
template <typename T>
__global__ void __launch_bounds__(64)
    emd_cost_fin_kernel(const T* __restrict__ part, int per_b, T* __restrict__ cost) {
  const int bb = blockIdx.x, lane = threadIdx.x;
  T t = 0;
  for (int i = lane; i < per_b; i += 64) t += part[(size_t)bb * per_b + i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
  if (lane == 0) cost[bb] = t;
}

// The match write with matchcost fused (the fused forward, pcfm_emd_approxmatch_cost_*):
// match[b, l, k] as emd_match_kernel (skipped when match == nullptr), and per
// block the partial sum over its entries of d2 * match -- matchcost's terms
// (emd_kernel.cu:199-241) -- to part[(bb * lblocks + lb) * kblocks + kb], so
// the 4-byte-per-entry match matrix is not read back for the cost.  A block
// = 256 k (lanes, coalesced rows) x kMatchL l, the l points and their 10
// ratioR values staged in LDS.
constexpr int kMatchL = 32;
template <typename T>
__global__ void __launch_bounds__(kThreads)
    emd_match_cost_kernel(const T* __restrict__ xyz1, const T* __restrict__ xyz2, int b, int n,
                          int m, const T* __restrict__ levL, const T* __restrict__ levR,
                          T* __restrict__ match, T* __restrict__ part) {
  constexpr int kW = kLevels + 3;  // per l: ratioR_0..9, x, y, z
  __shared__ T sl[kMatchL * kW];
  __shared__ T red[kThreads / 64];
  const int bb = blockIdx.z, kb = blockIdx.x, lb = blockIdx.y;
  const int k = kb * kThreads + threadIdx.x;
  const int kk = k < n ? k : n - 1;
  const int l0 = lb * kMatchL, nl = min(kMatchL, m - l0);
  for (int e = threadIdx.x; e < nl * kW; e += kThreads) {
    const int li = e / kW, q = e - li * kW;
    sl[e] = q < kLevels ? levR[(size_t)q * b * m + (size_t)bb * m + l0 + li]
                        : xyz2[((size_t)bb * m + l0 + li) * 3 + (q - kLevels)];
  }
  const T* p1 = xyz1 + ((size_t)bb * n + kk) * 3;
  const T x1 = p1[0], y1 = p1[1], z1 = p1[2];
  T rl[kLevels];
#pragma unroll
  for (int j = 0; j < kLevels; ++j) rl[j] = levL[(size_t)j * b * n + (size_t)bb * n + kk];
  __syncthreads();
  T csum = 0;
  T* mrow = match != nullptr ? match + ((size_t)bb * m + l0) * n + k : nullptr;
  for (int li = 0; li < nl; ++li) {
    const T* q = sl + li * kW;
    const T d2 = sqdist3(q[kLevels] - x1, q[kLevels + 1] - y1, q[kLevels + 2] - z1);
    T acc = 0;
#pragma unroll
    for (int j = 0; j < kLevels; ++j) {
      // level_j * log2(e) in one float factor (exact: level_j is a power of two)
      const T e = j == kLevels - 1 ? (T)1
                                   : (T)__builtin_amdgcn_exp2f((float)d2 *
                                                               (h_levels[j] * 1.4426950408889634f));
      acc += (e * rl[j]) * q[j];
    }
    if (mrow != nullptr && k < n) mrow[(size_t)li * n] = acc;
    csum = fmaT<T>(d2, acc, csum);
  }
  const T t = block_sum(k < n ? csum : (T)0, red);
  if (threadIdx.x == 0) part[((size_t)bb * gridDim.y + lb) * gridDim.x + kb] = t;
}

// grad1 partials: lanes over k, l split S ways: part[s][(bb*n + k)*3 + x].
template <typename T>
__global__ void __launch_bounds__(kThreads)
    emd_grad1_kernel(const T* __restrict__ xyz1, const T* __restrict__ xyz2,
                     const T* __restrict__ match, int b, int n, int m, int S,
                     T* __restrict__ part) {
  const int bb = blockIdx.z, s = blockIdx.y;
  const int k = blockIdx.x * kThreads + threadIdx.x;
  if (k >= n) return;
  const T* p1 = xyz1 + ((size_t)bb * n + k) * 3;
  const T x1 = p1[0], y1 = p1[1], z1 = p1[2];
  const int l0 = (int)(((long long)m * s) / S), l1 = (int)(((long long)m * (s + 1)) / S);
  const T* __restrict__ cb = xyz2 + (size_t)bb * m * 3;
  T dx = 0, dy = 0, dz = 0;
  for (int l = l0; l < l1; ++l) {
    const T d = match[((size_t)bb * m + l) * n + k] * (T)2;
    dx = fmaT<T>(x1 - cb[3 * l], d, dx);
    dy = fmaT<T>(y1 - cb[3 * l + 1], d, dy);
    dz = fmaT<T>(z1 - cb[3 * l + 2], d, dz);
  }
  T* o = part + (size_t)s * b * n * 3 + ((size_t)bb * n + k) * 3;
  o[0] = dx;
  o[1] = dy;
  o[2] = dz;
}

template <typename T>
__global__ void emd_grad1_fin_kernel(const T* __restrict__ part, int S, int b, int n,
                                     const T* __restrict__ gcost, T* __restrict__ grad1) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)b * n * 3;
  if (i >= total) return;
  const int bb = (int)(i / ((size_t)n * 3));
  grad1[i] = sum_parts(part, S, total, i) * gcost[bb];
}

// grad2: one block per (l, b); lanes stride over k, block reduce (:285-323).
template <typename T>
__global__ void __launch_bounds__(kThreads)
    emd_grad2_kernel(const T* __restrict__ xyz1, const T* __restrict__ xyz2,
                     const T* __restrict__ match, const T* __restrict__ gcost, int n, int m,
                     T* __restrict__ grad2) {
  __shared__ T red[kThreads / 64];
  const int l = blockIdx.x, bb = blockIdx.y;
  const T* p2 = xyz2 + ((size_t)bb * m + l) * 3;
  const T x2 = p2[0], y2 = p2[1], z2 = p2[2];
  const T* __restrict__ row = match + ((size_t)bb * m + l) * n;
  const T* __restrict__ pb = xyz1 + (size_t)bb * n * 3;
  T sx = 0, sy = 0, sz = 0;
  for (int k = threadIdx.x; k < n; k += kThreads) {
    const T d = row[k] * (T)2;
    sx = fmaT<T>(x2 - pb[3 * k], d, sx);
    sy = fmaT<T>(y2 - pb[3 * k + 1], d, sy);
    sz = fmaT<T>(z2 - pb[3 * k + 2], d, sz);
  }
  const T tx = block_sum(sx, red);
  const T ty = block_sum(sy, red);
  const T tz = block_sum(sz, red);
  if (threadIdx.x == 0) {
    const T g = gcost[bb];
    T* o = grad2 + ((size_t)bb * m + l) * 3;
    o[0] = tx * g;
    o[1] = ty * g;
    o[2] = tz * g;
  }
}

int emd_splits(int b, int n, int m) {
  const long long rows = (long long)b * std::max(n, m);
  const long long want_lanes = 4LL * kCUs * 4 * 64;  // ~4 waves per SIMD
  int s = (int)std::max(1LL, (want_lanes + rows - 1) / std::max(1LL, rows));
  s = std::min(s, std::max(1, std::min(n, m) / 64));
  return std::max(1, std::min(s, 32));
}

template <typename T>
struct EmdWs {
  T *remL, *remR, *ratL, *ratR, *levL, *levR, *part;
};

size_t emd_ws_elems(int b, int n, int m) {
  const size_t bn = (size_t)b * n, bm = (size_t)b * m;
  const int S = emd_splits(b, n, m);
  // the partials of the split form / the row-pass form's point packs (4 (bn + 2 bm));
  // the region starts at 12 (bn + bm) elements: 16-B aligned for f32, 32-B for f64
  const size_t part = std::max({(size_t)S * b * std::max(n, m) * 3,
                                (size_t)b * S * ceil_div(std::max(n, 1), kThreads),
                                4 * (bn + 2 * bm) +
                                    (size_t)b * ceil_div(std::max(m, 1), kMatchL) *
                                        ceil_div(std::max(n, 1), kThreads)});
  return 2 * (bn + bm) + kLevels * (bn + bm) + part;
}

template <typename T>
EmdWs<T> carve(void* ws, int b, int n, int m) {
  const size_t bn = (size_t)b * n, bm = (size_t)b * m;
  T* p = (T*)ws;
  EmdWs<T> w;
  w.remL = p;
  p += bn;
  w.remR = p;
  p += bm;
  w.ratL = p;
  p += bn;
  w.ratR = p;
  p += bm;
  w.levL = p;
  p += kLevels * bn;
  w.levR = p;
  p += kLevels * bm;
  w.part = p;
  return w;
}

inline dim3 grid1d(size_t total, int threads = 256) {
  return dim3(ceil_div((long long)std::max<size_t>(total, 1), threads));
}

// ---------------------------------------------------------------------------
// Row-pass form (the default): ONE launch per pass of each level, its finalize
// included, and no partial-sum buffer.  A block owns 64 rows (one per lane)
// and splits the column range over its 16 waves; the 16 wave sums of a row
// are added in wave order in LDS and the row's finalize (fin1 / fin2 / fin3
// of the split form) runs right there, so the next pass reads finished
// coefficients.  A level's third pass and the next level's first pass walk
// the same (row k, column l) pairs, so they share one launch and one d2 per
// pair: 21 pass launches + the pack + the match write (with the cost fused).
// Measured history (B = 8, N = 2048, MI355X): the split form below (6 launches
// per level, S-way partials reduced by separate finalize kernels) 0.67 ms; a
// form with the finalizes folded into the next pass, each block re-reducing
// the S partials of its columns, 0.80 ms (the serial partial reads sat in front
// of every pass); the round-3 cooperative one-launch form with
// cooperative_groups grid barriers 4.45 ms (a grid.sync() costs ~0.1 us per
// block on ROCm 7.2, ~100 us at 1024 blocks, against ~1.7 us for a kernel
// boundary); this form with 30 separate pass launches and scalar-loaded
// columns 0.51 ms, with LDS-staged columns and the fused cost 0.39 ms.
// ---------------------------------------------------------------------------
constexpr int kRowWaves = 16;  // column splits per block, one wave each

// A point with the coefficient it carries into a pass (x, y, z, w = coef),
// float4 / double4: a native vector type, so copies stay in registers.
template <typename T>
struct Vec4Of;
template <>
struct Vec4Of<float> {
  using type = float4;
};
template <>
struct Vec4Of<double> {
  using type = double4;
};
template <typename T>
using Col4 = typename Vec4Of<T>::type;

// packK[b, k] = {xyz1, ratL};  packL0[b, l] = {xyz2, remR};  packL1[b, l] = {xyz2, ratR}
template <typename T>
struct EmdRowState {
  Col4<T>* packK;
  Col4<T>* packL0;
  Col4<T>* packL1;
  T* remL;
  T* levL;  // [kLevels][b * n]
  T* levR;  // [kLevels][b * m]
};

template <typename T>
__global__ void emd_pack_kernel(const T* __restrict__ xyz1, size_t bn, T multiL,
                                const T* __restrict__ xyz2, size_t bm, T multiR,
                                EmdRowState<T> s) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < bn) {
    s.packK[i] = Col4<T>(xyz1[3 * i], xyz1[3 * i + 1], xyz1[3 * i + 2], (T)0);
    s.remL[i] = multiL;
  }
  if (i < bm) {
    const T x = xyz2[3 * i], y = xyz2[3 * i + 1], z = xyz2[3 * i + 2];
    s.packL0[i] = Col4<T>(x, y, z, multiR);
    s.packL1[i] = Col4<T>(x, y, z, (T)0);
  }
}

// PH 0: rows k (packK), cols packL0 (coef remR);  suml -> ratL = remL / (1e-9 + suml)  (:57-81)
// PH 1: rows l (packL0), cols packK (coef ratL);  sumr -> ratR, levR[lvl], remR (fin2) (:86-116)
// PH 2: rows k (packK, row scale ratL), cols packL1 (coef ratR);  -> remL, levL[lvl]   (:119-151)
// grid = (ceil(nr / 64), b), 1024 threads.  Each wave stages its column slice
// through a wave-private LDS chunk (one 16-B load per lane and column pair,
// the next chunk's loads in flight while this one is used); the column loop
// then reads a column as one broadcast ds_read, whose in-order completion
// lets the compiler keep several in flight (scalar loads of the columns
// complete out of order, so every use waited for all of them: 13.8 us/pass).
constexpr int kColChunk = 128;  // columns per wave per LDS chunk (64 for PH 3: two packs)

template <typename T, int PH>
__device__ __forceinline__ T rowpass_chunk(const Col4<T>* __restrict__ st, int cnt, T x1, T y1,
                                           T z1, T rl, T lvl2, T acc) {
  if (lvl2 == (T)0) {  // level 0: exp(0 * d2) = 1 exactly
#pragma unroll 8
    for (int c = 0; c < cnt; ++c) acc = fmaT<T>(PH == 2 ? rl : (T)1, st[c].w, acc);
    return acc;
  }
#pragma unroll 8
  for (int c = 0; c < cnt; ++c) {
    const Col4<T> q = st[c];
    const T d2 = sqdist3(q.x - x1, q.y - y1, q.z - z1);
    // level * log2(e) folded into one float factor: level is -4^j, a power of
    // two, so d2 * (level * log2 e) rounds exactly as emd_exp's (level * d2) * log2 e
    const T e = (T)__builtin_amdgcn_exp2f((float)d2 * (float)lvl2);
    if constexpr (PH == 2) {
      acc = fmaT<T>(e * rl, q.w, acc);
    } else {
      acc = fmaT<T>(e, q.w, acc);
    }
  }
  return acc;
}

// PH 3 = PH 2 of level j fused with PH 0 of level j+1 (same rows k, same
// columns l, one d2 per pair): st[c] = {xyz2, ratR_j}, st[64 + c].w = remR_{j+1}
template <typename T>
__device__ __forceinline__ void rowpass_pair(const Col4<T>* __restrict__ st, int cnt, T x1, T y1,
                                             T z1, T rl, T lvl2, T lvl2b, T& acc2, T& acc0) {
#pragma unroll 8
  for (int c = 0; c < cnt; ++c) {
    const Col4<T> q = st[c];
    const T rr = st[64 + c].w;
    const float d2 = (float)sqdist3(q.x - x1, q.y - y1, q.z - z1);
    const T e2 = (T)__builtin_amdgcn_exp2f(d2 * (float)lvl2);
    const T e0 = (T)__builtin_amdgcn_exp2f(d2 * (float)lvl2b);
    acc2 = fmaT<T>(e2 * rl, q.w, acc2);
    acc0 = fmaT<T>(e0, rr, acc0);
  }
}

// PH 0: rows k (packK), cols packL0 (coef remR);  suml -> ratL = remL / (1e-9 + suml)  (:57-81)
// PH 1: rows l (packL0), cols packK (coef ratL);  sumr -> ratR, levR[lvl], remR (fin2) (:86-116)
// PH 2: rows k (packK, row scale ratL), cols packL1 (coef ratR);  -> remL, levL[lvl]   (:119-151)
// PH 3: PH 2 of level lvl then PH 0 of level lvl+1 (lvl2b), one launch: the
//       column sums of both are taken in the same order as the two launches,
//       so the result is bit-identical (PCFM_EMD_FORM=unfused runs them apart).
// grid = (ceil(nr / 64), b), 1024 threads.  Each wave stages its column slice
// through a wave-private LDS chunk (16-B loads, the next chunk's loads in
// flight while this one is used); the column loop then reads a column as one
// broadcast ds_read, whose in-order completion lets the compiler keep several
// in flight (scalar loads of the columns complete out of order, so every use
// waited for all of them: 13.8 us/pass).
template <typename T, int PH>
__global__ void __launch_bounds__(64 * kRowWaves)
    emd_rowpass_kernel(int nr, int ncol, T lvl2, T lvl2b, int lvl, EmdRowState<T> s) {
  constexpr int CH = PH == 3 ? 64 : kColChunk;
  __shared__ T red[kRowWaves][64];
  __shared__ T red2[PH == 3 ? kRowWaves : 1][64];
  __shared__ Col4<T> stage[kRowWaves][kColChunk];
  Col4<T>* rows = PH == 1 ? s.packL0 : s.packK;
  const Col4<T>* __restrict__ cols = PH == 0 ? s.packL0 : (PH == 1 ? s.packK : s.packL1);
  const int bb = blockIdx.y, lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = blockIdx.x * 64 + lane;
  const int ii = i < nr ? i : nr - 1;
  const Col4<T> rp = rows[(size_t)bb * nr + ii];
  const T rl = rp.w;  // PH 2 / 3: ratL of the row
  const int c0 = (int)(((long long)ncol * w) / kRowWaves);
  const int c1 = (int)(((long long)ncol * (w + 1)) / kRowWaves);
  const Col4<T>* __restrict__ cb = cols + (size_t)bb * ncol;
  const Col4<T>* __restrict__ cb2 = s.packL0 + (size_t)bb * ncol;  // PH 3's remR_{lvl+1}
  Col4<T>* st = stage[w];
  T acc = 0, acc2 = 0;
  // unconditional loads (index clamped to the batch element's last column; the
  // extra columns are never read): no branch around a load in flight
  const int cl = ncol - 1;
  Col4<T> n0, n1;
  auto fetch = [&](int base) {
    n0 = cb[min(base + lane, cl)];
    n1 = PH == 3 ? cb2[min(base + lane, cl)] : cb[min(base + 64 + lane, cl)];
  };
  fetch(c0);
  for (int base = c0; base < c1; base += CH) {
    st[lane] = n0;
    st[64 + lane] = n1;
    fetch(base + CH);
    const int cnt = min(CH, c1 - base);
    if constexpr (PH == 3) {
      rowpass_pair<T>(st, cnt, rp.x, rp.y, rp.z, rl, lvl2, lvl2b, acc2, acc);
    } else {
      acc = rowpass_chunk<T, PH>(st, cnt, rp.x, rp.y, rp.z, rl, lvl2, acc);
    }
  }
  red[w][lane] = acc;
  if constexpr (PH == 3) red2[w][lane] = acc2;
  __syncthreads();
  if (w != 0 || i >= nr) return;
  T t = 0, t2 = 0;
#pragma unroll
  for (int q = 0; q < kRowWaves; ++q) {
    t += red[q][lane];
    if constexpr (PH == 3) t2 += red2[q][lane];
  }
  const size_t idx = (size_t)bb * nr + i;
  const size_t lv = (size_t)lvl * gridDim.y * nr + idx;
  if constexpr (PH == 0) {
    rows[idx].w = s.remL[idx] / ((T)1e-9f + t);
  } else if constexpr (PH == 1) {
    const T r = rp.w;
    const T sumr = t * r;
    const T cons = (T)fminf((float)(r / (sumr + (T)1e-9f)), 1.0f);
    const T rat = cons * r;
    s.packL1[idx].w = rat;
    s.levR[lv] = rat;
    rows[idx].w = (T)fmaxf(0.0f, (float)(r - sumr));
  } else if constexpr (PH == 2) {
    s.remL[idx] = (T)fmaxf(0.0f, (float)(s.remL[idx] - t));
    s.levL[lv] = rl;
  } else {
    const T rem = (T)fmaxf(0.0f, (float)(s.remL[idx] - t2));  // level lvl's fin3
    s.remL[idx] = rem;
    s.levL[lv] = rl;
    rows[idx].w = rem / ((T)1e-9f + t);  // level lvl+1's ratL
  }
}

// PCFM_EMD_FORM=split: every pass and finalize its own launch, S-way partials
// (measurement / the cross-form test); =unfused: the row-pass form with PH 2
// and the next level's PH 0 as separate launches; default: the fused row-pass form
bool emd_split_form() {
  const char* e = std::getenv("PCFM_EMD_FORM");
  return e != nullptr && e[0] == 's';
}
bool emd_unfused_form() {
  const char* e = std::getenv("PCFM_EMD_FORM");
  return e != nullptr && e[0] == 'u';
}

// match (when non-null) and, when cost is non-null, the fused matchcost.
template <typename T>
int approxmatch_rowpass(const T* xyz1, const T* xyz2, int b, int n, int m, T* match, T* cost,
                        EmdWs<T> w, hipStream_t st) {
  const size_t bn = (size_t)b * n, bm = (size_t)b * m;
  Col4<T>* pk = reinterpret_cast<Col4<T>*>(w.part);  // 16/32-B aligned: see emd_ws_elems
  EmdRowState<T> s{pk, pk + bn, pk + bn + bm, w.remL, w.levL, w.levR};
  const T multiL = n >= m ? (T)1 : (T)(m / n);  // integer ratio of the cloud sizes (:27-33)
  const T multiR = n >= m ? (T)(n / m) : (T)1;
  hipLaunchKernelGGL(emd_pack_kernel<T>, grid1d(std::max(bn, bm)), dim3(256), 0, st, xyz1, bn,
                     multiL, xyz2, bm, multiR, s);
  const dim3 gL(ceil_div(n, 64), b), gR(ceil_div(m, 64), b), blk(64 * kRowWaves);
  // level_j * log2(e), exact in float: level_j is a power of two
  auto lv2 = [](int j) { return (T)(h_levels[j] * 1.4426950408889634f); };
  const bool fused = !emd_unfused_form();
  hipLaunchKernelGGL((emd_rowpass_kernel<T, 0>), gL, blk, 0, st, n, m, lv2(0), (T)0, 0, s);
  for (int j = 0; j < kLevels; ++j) {
    hipLaunchKernelGGL((emd_rowpass_kernel<T, 1>), gR, blk, 0, st, m, n, lv2(j), (T)0, j, s);
    if (fused && j + 1 < kLevels) {
      hipLaunchKernelGGL((emd_rowpass_kernel<T, 3>), gL, blk, 0, st, n, m, lv2(j), lv2(j + 1), j,
                         s);
    } else {
      hipLaunchKernelGGL((emd_rowpass_kernel<T, 2>), gL, blk, 0, st, n, m, lv2(j), (T)0, j, s);
      if (j + 1 < kLevels)
        hipLaunchKernelGGL((emd_rowpass_kernel<T, 0>), gL, blk, 0, st, n, m, lv2(j + 1), (T)0,
                           j + 1, s);
    }
  }
  const dim3 gm(ceil_div(n, kThreads), ceil_div(m, kMatchL), b);
  T* cpart = w.part + 4 * (bn + 2 * bm);  // after the packs (emd_ws_elems)
  hipLaunchKernelGGL(emd_match_cost_kernel<T>, gm, dim3(kThreads), 0, st, xyz1, xyz2, b, n, m,
                     (const T*)w.levL, (const T*)w.levR, match, cpart);
  if (cost != nullptr)
    hipLaunchKernelGGL(emd_cost_fin_kernel<T>, dim3(b), dim3(64), 0, st, (const T*)cpart,
                       (int)(gm.x * gm.y), cost);
  return check_launch("approxmatch");
}

template <typename T>
int approxmatch(const T* xyz1, const T* xyz2, int b, int n, int m, T* match, void* ws,
                size_t ws_bytes, hipStream_t st) {
  PCFM_CHECK_ARG(b >= 0 && n >= 0 && m >= 0, "approxmatch: negative size");
  PCFM_CHECK_ARG(ws_bytes >= emd_ws_elems(b, n, m) * sizeof(T),
                 "approxmatch: workspace %zu < %zu bytes", ws_bytes,
                 emd_ws_elems(b, n, m) * sizeof(T));
  if (b == 0 || n == 0 || m == 0) return PCFM_OK;
  EmdWs<T> w = carve<T>(ws, b, n, m);
  if (!emd_split_form()) return approxmatch_rowpass(xyz1, xyz2, b, n, m, match, (T*)nullptr, w, st);
  const int S = emd_splits(b, n, m);
  // multiL/multiR: integer ratio of the cloud sizes (:27-33)
  const T multiL = n >= m ? (T)1 : (T)(m / n);
  const T multiR = n >= m ? (T)(n / m) : (T)1;
  const size_t bn = (size_t)b * n, bm = (size_t)b * m;
  hipLaunchKernelGGL(emd_init_kernel<T>, grid1d(std::max(bn, bm)), dim3(256), 0, st, w.remL, bn,
                     multiL, w.remR, bm, multiR);
  const dim3 gL(ceil_div(n, kThreads), S, b), gR(ceil_div(m, kThreads), S, b);
  for (int j = 0; j < kLevels; ++j) {
    const T level = (T)h_levels[j];
    // pass 1: rows = xyz1 (k), cols = xyz2 (l), coef = remainR
    hipLaunchKernelGGL((emd_pass_kernel<T, 0>), gL, dim3(kThreads), 0, st, xyz1, n, xyz2, m, b,
                       level, w.remR, (const T*)nullptr, S, w.part);
    hipLaunchKernelGGL(emd_fin1_kernel<T>, grid1d(bn), dim3(256), 0, st, w.part, S, bn, w.remL,
                       w.ratL);
    // pass 2: rows = xyz2 (l), cols = xyz1 (k), coef = ratioL
    hipLaunchKernelGGL((emd_pass_kernel<T, 1>), gR, dim3(kThreads), 0, st, xyz2, m, xyz1, n, b,
                       level, w.ratL, (const T*)nullptr, S, w.part);
    hipLaunchKernelGGL(emd_fin2_kernel<T>, grid1d(bm), dim3(256), 0, st, w.part, S, bm, w.remR,
                       w.ratR, w.levR + (size_t)j * bm);
    // pass 3: rows = xyz1 (k), cols = xyz2 (l), coef = ratioR, rowscale = ratioL
    hipLaunchKernelGGL((emd_pass_kernel<T, 2>), gL, dim3(kThreads), 0, st, xyz1, n, xyz2, m, b,
                       level, w.ratR, (const T*)w.ratL, S, w.part);
    hipLaunchKernelGGL(emd_fin3_kernel<T>, grid1d(bn), dim3(256), 0, st, w.part, S, bn, w.remL,
                       w.ratL, w.levL + (size_t)j * bn);
  }
  dim3 gm(ceil_div(n, kThreads), ceil_div(m, kLPer), b);
  hipLaunchKernelGGL(emd_match_kernel<T>, gm, dim3(kThreads), 0, st, xyz1, xyz2, b, n, m, w.levL,
                     w.levR, match);
  return check_launch("approxmatch");
}

// approxmatch + matchcost in one call (row-pass form; the cost from the match
// kernel's partials).  match may be null: the cost alone, match not written.
template <typename T>
int approxmatch_cost(const T* xyz1, const T* xyz2, int b, int n, int m, T* match, T* cost,
                     void* ws, size_t ws_bytes, hipStream_t st) {
  PCFM_CHECK_ARG(b >= 0 && n >= 0 && m >= 0, "approxmatch_cost: negative size");
  PCFM_CHECK_ARG(cost != nullptr, "approxmatch_cost: cost is required");
  PCFM_CHECK_ARG(ws_bytes >= emd_ws_elems(b, n, m) * sizeof(T),
                 "approxmatch_cost: workspace %zu < %zu bytes", ws_bytes,
                 emd_ws_elems(b, n, m) * sizeof(T));
  if (b == 0) return PCFM_OK;
  if (n == 0 || m == 0) {
    hipError_t e = hipMemsetAsync(cost, 0, (size_t)b * sizeof(T), st);
    if (e == hipSuccess && match != nullptr)
      e = hipMemsetAsync(match, 0, (size_t)b * n * m * sizeof(T), st);
    if (e != hipSuccess) {
      set_error("approxmatch_cost: hipMemsetAsync: %s", hipGetErrorString(e));
      return (int)e;
    }
    return PCFM_OK;
  }
  return approxmatch_rowpass(xyz1, xyz2, b, n, m, match, cost, carve<T>(ws, b, n, m), st);
}

template <typename T>
int matchcost(const T* xyz1, const T* xyz2, const T* match, int b, int n, int m, T* cost,
              void* ws, size_t ws_bytes, hipStream_t st) {
  PCFM_CHECK_ARG(b >= 0 && n >= 0 && m >= 0, "matchcost: negative size");
  PCFM_CHECK_ARG(ws_bytes >= emd_ws_elems(b, n, m) * sizeof(T),
                 "matchcost: workspace %zu < %zu bytes", ws_bytes,
                 emd_ws_elems(b, n, m) * sizeof(T));
  if (b == 0) return PCFM_OK;
  if (n == 0 || m == 0) {
    hipError_t e = hipMemsetAsync(cost, 0, (size_t)b * sizeof(T), st);
    if (e != hipSuccess) {
      set_error("matchcost: hipMemsetAsync: %s", hipGetErrorString(e));
      return (int)e;
    }
    return PCFM_OK;
  }
  EmdWs<T> w = carve<T>(ws, b, n, m);
  const int S = emd_splits(b, n, m);
  dim3 g(ceil_div(n, kThreads), S, b);
  hipLaunchKernelGGL(emd_cost_kernel<T>, g, dim3(kThreads), 0, st, xyz1, xyz2, match, b, n, m, S,
                     w.part);
  const int per_b = S * (int)g.x;
  hipLaunchKernelGGL(emd_cost_fin_kernel<T>, dim3(b), dim3(64), 0, st, (const T*)w.part, per_b,
                     cost);
  return check_launch("matchcost");
}

template <typename T>
int matchcost_bwd(const T* gcost, const T* xyz1, const T* xyz2, const T* match, int b, int n,
                  int m, T* grad1, T* grad2, void* ws, size_t ws_bytes, hipStream_t st) {
  PCFM_CHECK_ARG(b >= 0 && n >= 0 && m >= 0, "matchcost_bwd: negative size");
  PCFM_CHECK_ARG(ws_bytes >= emd_ws_elems(b, n, m) * sizeof(T),
                 "matchcost_bwd: workspace %zu < %zu bytes", ws_bytes,
                 emd_ws_elems(b, n, m) * sizeof(T));
  if (b == 0) return PCFM_OK;
  if (n == 0 || m == 0) {
    hipError_t e = hipSuccess;
    if (n) e = hipMemsetAsync(grad1, 0, (size_t)b * n * 3 * sizeof(T), st);
    if (m && e == hipSuccess) e = hipMemsetAsync(grad2, 0, (size_t)b * m * 3 * sizeof(T), st);
    if (e != hipSuccess) {
      set_error("matchcost_bwd: hipMemsetAsync: %s", hipGetErrorString(e));
      return (int)e;
    }
    return PCFM_OK;
  }
  EmdWs<T> w = carve<T>(ws, b, n, m);
  const int S = emd_splits(b, n, m);
  hipLaunchKernelGGL(emd_grad1_kernel<T>, dim3(ceil_div(n, kThreads), S, b), dim3(kThreads), 0,
                     st, xyz1, xyz2, match, b, n, m, S, w.part);
  hipLaunchKernelGGL(emd_grad1_fin_kernel<T>, grid1d((size_t)b * n * 3), dim3(256), 0, st,
                     w.part, S, b, n, gcost, grad1);
  hipLaunchKernelGGL(emd_grad2_kernel<T>, dim3(m, b), dim3(kThreads), 0, st, xyz1, xyz2, match,
                     gcost, n, m, grad2);
  return check_launch("matchcost_bwd");
}

}  // namespace
}  // namespace pcfm

using namespace pcfm;

extern "C" size_t pcfm_emd_workspace_bytes(int b, int n, int m, int elem_bytes) {
  if (b < 0 || n < 0 || m < 0 || (elem_bytes != 4 && elem_bytes != 8)) return 0;
  return emd_ws_elems(b, n, m) * (size_t)elem_bytes;
}

extern "C" int pcfm_emd_approxmatch_f32(const float* xyz1, const float* xyz2, int b, int n, int m,
                                        float* match, void* ws, size_t ws_bytes, void* stream) {
  return approxmatch<float>(xyz1, xyz2, b, n, m, match, ws, ws_bytes, (hipStream_t)stream);
}
extern "C" int pcfm_emd_approxmatch_f64(const double* xyz1, const double* xyz2, int b, int n,
                                        int m, double* match, void* ws, size_t ws_bytes,
                                        void* stream) {
  return approxmatch<double>(xyz1, xyz2, b, n, m, match, ws, ws_bytes, (hipStream_t)stream);
}
extern "C" int pcfm_emd_approxmatch_cost_f32(const float* xyz1, const float* xyz2, int b, int n,
                                             int m, float* match, float* cost, void* ws,
                                             size_t ws_bytes, void* stream) {
  return approxmatch_cost<float>(xyz1, xyz2, b, n, m, match, cost, ws, ws_bytes,
                                 (hipStream_t)stream);
}
extern "C" int pcfm_emd_approxmatch_cost_f64(const double* xyz1, const double* xyz2, int b, int n,
                                             int m, double* match, double* cost, void* ws,
                                             size_t ws_bytes, void* stream) {
  return approxmatch_cost<double>(xyz1, xyz2, b, n, m, match, cost, ws, ws_bytes,
                                  (hipStream_t)stream);
}
extern "C" int pcfm_emd_matchcost_f32(const float* xyz1, const float* xyz2, const float* match,
                                      int b, int n, int m, float* cost, void* ws,
                                      size_t ws_bytes, void* stream) {
  return matchcost<float>(xyz1, xyz2, match, b, n, m, cost, ws, ws_bytes, (hipStream_t)stream);
}
extern "C" int pcfm_emd_matchcost_f64(const double* xyz1, const double* xyz2,
                                      const double* match, int b, int n, int m, double* cost,
                                      void* ws, size_t ws_bytes, void* stream) {
  return matchcost<double>(xyz1, xyz2, match, b, n, m, cost, ws, ws_bytes, (hipStream_t)stream);
}
extern "C" int pcfm_emd_matchcost_bwd_f32(const float* grad_cost, const float* xyz1,
                                          const float* xyz2, const float* match, int b, int n,
                                          int m, float* grad1, float* grad2, void* ws,
                                          size_t ws_bytes, void* stream) {
  return matchcost_bwd<float>(grad_cost, xyz1, xyz2, match, b, n, m, grad1, grad2, ws, ws_bytes,
                              (hipStream_t)stream);
}
extern "C" int pcfm_emd_matchcost_bwd_f64(const double* grad_cost, const double* xyz1,
                                          const double* xyz2, const double* match, int b, int n,
                                          int m, double* grad1, double* grad2, void* ws,
                                          size_t ws_bytes, void* stream) {
  return matchcost_bwd<double>(grad_cost, xyz1, xyz2, match, b, n, m, grad1, grad2, ws,
                               ws_bytes, (hipStream_t)stream);
}
