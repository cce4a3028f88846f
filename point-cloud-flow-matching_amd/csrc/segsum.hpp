// Sorted, atomic-free scatter ("segment sum") for the PVConv path.
//
// Measured on MI355X (tools/voxel_probe.py): an LDS float atomic (ds_add_f32)
// costs ~200 cycles per wave instruction whatever the address pattern, so the
// LDS-privatised scatter of rows.hpp runs at 0.15-0.9 TB/s.  The scatters are
// therefore recast as gathers over points sorted by their target cell:
//
//   1. count   cnt[b, key]              integer atomics (exact)
//   2. scan    start[b, 0..V]           exclusive prefix sums, one block per b
//   3. place   perm[b, start[key] + r]  points grouped by key
//   4. gather-transpose  XS[b, j, c] = in[b, c, perm[j]] * scale[perm[j]]
//                        (channels-last rows, 256 B per point per 64 channels)
//   5. tap sum out[b, c, v] = sum_k sum_{j in run(v - off_k)} w_k(j) * XS[b, j, c]
//      lanes = 64 channels, one wave per tap (8 waves for the trilinear
//      stencil, 4 voxel-interleaved waves for 1 tap), partials reduced in a
//      fixed tap order in LDS, rows written out coalesced.  No atomics.
//
// Used by avg_voxelize forward (key = voxel, scale = 1/cnt), trilinear
// devoxelize backward (key = base cell inds[b,0,:], 8 taps with wgts) and
// grouping backward (key = neighbour index).  The order of points inside one
// key comes from step 3's atomics, so float sums are order-nondeterministic
// at the last bit -- exactly like the reference's float atomics.
#pragma once

#include <algorithm>

#include "pcfm_common.hpp"

namespace pcfm {
namespace {  // kernels get internal linkage: this header is included by several .hip files

// --------------------------------------------------------------------------
// 1-3: sort items by key
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
    seg_count_kernel(const int* __restrict__ key, long long key_bstride, int n, int V,
                     int* __restrict__ cnt) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int k = key[(size_t)b * key_bstride + i];
  if ((unsigned)k < (unsigned)V) atomicAdd(cnt + (size_t)b * V + k, 1);
}

// One block (1024 threads) per batch element: start[b, v] = sum_{u<v} cnt[b, u],
// start[b, V] = total; cursor = start[0..V).
__global__ void __launch_bounds__(1024)
    seg_scan_kernel(const int* __restrict__ cnt, int V, int* __restrict__ start,
                    int* __restrict__ cursor) {
  __shared__ int wsum[16];
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int per = (V + 1023) / 1024;
  const int lo = min(V, t * per), hi = min(V, lo + per);
  const int* cb = cnt + (size_t)b * V;
  int local = 0;
  for (int v = lo; v < hi; ++v) local += cb[v];
  // inclusive scan of `local` across the block
  int x = local;
  const int lane = t & 63, w = t >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (t < 64) {
    int s = (t < 16) ? wsum[t] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int y = __shfl_up(s, o, 64);
      if (lane >= o) s += y;
    }
    if (t < 16) wsum[t] = s;
  }
  __syncthreads();
  int run = x - local + (w > 0 ? wsum[w - 1] : 0);  // exclusive prefix of this thread
  int* sb = start + (size_t)b * (V + 1);
  int* kb = cursor + (size_t)b * V;
  for (int v = lo; v < hi; ++v) {
    sb[v] = run;
    kb[v] = run;
    run += cb[v];
  }
  if (t == 1023) sb[V] = wsum[15];
}

__global__ void __launch_bounds__(256)
    seg_place_kernel(const int* __restrict__ key, long long key_bstride, int n, int V,
                     int* __restrict__ cursor, int* __restrict__ perm) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int k = key[(size_t)b * key_bstride + i];
  if ((unsigned)k < (unsigned)V) {
    const int pos = atomicAdd(cursor + (size_t)b * V + k, 1);
    perm[(size_t)b * n + pos] = i;
  }
}

// --------------------------------------------------------------------------
// 4: gather-transpose into sorted channels-last rows
// grid = (ceil(n/64), ceil(C/64), B), 256 threads.  perm entries past the
// valid count are -1 (pre-filled) and produce zero rows.
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
    seg_gather_t_kernel(const float* __restrict__ in, const int* __restrict__ perm,
                        const float* __restrict__ scale, const float* __restrict__ tapw,
                        int C, int n, float* __restrict__ xs, float* __restrict__ ws8) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z;
  const int j0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int jj = j0 + lane;
  const int p = jj < n ? perm[(size_t)b * n + jj] : -1;
  const float sc = (scale != nullptr && p >= 0) ? scale[(size_t)b * n + p] : 1.0f;
  for (int cc = w; cc < 64; cc += 4) {
    const int c = c0 + cc;
    float v = 0.0f;
    if (c < C && p >= 0) {
      v = in[((size_t)b * C + c) * n + p];
      if (scale != nullptr) v = v * sc;  // the reference's per-term product (vox.cu:68)
    }
    tile[cc][lane] = v;
  }
  if (tapw != nullptr && blockIdx.y == 0 && w == 0 && jj < n) {
    float4 lo, hi;  // WS[b, j, 0..7] = wgts[b, 0..7, perm[j]]
    const float* tb = tapw + (size_t)b * 8 * n + (p >= 0 ? p : 0);
    lo.x = p >= 0 ? tb[0] : 0.0f;
    lo.y = p >= 0 ? tb[(size_t)n] : 0.0f;
    lo.z = p >= 0 ? tb[(size_t)2 * n] : 0.0f;
    lo.w = p >= 0 ? tb[(size_t)3 * n] : 0.0f;
    hi.x = p >= 0 ? tb[(size_t)4 * n] : 0.0f;
    hi.y = p >= 0 ? tb[(size_t)5 * n] : 0.0f;
    hi.z = p >= 0 ? tb[(size_t)6 * n] : 0.0f;
    hi.w = p >= 0 ? tb[(size_t)7 * n] : 0.0f;
    float4* o = reinterpret_cast<float4*>(ws8 + ((size_t)b * n + jj) * 8);
    o[0] = lo;
    o[1] = hi;
  }
  __syncthreads();
  const int c = c0 + lane;
  if (c < C) {
    for (int jr = w; jr < 64; jr += 4) {
      const int j = j0 + jr;
      if (j < n) xs[((size_t)b * n + j) * C + c] = tile[lane][jr];
    }
  }
}

// --------------------------------------------------------------------------
// 5: tap sums, output-stationary
// grid = (ceil(V/TV), ceil(C/64), B).  TAPS == 8: 8 waves, wave k = corner k
// (dx,dy,dz) = (k>>2, (k>>1)&1, k&1) of the trilinear stencil (the reference's
// wgt000..wgt111 order, trilinear_devox.cu:178-185).  TAPS == 1: 4 waves share
// the tile's voxels round robin.
// --------------------------------------------------------------------------
template <int TAPS>
__global__ void __launch_bounds__(512)
    seg_tap_sum_kernel(const float* __restrict__ xs, const float* __restrict__ ws8,
                       const int* __restrict__ start, int C, int n, int V, int r, int TV,
                       float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float part[];  // [TAPS][TV][65]
  const int b = blockIdx.z;
  const int v0 = blockIdx.x * TV, c0 = blockIdx.y * 64;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = c0 + lane;
  const bool cok = c < C;
  const int* sb = start + (size_t)b * (V + 1);
  const float* xb = xs + (size_t)b * n * C + (cok ? c : 0);
  const int r2 = r * r;
  if constexpr (TAPS == 8) {
    const int k = w;
    const int dx = k >> 2, dy = (k >> 1) & 1, dz = k & 1;
    const int off = dx * r2 + dy * r + dz;
    const float* wb = ws8 + (size_t)b * n * 8 + k;
    for (int vi = 0; vi < TV; ++vi) {
      const int v = v0 + vi;
      float acc = 0.0f;
      if (v < V) {
        const int X = v / r2, Y = (v / r) % r, Z = v % r;
        if (X >= dx && Y >= dy && Z >= dz) {
          const int q = v - off;
          int j = sb[q];
          const int e = sb[q + 1];
          for (; j + 4 <= e; j += 4) {
            const float x0 = xb[(size_t)j * C], x1 = xb[(size_t)(j + 1) * C];
            const float x2 = xb[(size_t)(j + 2) * C], x3 = xb[(size_t)(j + 3) * C];
            const float w0 = wb[(size_t)j * 8], w1 = wb[(size_t)(j + 1) * 8];
            const float w2 = wb[(size_t)(j + 2) * 8], w3 = wb[(size_t)(j + 3) * 8];
            acc = acc + w0 * x0;
            acc = acc + w1 * x1;
            acc = acc + w2 * x2;
            acc = acc + w3 * x3;
          }
          for (; j < e; ++j) acc = acc + wb[(size_t)j * 8] * xb[(size_t)j * C];
        }
      }
      part[(k * TV + vi) * 65 + lane] = acc;
    }
  } else {
    for (int vi = w; vi < TV; vi += (int)(blockDim.x >> 6)) {
      const int v = v0 + vi;
      float acc = 0.0f;
      if (v < V) {
        int j = sb[v];
        const int e = sb[v + 1];
        for (; j + 4 <= e; j += 4) {
          const float x0 = xb[(size_t)j * C], x1 = xb[(size_t)(j + 1) * C];
          const float x2 = xb[(size_t)(j + 2) * C], x3 = xb[(size_t)(j + 3) * C];
          acc = acc + x0;
          acc = acc + x1;
          acc = acc + x2;
          acc = acc + x3;
        }
        for (; j < e; ++j) acc = acc + xb[(size_t)j * C];
      }
      part[vi * 65 + lane] = acc;
    }
  }
  __syncthreads();
  // out[b, c0 + cc, v0 + vi] = sum_k part[k][vi][cc], k in order
  const int nthreads = blockDim.x;
  for (int e = threadIdx.x; e < 64 * TV; e += nthreads) {
    const int cc = e / TV, vi = e - cc * TV;
    const int cg = c0 + cc, v = v0 + vi;
    if (cg < C && v < V) {
      float s = part[vi * 65 + cc];
#pragma unroll
      for (int k = 1; k < TAPS; ++k) s = s + part[(k * TV + vi) * 65 + cc];
      out[((size_t)b * C + cg) * V + v] = s;
    }
  }
}

}  // namespace

// --------------------------------------------------------------------------
// host driver
// --------------------------------------------------------------------------
struct SegWs {
  int* start;   // B*(V+1)
  int* cursor;  // B*V
  int* perm;    // B*n
  int* cnt;     // B*V (when the caller does not own one)
  float* xs;    // B*n*C
  float* ws8;   // B*n*8 (TAPS == 8)
};

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

inline size_t seg_ws_bytes(int B, int C, int n, int V, int taps) {
  size_t s = 0;
  s += align256((size_t)B * (V + 1) * 4);
  s += align256((size_t)B * V * 4);
  s += align256((size_t)B * n * 4);
  s += align256((size_t)B * V * 4);
  s += align256((size_t)B * n * std::max(C, 1) * 4);
  if (taps == 8) s += align256((size_t)B * n * 8 * 4);
  return s;
}

inline SegWs seg_ws_carve(void* ws, int B, int C, int n, int V, int taps) {
  char* p = (char*)ws;
  SegWs w;
  w.start = (int*)p;
  p += align256((size_t)B * (V + 1) * 4);
  w.cursor = (int*)p;
  p += align256((size_t)B * V * 4);
  w.perm = (int*)p;
  p += align256((size_t)B * n * 4);
  w.cnt = (int*)p;
  p += align256((size_t)B * V * 4);
  w.xs = (float*)p;
  p += align256((size_t)B * n * std::max(C, 1) * 4);
  w.ws8 = taps == 8 ? (float*)p : nullptr;
  return w;
}

inline int seg_tile_voxels(int V) { return V >= 32768 ? 32 : (V >= 4096 ? 16 : 8); }

// out[b, c, v] = sum over items i with key(i) (+ stencil offset) = v of w * in[b, c, i].
//   key: [b, key_bstride] ints (first n used); cnt: [b, V] counts if already
//   computed by the caller (nullptr: computed here into the workspace).
template <int TAPS>
inline int seg_scatter(const float* in, const int* key, long long key_bstride,
                       const float* scale, const float* tapw, int r, int B, int C, int n, int V,
                       const int* cnt, float* out, void* ws, hipStream_t st, const char* what) {
  if (B == 0 || C == 0 || V == 0) return PCFM_OK;
  SegWs w = seg_ws_carve(ws, B, C, n, V, TAPS);
  hipError_t he = hipSuccess;
  if (cnt == nullptr) {
    he = hipMemsetAsync(w.cnt, 0, (size_t)B * V * 4, st);
    if (he == hipSuccess && n > 0)
      hipLaunchKernelGGL(seg_count_kernel, dim3(ceil_div(n, 256), B), dim3(256), 0, st, key,
                         key_bstride, n, V, w.cnt);
    cnt = w.cnt;
  }
  if (he == hipSuccess && n > 0) he = hipMemsetAsync(w.perm, 0xff, (size_t)B * n * 4, st);
  if (he != hipSuccess) {
    set_error("%s: hipMemsetAsync: %s", what, hipGetErrorString(he));
    return (int)he;
  }
  hipLaunchKernelGGL(seg_scan_kernel, dim3(B), dim3(1024), 0, st, cnt, V, w.start, w.cursor);
  if (n > 0) {
    hipLaunchKernelGGL(seg_place_kernel, dim3(ceil_div(n, 256), B), dim3(256), 0, st, key,
                       key_bstride, n, V, w.cursor, w.perm);
    hipLaunchKernelGGL(seg_gather_t_kernel, dim3(ceil_div(n, 64), ceil_div(C, 64), B),
                       dim3(256), 0, st, in, w.perm, scale, tapw, C, n, w.xs, w.ws8);
  }
  const int TV = seg_tile_voxels(V);
  const size_t lds = (size_t)TAPS * TV * 65 * sizeof(float);
  const int threads = TAPS == 8 ? 512 : 256;
  int e = allow_big_lds((const void*)seg_tap_sum_kernel<TAPS>);
  if (e) return e;
  hipLaunchKernelGGL(seg_tap_sum_kernel<TAPS>, dim3(ceil_div(V, TV), ceil_div(C, 64), B),
                     dim3(threads), lds, st, w.xs, w.ws8, w.start, C, n, V, r, TV, out);
  return check_launch(what);
}

}  // namespace pcfm
