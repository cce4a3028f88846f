// Sorted, atomic-free scatter ("segment sum") for the PVConv path.
//
// Measured on MI355X (tools/voxel_probe.py): an LDS float atomic (ds_add_f32)
// costs ~200 cycles per wave instruction whatever the address pattern, so an
// LDS-privatised scatter with one atomic per (item, channel, tap) runs at
// 0.15-0.9 TB/s.  The scatters are recast as gathers over items sorted by
// their target cell:
//
//   1-3. counting sort, one block per batch element, histogram in LDS:
//      start[b, 0..V] (exclusive prefix of the counts) and perm / skey at
//      start[key] + rank
//   4. transpose  xt[b, i, c] = in[b, c, i]       channels-last rows, item order
//   5. range gather, output-stationary per voxel tile, lanes = 64 channels.
//      The items feeding a tile [v0, v0+TV) through stencil column (dx, dy)
//      are ONE contiguous sorted range (cells v0-off-1 .. v0+TV-off-1 are
//      consecutive keys), so a wave streams that range, keeps one register
//      accumulator per dz tap for the current run of equal keys, and flushes
//      it into its own LDS partial tile when the key changes.  Ranges are cut
//      into chunks shared round robin by the block's waves and, for crowded
//      tiles, by up to P blocks (a dense r=8 cell holds thousands of points);
//      partial tiles are summed in a fixed order and leave as coalesced rows.
//      No atomics in the data path.
//
// Used by avg_voxelize forward (key = voxel, term = feat * (1/cnt)),
// trilinear devoxelize backward (key = base cell inds[b,0,:], term = wgt * g
// for the 8 corners) and grouping backward (key = neighbour index, term = g).
// The order of items inside one key comes from step 3's atomics, so float sums
// are order-nondeterministic at the last bit -- exactly like the reference's
// float atomics.
#pragma once

#include <algorithm>

#include "pcfm_common.hpp"

namespace pcfm {
namespace {  // kernels get internal linkage: this header is included by several .hip files

// --------------------------------------------------------------------------
// 1-3: counting sort by key, one block (1024 threads) per batch element.
// The key histogram lives in LDS (kSortKeys ints = 128 KiB; larger key spaces
// take several passes over the keys), so counting and ranking use LDS atomics
// only -- device-scope global atomics cost ~5 G/s on this part (measured:
// 160K of them took ~30 us), an LDS atomic a few hundred cycles per wave.
//   start[b, 0..V]  exclusive prefix of the counts (start[b, V] = total)
//   cnt_out[b, v]   the counts (optional: the voxelization's `cnt` output)
//   vinv[b, v]      (float)(1.0 / (double)cnt) (optional, vox.cu:66)
//   perm/skey[b, pos]  item and key at pos = start[key] + (arrival rank)
// --------------------------------------------------------------------------
constexpr int kSortKeys = 32768;
constexpr int kSortBatch = 8;  // keys per thread in flight

__global__ void __launch_bounds__(1024)
    seg_sort_kernel(const int* __restrict__ key, long long key_bstride, int n, int V,
                    int* __restrict__ start, int* __restrict__ cnt_out, float* __restrict__ vinv,
                    int* __restrict__ perm, int* __restrict__ skey) {
  extern __shared__ int hist[];  // [min(V, kSortKeys)]
  __shared__ int wsum[16];
  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int* __restrict__ kb = key + (size_t)b * key_bstride;
  int* __restrict__ sb = start + (size_t)b * (V + 1);
  int carry = 0;
  for (int k0 = 0; k0 < V; k0 += kSortKeys) {
    const int len = min(kSortKeys, V - k0);
    for (int e = t; e < len; e += 1024) hist[e] = 0;
    __syncthreads();
    for (int i0 = 0; i0 < n; i0 += 1024 * kSortBatch) {
      int kk[kSortBatch];  // keys first (independent loads), then the LDS atomics
#pragma unroll
      for (int q = 0; q < kSortBatch; ++q) {
        const int i = i0 + q * 1024 + t;
        kk[q] = i < n ? kb[i] - k0 : -1;
      }
#pragma unroll
      for (int q = 0; q < kSortBatch; ++q)
        if ((unsigned)kk[q] < (unsigned)len) atomicAdd(hist + kk[q], 1);
    }    __syncthreads();
    // exclusive scan: wave w owns the 64-aligned segment [lo, hi)
    const int seg = ((len + 15) / 16 + 63) & ~63;
    const int lo = min(len, w * seg), hi = min(len, lo + seg);
    int part = 0;
    for (int e = lo + lane; e < hi; e += 64) part += hist[e];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    if (lane == 0) wsum[w] = part;
    __syncthreads();
    int run = carry, total = 0;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int x = wsum[g];
      run += g < w ? x : 0;
      total += x;
    }
    for (int e0 = lo; e0 < hi; e0 += 64) {
      const int e = e0 + lane;
      const int c = e < hi ? hist[e] : 0;
      int x = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (e < hi) {
        const int pos = run + x - c;
        hist[e] = pos;
        sb[k0 + e] = pos;
        if (cnt_out != nullptr) cnt_out[(size_t)b * V + k0 + e] = c;
        if (vinv != nullptr) vinv[(size_t)b * V + k0 + e] = c > 0 ? (float)(1.0 / (double)c) : 0.0f;
      }
      run += __shfl(x, 63, 64);
    }
    __syncthreads();
    for (int i0 = 0; i0 < n; i0 += 1024 * kSortBatch) {
      int kk[kSortBatch];
#pragma unroll
      for (int q = 0; q < kSortBatch; ++q) {
        const int i = i0 + q * 1024 + t;
        kk[q] = i < n ? kb[i] - k0 : -1;
      }
#pragma unroll
      for (int q = 0; q < kSortBatch; ++q) {
        if ((unsigned)kk[q] < (unsigned)len) {
          const int pos = atomicAdd(hist + kk[q], 1);
          const size_t o = (size_t)b * n + pos;
          perm[o] = i0 + q * 1024 + t;
          skey[o] = kk[q] + k0;
        }
      }
    }
    carry += total;
    __syncthreads();
  }
  if (t == 0) sb[V] = carry;
}

// --------------------------------------------------------------------------
// 4: transpose the item features to channels-last rows, ORIGINAL item order:
//    xt[b, i, c] = in[b, c, i]   (64x64 LDS tiles; 256-B reads and writes)
// grid = (ceil(n/64), ceil(C/64), B), 256 threads.
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
    seg_transpose_kernel(const float* __restrict__ in, int C, int n, float* __restrict__ xt) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z;
  const int j0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int j = j0 + lane;
  for (int cc = w; cc < 64; cc += 4) {
    const int c = c0 + cc;
    tile[cc][lane] = (c < C && j < n) ? in[((size_t)b * C + c) * n + j] : 0.0f;
  }
  __syncthreads();
  const int c = c0 + lane;
  if (c < C) {
    for (int jr = w; jr < 64; jr += 4) {
      const int jj = j0 + jr;
      if (jj < n) xt[((size_t)b * n + jj) * C + c] = tile[lane][jr];
    }
  }
}

// --------------------------------------------------------------------------
// 5: range gather
//   TAPS == 8: column g = (dx, dy) in 0..3, off = dx r^2 + dy r.  A point of
//     cell q adds w[dx,dy,0] * x to voxel q + off and w[dx,dy,1] * x to voxel
//     q + off + 1; the column's source cells are [v0 - off - 1, v0 + TV - off).
//     (When a fraction is 0 the reference folds that corner onto the low cell
//     with weight exactly 0, trilinear_devox.cu:64-75, so both placements add
//     the same zeros.)
//   TAPS == 1: one range [v0, v0 + TV); a point of cell q adds x * vscale[q]
//     (or x) to voxel q.
// A tile's ranges are cut into chunks of kChunk sorted items.  Chunk t goes
// to part t / kWaves mod P (one block per part) and to wave t mod kWaves in
// it, so a crowded tile (the centre cells of a Gaussian cloud hold thousands
// of points at r = 8) is spread over up to P blocks.  Part 0 writes the tile
// to `out` (zeros if empty); parts 1.. that received chunks write partial
// tiles that seg_part_sum_kernel adds in part order.  No atomics.
// grid = (ceil(V/TV) * P, ceil(C/64), B), kWaves waves; LDS = kWaves partial tiles.
// --------------------------------------------------------------------------
constexpr int kWaves = 4;
constexpr int kChunk = 128;
constexpr int kInFlight = 16;  // row loads issued back to back per wave

template <int TAPS>
struct TileRanges {
  static constexpr int NR = TAPS == 8 ? 4 : 1;
  int rs[NR], re[NR], nch[NR];
  int total;
  // every lane of the wave ends with the same (wave-uniform) values
  __device__ __forceinline__ TileRanges(const int* sb, int v0, int TV, int V, int r, int lane) {
    int bnd = 0;
    if (lane < 2 * NR) {
      const int g = lane >> 1;
      int lo = v0, hi = v0 + TV;
      if constexpr (TAPS == 8) {
        const int off = (g >> 1) * r * r + (g & 1) * r;
        lo = v0 - off - 1;
        hi = v0 + TV - off;
      }
      bnd = sb[min(max((lane & 1) ? hi : lo, 0), V)];
    }
    total = 0;
#pragma unroll
    for (int g = 0; g < NR; ++g) {
      rs[g] = __builtin_amdgcn_readlane(bnd, 2 * g);
      re[g] = __builtin_amdgcn_readlane(bnd, 2 * g + 1);
      nch[g] = (re[g] - rs[g] + kChunk - 1) / kChunk;
      total += nch[g];
    }
  }
  __device__ __forceinline__ int parts_used(int P) const {
    return min(P, (total + kWaves - 1) / kWaves);
  }
};

template <int TAPS>
__device__ __forceinline__ void seg_flush(float* part, int slot0, int TV, int lane, float a0,
                                          float a1) {
  if ((unsigned)slot0 < (unsigned)TV) part[slot0 * 65 + lane] += a0;
  if constexpr (TAPS == 8) {
    if ((unsigned)(slot0 + 1) < (unsigned)TV) part[(slot0 + 1) * 65 + lane] += a1;
  }
}

__device__ __forceinline__ float rl_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

template <int TAPS>
__global__ void __launch_bounds__(kWaves * 64)
    seg_range_gather_kernel(const float* __restrict__ xt, const int* __restrict__ perm,
                            const int* __restrict__ skey, const float* __restrict__ tapw,
                            const int* __restrict__ start, const float* __restrict__ vscale,
                            int C, int n, int V, int r, int TV, int P, float* __restrict__ out,
                            float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float part[];  // [kWaves][TV][65]
  constexpr int NR = TileRanges<TAPS>::NR;
  const int b = blockIdx.z;
  const int tile = blockIdx.x / P, pp = blockIdx.x - tile * P;
  const int v0 = tile * TV, c0 = blockIdx.y * 64;
  // readfirstlane: tells the compiler the wave index is uniform, so the whole
  // chunk walk below stays scalar (no exec-mask branches, no vmcnt(0) stalls
  // between the row loads)
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int c = c0 + lane;
  const bool cok = c < C;
  const int* __restrict__ sb = start + (size_t)b * (V + 1);
  const TileRanges<TAPS> tr(sb, v0, TV, V, r, lane);
  if (pp > 0 && pp >= tr.parts_used(P)) return;  // block-uniform
  const int* __restrict__ pb = perm + (size_t)b * n;
  const int* __restrict__ kb = skey + (size_t)b * n;
  const float* __restrict__ xb = xt + (size_t)b * n * C + (cok ? c : 0);
  const float* __restrict__ wb = TAPS == 8 ? tapw + (size_t)b * 8 * n : nullptr;
  const float* __restrict__ vb = vscale != nullptr ? vscale + (size_t)b * V : nullptr;

  for (int e = threadIdx.x; e < kWaves * TV * 65; e += kWaves * 64) part[e] = 0.0f;
  __syncthreads();
  float* mypart = part + w * TV * 65;
  for (int t = pp * kWaves + w; t < tr.total; t += P * kWaves) {
    // chunk t -> (range g, chunk tt within it)
    int g = 0, tt = t;
#pragma unroll
    for (int q = 0; q < NR - 1; ++q) {
      if (g == q && tt >= tr.nch[q]) {
        tt -= tr.nch[q];
        g = q + 1;
      }
    }
    int s = 0, e = 0, off = 0;
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      if (g == q) {
        s = tr.rs[q] + tt * kChunk;
        e = min(tr.re[q], s + kChunk);
        if constexpr (TAPS == 8) off = (q >> 1) * r * r + (q & 1) * r;
      }
    }
    const int slot_base = off - v0;
    int cur = -1;
    float a0 = 0.0f, a1 = 0.0f, sc = 1.0f;
    for (int base = s; base < e; base += 64) {
      const int m = min(64, e - base);
      const bool act = lane < m;
      const int pv = act ? pb[base + lane] : 0;
      const int kv = act ? kb[base + lane] : -1;
      float w0v = 0.0f, w1v = 0.0f;
      if constexpr (TAPS == 8) {
        if (act) {  // taps k = 4dx + 2dy + dz = 2g + dz of wgts [b, 8, n]
          w0v = wb[(size_t)(2 * g) * n + pv];
          w1v = wb[(size_t)(2 * g + 1) * n + pv];
        }
      }
      for (int u0 = 0; u0 < m; u0 += kInFlight) {
        const int cnt = min(kInFlight, m - u0);
        float x[kInFlight];
        // unconditional: lanes >= m hold pv = 0, a valid row
#pragma unroll
        for (int q = 0; q < kInFlight; ++q)
          x[q] = xb[(size_t)__builtin_amdgcn_readlane(pv, u0 + q) * C];
#pragma unroll
        for (int q = 0; q < kInFlight; ++q) {
          if (q < cnt) {
            const int key = __builtin_amdgcn_readlane(kv, u0 + q);
            if (key != cur) {
              if (cur >= 0) seg_flush<TAPS>(mypart, cur + slot_base, TV, lane, a0, a1);
              cur = key;
              a0 = 0.0f;
              a1 = 0.0f;
              if constexpr (TAPS == 1) sc = vb != nullptr ? vb[key] : 1.0f;
            }
            if constexpr (TAPS == 8) {
              a0 = a0 + rl_f(w0v, u0 + q) * x[q];
              a1 = a1 + rl_f(w1v, u0 + q) * x[q];
            } else {
              a0 = vb != nullptr ? a0 + x[q] * sc : a0 + x[q];
            }
          }
        }
      }
    }
    if (cur >= 0) seg_flush<TAPS>(mypart, cur + slot_base, TV, lane, a0, a1);
  }
  __syncthreads();
  float* dst = pp == 0 ? out : partial + (size_t)(pp - 1) * gridDim.z * C * V;
  for (int e = threadIdx.x; e < 64 * TV; e += kWaves * 64) {
    const int cc = e / TV, vi = e - cc * TV;
    const int cg = c0 + cc, v = v0 + vi;
    if (cg < C && v < V) {
      float sum = part[vi * 65 + cc];
#pragma unroll
      for (int q = 1; q < kWaves; ++q) sum = sum + part[(q * TV + vi) * 65 + cc];
      dst[((size_t)b * C + cg) * V + v] = sum;
    }
  }
}

// out += partial[0 .. used-2] for the tiles that were split over several parts.
// grid = (ceil(V/TV), ceil(C/64), B), 256 threads.
template <int TAPS>
__global__ void __launch_bounds__(256)
    seg_part_sum_kernel(const int* __restrict__ start, const float* __restrict__ partial, int C,
                        int V, int r, int TV, int P, float* __restrict__ out) {
  const int b = blockIdx.z;
  const int v0 = blockIdx.x * TV, c0 = blockIdx.y * 64;
  const TileRanges<TAPS> tr(start + (size_t)b * (V + 1), v0, TV, V, r, threadIdx.x & 63);
  const int used = tr.parts_used(P);
  if (used <= 1) return;
  const size_t pstride = (size_t)gridDim.z * C * V;
  for (int e = threadIdx.x; e < 64 * TV; e += 256) {
    const int cc = e / TV, vi = e - cc * TV;
    const int cg = c0 + cc, v = v0 + vi;
    if (cg < C && v < V) {
      const size_t o = ((size_t)b * C + cg) * V + v;
      float sum = out[o];
      for (int q = 0; q < used - 1; ++q) sum = sum + partial[q * pstride + o];
      out[o] = sum;
    }
  }
}

}  // namespace

// --------------------------------------------------------------------------
// host driver
// --------------------------------------------------------------------------
inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

inline int seg_tile_voxels(int V) { return V >= 4096 ? 32 : 16; }
// parts per tile: small grids (coarse voxel grids hold the dense cells) split more
inline int seg_parts(int V) { return V <= 4096 ? 16 : 4; }

struct SegWs {
  int* start;      // B*(V+1)
  float* vinv;     // B*V (per-voxel 1/cnt)
  int* perm;       // B*n
  int* skey;       // B*n
  float* xt;       // B*n*C
  float* partial;  // (P-1)*B*C*V
};

inline size_t seg_ws_bytes(int B, int C, int n, int V, int taps) {
  size_t s = align256((size_t)B * (V + 1) * 4);
  s += align256((size_t)B * V * 4);
  s += 2 * align256((size_t)B * n * 4);
  s += align256((size_t)B * n * std::max(C, 1) * 4);
  s += align256((size_t)(seg_parts(V) - 1) * B * C * V * 4);
  return s;
}

inline SegWs seg_ws_carve(void* ws, int B, int C, int n, int V, int taps) {
  char* p = (char*)ws;
  auto take = [&p](size_t bytes) {
    char* q = p;
    p += align256(bytes);
    return q;
  };
  SegWs w;
  w.start = (int*)take((size_t)B * (V + 1) * 4);
  w.vinv = (float*)take((size_t)B * V * 4);
  w.perm = (int*)take((size_t)B * n * 4);
  w.skey = (int*)take((size_t)B * n * 4);
  w.xt = (float*)take((size_t)B * n * std::max(C, 1) * 4);
  w.partial = (float*)take((size_t)(seg_parts(V) - 1) * B * C * V * 4);
  return w;
}

// out[b, c, v] = sum over items i whose key (+ stencil offset) is v of the tap term.
//   key: ints at key + b*key_bstride (first n used); cnt_out: [b, V] counts are
//   written there when non-null; avg: scale by 1/cnt[v] (average pooling);
//   tapw: [b, 8, n] trilinear weights (TAPS == 8).
template <int TAPS>
inline int seg_scatter(const float* in, const int* key, long long key_bstride, bool avg,
                       const float* tapw, int r, int B, int C, int n, int V, int* cnt_out,
                       float* out, void* ws, hipStream_t st, const char* what) {
  if (B == 0 || V == 0) return PCFM_OK;
  SegWs w = seg_ws_carve(ws, B, C, n, V, TAPS);
  const size_t sort_lds = (size_t)std::min(V, kSortKeys) * sizeof(int);
  int e = allow_big_lds((const void*)seg_sort_kernel);
  if (e) return e;
  hipLaunchKernelGGL(seg_sort_kernel, dim3(B), dim3(1024), sort_lds, st, key, key_bstride, n, V,
                     w.start, cnt_out, avg ? w.vinv : nullptr, w.perm, w.skey);
  if (C == 0) return check_launch(what);
  if (n > 0)
    hipLaunchKernelGGL(seg_transpose_kernel, dim3(ceil_div(n, 64), ceil_div(C, 64), B),
                       dim3(256), 0, st, in, C, n, w.xt);
  const int TV = seg_tile_voxels(V), P = seg_parts(V);
  const int tiles = ceil_div(V, TV);
  const size_t lds = (size_t)kWaves * TV * 65 * sizeof(float);
  hipLaunchKernelGGL(seg_range_gather_kernel<TAPS>, dim3(tiles * P, ceil_div(C, 64), B),
                     dim3(kWaves * 64), lds, st, w.xt, w.perm, w.skey, tapw, w.start,
                     avg ? w.vinv : nullptr, C, n, V, r, TV, P, out, w.partial);
  if (P > 1)
    hipLaunchKernelGGL(seg_part_sum_kernel<TAPS>, dim3(tiles, ceil_div(C, 64), B), dim3(256), 0,
                       st, w.start, w.partial, C, V, r, TV, P, out);
  return check_launch(what);
}

}  // namespace pcfm
