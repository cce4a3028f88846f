// Sorted, atomic-free scatter ("segment sum") for the PVConv path.
//
// The reference scatters with one float atomic per (item, channel, tap)
// (vox.cu:48-72, trilinear_devox.cu:119-162, grouping.cu:58-77).  On MI355X a
// device-scope float atomic executes at the memory side (~1.3 TB/s of added
// bytes chip-wide) and an LDS float atomic costs ~200 cycles per wave
// instruction (measured, tools/voxel_probe.py), so the scatters are recast as
// gathers over items sorted by their target cell:
//
//   1. seg_sort     stable counting sort, up to 16 blocks per batch element,
//                   per-wave histograms in LDS: start[b, 0..V] and rank[b, i]
//                   (sorted position of item i, item order kept inside a key)
//   2. seg_units    tiles of kTV voxels -> balanced work units (device-built)
//   3. seg_rows     xs[b, rank[i], :] = in[b, :, i]: channels-last rows in
//                   SORTED order, plus the item's key and tap weights at the
//                   same sorted position (the main loop then streams
//                   contiguous memory and chases no index)
//   4. seg_unit_gather  output-stationary, lanes = 64 channels: one wave per
//                   unit, register run-accumulators per tap flushed into a
//                   wave-private LDS tile, coalesced tile store
//   5. seg_part_sum adds the partial tiles of tiles split over several units
//
// Used by avg_voxelize forward (key = voxel, term = feat * (1/cnt)),
// trilinear devoxelize backward (key = base cell inds[b,0,:], term = wgt * g
// for the 8 corners) and grouping backward (key = neighbour index, term = g).
// The sort is stable (items inside one key keep their index order) and every
// float sum runs in a fixed order, so the scatters are deterministic -- unlike
// the reference's float atomics.
#pragma once

#include <algorithm>
#include <cstdlib>

#include "pcfm_common.hpp"

namespace pcfm {

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Key shift of a scatter's sort.  The trilinear stencil (TAPS == 8) reaches
// from a point's base cell q to q + dx r^2 + dy r + dz (dx, dy, dz in {0, 1}),
// so a point whose base cell lies below the volume (coordinates outside
// [0, r - 1]: a negative linear index) can still have corners inside it, and
// the forward reads them (trilinear_devox.cu:64-105).  Its sort key is q + koff
// with koff = r^2 + r + 1, over V + koff keys: every point with a corner in
// [0, V) is kept.  (Keys >= V have every corner >= V: dropped.)
inline int seg_koff(int V, int taps) {
  if (taps != 8) return 0;
  int r = 1;
  while ((long long)r * r * r < V) ++r;
  return r * r + r + 1;
}
inline int seg_keys(int V, int taps) { return V + seg_koff(V, taps); }

namespace {  // kernels get internal linkage: this header is included by several .hip files

// --------------------------------------------------------------------------
// 1: STABLE counting sort by key.  Block (p, b) owns the key range [p, p+1) *
// span of batch element b (grid = (P, B), 1024 threads = 16 waves): every block
// reads all n keys of its batch element (L2-resident, 80 KB at N = 20000) and
// counts the keys BELOW its range itself -- its base in the sorted order, so
// the P blocks never wait for each other.  Keys are handled in chunks of
// kSortChunk (a wider range takes several passes).  Wave w owns the item
// segment [w n / 16, (w+1) n / 16) and keeps its own per-key counts in LDS:
//   A  count:  per-wave histograms of the chunk (LDS int atomics; counts are
//              order-free);
//   B  scan:   per key the exclusive prefix over keys (-> start) and over the
//              waves (-> each wave's first rank of that key);
//   C  rank:   each wave walks its segment in index order, 64 items per step;
//              the items of one step that share a key are ranked by lane, and
//              only the owning wave advances its counters -- so
//              rank[i] = start[key_i] + #{j < i : key_j = key_i}:
//              the order inside a key is the item order, independent of
//              scheduling.  Every float sum downstream (unit gathers, partial
//              tiles) then runs in a fixed order: the scatters are
//              deterministic (the reference's float atomics are not).
//   start[b, 0..V]  exclusive prefix of the counts (start[b, V] = total)
//   cnt_out[b, v]   the counts (optional: the voxelization's `cnt` output)
//   vinv[b, v]      (float)(1.0 / (double)cnt) (optional, vox.cu:66)
//   rank[b, i]      start[key_i] + rank within the key; -1 when the key is
//                   outside [0, V) (the item contributes nothing)
// Keys are key[i] + koff (seg_koff; V then counts the shifted key range and
// cnt_out / vinv are not asked for).
// --------------------------------------------------------------------------
constexpr int kSortWaves = 16;
constexpr int kSortChunk = 2048;   // keys per pass: 16 waves x 2048 ints = 128 KiB of LDS
constexpr int kSortBatch = 8;      // 64-item key loads per wave in flight
#ifndef PCFM_SORT_MIN_SPAN
#define PCFM_SORT_MIN_SPAN 32
#endif
constexpr int kSortMinSpan = PCFM_SORT_MIN_SPAN;  // keys per block at least
constexpr int kSortMaxParts = 16;  // blocks per batch element at most

inline int seg_sort_parts(int V) {
  return std::max(1, std::min(kSortMaxParts, V / kSortMinSpan));
}
inline int seg_sort_span(int V) { return (V + seg_sort_parts(V) - 1) / seg_sort_parts(V); }
inline size_t seg_sort_lds(int V) {
  return (size_t)kSortWaves * std::min(seg_sort_span(V), kSortChunk) * sizeof(int);
}

__global__ void __launch_bounds__(1024)
    seg_sort_kernel(const int* __restrict__ key, long long key_bstride, int n, int V, int span,
                    int* __restrict__ start, int* __restrict__ cnt_out, float* __restrict__ vinv,
                    int* __restrict__ rank, int koff = 0) {
  extern __shared__ int hw[];  // [kSortWaves][len]
  __shared__ int wsum[kSortWaves];
  const int p = blockIdx.x, b = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int* __restrict__ kb = key + (size_t)b * key_bstride;
  int* __restrict__ sb = start + (size_t)b * (V + 1);
  int* __restrict__ rb = rank + (size_t)b * n;
  const int pk0 = min(V, p * span), pk1 = min(V, pk0 + span);
  const int i_lo = (int)((long long)n * w / kSortWaves);
  const int i_hi = (int)((long long)n * (w + 1) / kSortWaves);
  int carry = 0;
  for (int k0 = pk0; k0 < pk1; k0 += kSortChunk) {
    const int len = min(kSortChunk, pk1 - k0);
    for (int e = t; e < kSortWaves * len; e += 1024) hw[e] = 0;
    __syncthreads();
    // A: per-wave counts (+ the keys below the block's range: its base)
    int* hmine = hw + w * len;
    int below = 0;
    for (int i0 = i_lo; i0 < i_hi; i0 += 64 * kSortBatch) {
      int kk[kSortBatch];  // keys first (independent loads in flight), then the atomics
#pragma unroll
      for (int q = 0; q < kSortBatch; ++q) {
        const int i = i0 + 64 * q + lane;
        kk[q] = i < i_hi ? kb[i] + koff : -1;
      }
#pragma unroll
      for (int q = 0; q < kSortBatch; ++q) {
#ifndef PCFM_SORT_SKIP_A
        if ((unsigned)(kk[q] - k0) < (unsigned)len) atomicAdd(hmine + (kk[q] - k0), 1);
#endif
        below += (k0 == pk0 && (unsigned)kk[q] < (unsigned)pk0) ? 1 : 0;
      }
    }
    if (k0 == pk0) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) below += __shfl_xor(below, o, 64);
      if (lane == 0) wsum[w] = below;
    }
    __syncthreads();
    if (k0 == pk0) {
#pragma unroll
      for (int g = 0; g < kSortWaves; ++g) carry += wsum[g];
    }
    __syncthreads();
    // B: wave w owns the 64-aligned key segment [lo, hi)
    const int seg = ((len + kSortWaves - 1) / kSortWaves + 63) & ~63;
    const int lo = min(len, w * seg), hi = min(len, lo + seg);
    int part = 0;
    for (int e = lo + lane; e < hi; e += 64) {
#pragma unroll
      for (int g = 0; g < kSortWaves; ++g) part += hw[g * len + e];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    if (lane == 0) wsum[w] = part;
    __syncthreads();
    int run = carry, total = 0;
#pragma unroll
    for (int g = 0; g < kSortWaves; ++g) {
      const int x = wsum[g];
      run += g < w ? x : 0;
      total += x;
    }
    for (int e0 = lo; e0 < hi; e0 += 64) {
      const int e = e0 + lane;
      int c = 0;
      if (e < hi) {
#pragma unroll
        for (int g = 0; g < kSortWaves; ++g) c += hw[g * len + e];
      }
      int x = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (e < hi) {
        int pos = run + x - c;
        sb[k0 + e] = pos;
        if (cnt_out != nullptr) cnt_out[(size_t)b * V + k0 + e] = c;
        if (vinv != nullptr) vinv[(size_t)b * V + k0 + e] = c > 0 ? (float)(1.0 / (double)c) : 0.0f;
#pragma unroll
        for (int g = 0; g < kSortWaves; ++g) {  // first rank of key e for wave g
          const int cg = hw[g * len + e];
          hw[g * len + e] = pos;
          pos += cg;
        }
      }
      run += __shfl(x, 63, 64);
    }
    __syncthreads();
    // C: ranks in item order (only wave w touches its counters)
    const int nbits = len > 1 ? 32 - __clz(len - 1) : 0;
    for (int j0 = i_lo; j0 < i_hi; j0 += 64 * kSortBatch) {
      int kq[kSortBatch];
#pragma unroll
      for (int q = 0; q < kSortBatch; ++q) {
        const int i = j0 + 64 * q + lane;
        kq[q] = i < i_hi ? kb[i] + koff : -1;
      }
#pragma unroll
      for (int q = 0; q < kSortBatch; ++q) {
        const int i = j0 + 64 * q + lane;
        const int k = kq[q];
        const bool inr = i < i_hi && (unsigned)(k - k0) < (unsigned)len;
        const unsigned long long act = __ballot(inr);
        if (act) {
          // lanes of this step with the same key, by bit-plane ballots of the
          // chunk-local key (nbits of them); the lane's rank among them is the
          // count of lower lanes (mbcnt), and the LAST lane of each group alone
          // advances the wave's counter: no lane-order-dependent atomics
          const unsigned kl = inr ? (unsigned)(k - k0) : 0u;
          unsigned long long same = act;
          for (int bit = 0; bit < nbits; ++bit) {
            const bool on = (kl >> bit) & 1u;
            const unsigned long long m = __ballot(on);
            same &= on ? m : ~m;
          }
          if (inr) {
            const int within = __builtin_amdgcn_mbcnt_hi(
                (unsigned)(same >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)same, 0u));
            const int base = hmine[kl];
            rb[i] = base + within;
            if ((same >> lane) >> 1 == 0ull) hmine[kl] = base + __popcll(same);
          }
        }
        if (p == 0 && k0 == pk0 && i < i_hi && (unsigned)k >= (unsigned)V) rb[i] = -1;
      }
    }
    carry += total;
    __syncthreads();
  }
  if (t == 0 && pk1 == V && (pk0 < V || p == 0)) sb[V] = carry;
}

// --------------------------------------------------------------------------
// 3: rows in sorted order.  xs[b, rank[i], c] = in[b, c, i] (64 x 64 LDS
// tile: 256-B coalesced reads along i, one 256-B row segment per store).
// Blocks of channel group 0 also write skey[b, rank[i]] = key[i] and, for the
// trilinear stencil, ws8[b, rank[i], k] = tapw[b, k, i].
// grid = (ceil(n/64), ceil(C/64), B), 256 threads.
// --------------------------------------------------------------------------
#ifndef PCFM_ROWS_ITEMS
#define PCFM_ROWS_ITEMS 64
#endif
constexpr int kRowsItems = PCFM_ROWS_ITEMS;  // items per block (64 or 128)
#ifndef PCFM_ROWS_ALLC
#define PCFM_ROWS_ALLC 1
#endif
// 64-item blocks loop over all channel groups (grid.y = 1)
constexpr bool kRowsAllC = PCFM_ROWS_ALLC && kRowsItems == 64;

__global__ void __launch_bounds__(256)
    seg_rows_kernel(const float* __restrict__ in, const int* __restrict__ rank,
                    const int* __restrict__ key, long long key_bstride,
                    const float* __restrict__ tapw, int C, int n, float* __restrict__ xs,
                    int* __restrict__ skey, float* __restrict__ ws8) {
  __shared__ float tile[64][kRowsItems + 1];
  __shared__ int rk[kRowsItems];
  const int b = blockIdx.z;
  const int j0 = blockIdx.x * kRowsItems, c0 = blockIdx.y * 64;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int jj = threadIdx.x; jj < kRowsItems; jj += 256) {
    const int j = j0 + jj;
    const int r = j < n ? rank[(size_t)b * n + j] : -1;
    rk[jj] = r;
    if (skey != nullptr && blockIdx.y == 0 && r >= 0) {
      const size_t o = (size_t)b * n + r;
      skey[o] = key[(size_t)b * key_bstride + j];
      if (tapw != nullptr) {
        const float* tb = tapw + (size_t)b * 8 * n + j;
        float4* d = reinterpret_cast<float4*>(ws8 + o * 8);
        d[0] = make_float4(tb[0], tb[(size_t)n], tb[(size_t)2 * n], tb[(size_t)3 * n]);
        d[1] = make_float4(tb[(size_t)4 * n], tb[(size_t)5 * n], tb[(size_t)6 * n],
                           tb[(size_t)7 * n]);
      }
    }
  }
  if constexpr (kRowsItems == 128) {
    // one wave reads 128 items of a channel row as float2 (512 B)
    const int j = j0 + 2 * lane;
    const bool vec = (n & 1) == 0 && j + 1 < n;
    for (int cc = w; cc < 64; cc += 4) {
      const int c = c0 + cc;
      float2 v = make_float2(0.0f, 0.0f);
      if (c < C) {
        const float* src = in + ((size_t)b * C + c) * n + j;
        if (vec) {
          v = *reinterpret_cast<const float2*>(src);
        } else {
          if (j < n) v.x = src[0];
          if (j + 1 < n) v.y = src[1];
        }
      }
      tile[cc][2 * lane] = v.x;
      tile[cc][2 * lane + 1] = v.y;
    }
  } else if (kRowsAllC) {
    // every channel group of the block's items in turn: an item's whole row
    // (C floats) is written by one wave within a few hundred cycles, instead of
    // in C/64 pieces by blocks dispatched far apart
    const int j = j0 + lane;
    __syncthreads();
    for (int g0 = 0; g0 < C; g0 += 64) {
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int c = g0 + w + 4 * q;
        v[q] = (c < C && j < n) ? in[((size_t)b * C + c) * n + j] : 0.0f;
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) tile[w + 4 * q][lane] = v[q];
      __syncthreads();
      const int c = g0 + lane;
      if (c < C) {
        for (int jr = w; jr < kRowsItems; jr += 4) {
          const int r = rk[jr];
          if (r >= 0) xs[((size_t)b * n + r) * C + c] = tile[lane][jr];
        }
      }
      __syncthreads();
    }
    return;
  } else {
    const int j = j0 + lane;
    for (int cc = w; cc < 64; cc += 4) {
      const int c = c0 + cc;
      tile[cc][lane] = (c < C && j < n) ? in[((size_t)b * C + c) * n + j] : 0.0f;
    }
  }
  __syncthreads();
  const int c = c0 + lane;
  if (c < C) {
    for (int jr = w; jr < kRowsItems; jr += 4) {
      const int r = rk[jr];
      if (r >= 0) xs[((size_t)b * n + r) * C + c] = tile[lane][jr];
    }
  }
}

// Plan-side part of step 3: the sorted keys (skey[b, rank[i]] = key[i]) and,
// for the trilinear stencil, the sorted tap weights (ws8[b, rank[i], k] =
// tapw[b, k, i]) -- built once per plan, reused by every scatter over it.
// grid = (ceil(n / 256), B).
__global__ void __launch_bounds__(256)
    seg_plan_rows_kernel(const int* __restrict__ rank, const int* __restrict__ key,
                         long long key_bstride, const float* __restrict__ tapw, int n,
                         int* __restrict__ skey, float* __restrict__ ws8) {
  const int b = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int r = rank[(size_t)b * n + i];
  if (r < 0) return;
  const size_t o = (size_t)b * n + r;
  skey[o] = key[(size_t)b * key_bstride + i];
  if (tapw != nullptr) {
    const float* tb = tapw + (size_t)b * 8 * n + i;
    float4* d = reinterpret_cast<float4*>(ws8 + o * 8);
    d[0] = make_float4(tb[0], tb[(size_t)n], tb[(size_t)2 * n], tb[(size_t)3 * n]);
    d[1] = make_float4(tb[(size_t)4 * n], tb[(size_t)5 * n], tb[(size_t)6 * n], tb[(size_t)7 * n]);
  }
}

// --------------------------------------------------------------------------
// 2 + 4 + 5: units, unit gather, partial sums.
//   The output is cut into tiles of kTV consecutive voxels.  Items feeding a
//   tile form NR contiguous sorted ranges:
//   TAPS == 8: column g = (dx, dy) in 0..3, off = dx r^2 + dy r.  A point of
//     cell q adds w[dx,dy,0] * x to voxel q + off and w[dx,dy,1] * x to voxel
//     q + off + 1; the column's source cells are [v0 - off - 1, v0 + kTV - off).
//     (When a fraction is 0 the reference folds that corner onto the low cell
//     with weight exactly 0, trilinear_devox.cu:64-75, so both placements add
//     the same zeros.)
//   TAPS == 1: one range [v0, v0 + kTV); a point of cell q adds x * vscale[q]
//     (or x) to voxel q.
//   A tile with T items (its ranges concatenated) becomes P = ceil(T / kItems)
//   work units of ~T/P items (at least one, so empty tiles are written as
//   zeros).  ONE wave runs a unit: per 64 items one load round fetches the
//   sorted keys and tap weights, the 16 next feature rows (consecutive rows
//   of xs) are loaded back to back, a register accumulator per tap runs over
//   equal target voxels and is added into the wave's private LDS tile when the
//   voxel changes.  Unit 0 of a tile writes the tile to `out`; units 1.. of a
//   crowded tile write partial tiles that seg_part_sum_kernel adds in unit
//   order.  Waves never wait for each other and nothing is atomic.
// --------------------------------------------------------------------------
#ifndef PCFM_SEG_XCD
#define PCFM_SEG_XCD 1
#endif
#ifndef PCFM_KTV
#define PCFM_KTV 16
#endif
constexpr int kTV = PCFM_KTV;    // voxels per tile
#ifndef PCFM_SEG_ITEMS
#define PCFM_SEG_ITEMS 256
#endif
constexpr int kItems = PCFM_SEG_ITEMS;  // target items per work unit
constexpr int kInFlight = 16;    // feature-row loads issued back to back per wave
constexpr int kUnitWaves = 4;    // waves (independent units) per block

template <int TAPS>
constexpr int seg_ranges() { return TAPS == 8 ? 4 : 1; }

// seg_koff on the device
template <int TAPS>
__device__ __forceinline__ int seg_koff_r(int r) { return TAPS == 8 ? r * r + r + 1 : 0; }

// Range g of tile v0: lanes 2g / 2g+1 return the sorted positions [lo, hi).
// sb: the batch element's start row over the V + koff shifted keys.
template <int TAPS>
__device__ __forceinline__ int seg_range_bound(const int* sb, int v0, int V, int r, int lane) {
  int bnd = 0;
  if (lane < 2 * seg_ranges<TAPS>()) {
    const int g = lane >> 1;
    const int koff = seg_koff_r<TAPS>(r);
    int lo = v0, hi = v0 + kTV;
    if constexpr (TAPS == 8) {
      const int off = (g >> 1) * r * r + (g & 1) * r;
      lo = v0 - off - 1;
      hi = v0 + kTV - off;
    }
    bnd = sb[min(max(((lane & 1) ? hi : lo) + koff, 0), V + koff)];
  }
  return bnd;
}

// Work-unit list, one block (1024 threads) per batch element:
//   units[b, u] = {tile, part, parts, items}, tinfo[b, tile] = {parts, first
//   partial slot}, nunits[b].
template <int TAPS>
__global__ void __launch_bounds__(1024)
    seg_units_kernel(const int* __restrict__ start, int V, int r, int tiles, int umax,
                     int4* __restrict__ units, int2* __restrict__ tinfo, int* __restrict__ nunits) {
  __shared__ int wsum[16];
  constexpr int NR = seg_ranges<TAPS>();
  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int koff = seg_koff_r<TAPS>(r), VK = V + koff;
  const int* sb = start + (size_t)b * (VK + 1);
  int carry = 0;
  for (int t0 = 0; t0 < tiles; t0 += 1024) {
    const int tile = t0 + t;
    int T = 0, P = 0;
    if (tile < tiles) {
      const int v0 = tile * kTV;
#pragma unroll
      for (int g = 0; g < NR; ++g) {
        int lo = v0, hi = v0 + kTV;
        if constexpr (TAPS == 8) {
          const int off = (g >> 1) * r * r + (g & 1) * r;
          lo = v0 - off - 1;
          hi = v0 + kTV - off;
        }
        T += sb[min(max(hi + koff, 0), VK)] - sb[min(max(lo + koff, 0), VK)];
      }
      P = max(1, (T + kItems - 1) / kItems);
    }
    int x = P;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int ofs = carry, total = 0;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int s = wsum[g];
      ofs += g < w ? s : 0;
      total += s;
    }
    const int U = ofs + x - P;
    if (tile < tiles) {
      tinfo[(size_t)b * tiles + tile] = make_int2(P, U - tile);
      for (int p = 0; p < P && U + p < umax; ++p)
        units[(size_t)b * umax + U + p] = make_int4(tile, p, P, T);
    }
    carry += total;
    __syncthreads();
  }
  if (t == 0) nunits[b] = min(carry, umax);
}

// Run bookkeeping: when a run of equal target voxels starts, the tile's
// current partials for its slots are READ (p0, p1) without waiting; when it
// ends, p + acc is written back.  The LDS read latency then hides behind the
// run's row loads instead of stalling every flush (LDS ops of one wave stay in
// order, so a read of slot s+1 after the previous run's write of s+1 sees it).
template <int TAPS>
__device__ __forceinline__ void seg_run_end(float* tl, int slot, int lane, float p0, float p1,
                                            float a0, float a1) {
  if ((unsigned)slot < (unsigned)kTV) tl[slot * 65 + lane] = p0 + a0;
  if constexpr (TAPS == 8) {
    if ((unsigned)(slot + 1) < (unsigned)kTV) tl[(slot + 1) * 65 + lane] = p1 + a1;
  }
}
template <int TAPS>
__device__ __forceinline__ void seg_run_begin(const float* tl, int slot, int lane, float& p0,
                                              float& p1) {
  p0 = (unsigned)slot < (unsigned)kTV ? tl[slot * 65 + lane] : 0.0f;
  if constexpr (TAPS == 8) p1 = (unsigned)(slot + 1) < (unsigned)kTV ? tl[(slot + 1) * 65 + lane] : 0.0f;
}

__device__ __forceinline__ float rl_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// grid = (ceil(umax / kUnitWaves), ceil(C/64), B), kUnitWaves * 64 threads.
template <int TAPS>
__global__ void __launch_bounds__(kUnitWaves * 64)
    seg_unit_gather_kernel(const float* __restrict__ xs, const int* __restrict__ skey,
                           const float* __restrict__ ws8, const int* __restrict__ start,
                           const float* __restrict__ vscale, const int4* __restrict__ units,
                           const int* __restrict__ nunits, int C, int n, int V, int r, int umax,
                           int slots, float* __restrict__ out, float* __restrict__ partial) {
  __shared__ float lds[kUnitWaves][kTV * 65];
  constexpr int NR = seg_ranges<TAPS>();
#if PCFM_SEG_XCD
  // XCD-contiguous deal: consecutive blocks in dispatch order go round-robin
  // to the 8 XCDs; give each XCD a contiguous run of (unit block, channel
  // group, batch) so a row's re-reads by the other stencil columns hit its L2
  int bx, by, bz;
  {
    const int gx = (int)gridDim.x, gy = (int)gridDim.y;
    const int tot = gx * gy * (int)gridDim.z;
    int id = (int)(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z));
    const int q = tot / 8, rr = tot % 8, xcd = id % 8;
    id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + id / 8;
    bx = id % gx;
    by = (id / gx) % gy;
    bz = id / (gx * gy);
  }
  const int b = bz, c0 = by * 64;
#else
  const int bx = blockIdx.x;
  const int b = blockIdx.z, c0 = blockIdx.y * 64;
#endif
  // readfirstlane: the wave index is uniform, so the whole walk stays scalar
  // (no exec-mask branches, no vmcnt(0) stalls between the row loads)
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  // (XCD-contiguous deal vs dispatch order, tools/scatter_ab.py on MI355X:
  // devox backward 0.183 -> 0.175 ms C128 R32, 0.235 -> 0.215 C256 R16,
  // 0.224 -> 0.207 C256 R8; the voxelize forward unchanged)
  const int nu = nunits[b];
  const int u = bx * kUnitWaves + w;
  if (u >= nu) return;  // wave-uniform; no block barrier below
  const int4 un = units[(size_t)b * umax + u];
  const int tile = un.x, part = un.y, parts = un.z, T = un.w;
  const int v0 = tile * kTV;
  const int c = c0 + lane;
  const bool cok = c < C;
  const int* __restrict__ sb = start + (size_t)b * (V + seg_koff_r<TAPS>(r) + 1);
  const int* __restrict__ kb = skey + (size_t)b * n;
  const float* __restrict__ xb = xs + (size_t)b * n * C + (cok ? c : 0);
  const float* __restrict__ wb = TAPS == 8 ? ws8 + (size_t)b * n * 8 : nullptr;

  const int bnd = seg_range_bound<TAPS>(sb, v0, V, r, lane);
  int rs[NR], pre[NR + 1];
  pre[0] = 0;
#pragma unroll
  for (int g = 0; g < NR; ++g) {
    rs[g] = __builtin_amdgcn_readlane(bnd, 2 * g);
    pre[g + 1] = pre[g] + __builtin_amdgcn_readlane(bnd, 2 * g + 1) - rs[g];
  }
  const int i0 = (int)((long long)T * part / parts);
  const int i1 = (int)((long long)T * (part + 1) / parts);
  float vs = 0.0f;  // TAPS == 1 average pool: lane l holds 1/cnt of voxel v0 + l
  if (TAPS == 1 && vscale != nullptr && lane < kTV && v0 + lane < V)
    vs = vscale[(size_t)b * V + v0 + lane];

  float* tl = lds[w];
  for (int e = lane; e < kTV * 65; e += 64) tl[e] = 0.0f;

  int cur = -1000;
  float a0 = 0.0f, a1 = 0.0f, p0 = 0.0f, p1 = 0.0f, sc = 1.0f;
  for (int base = i0; base < i1; base += 64) {
    const int m = min(64, i1 - base);
    const int it = base + lane;
    int pos = 0, sl = -1000;
    float w0v = 0.0f, w1v = 0.0f;
    if (lane < m) {
      int g = 0;
#pragma unroll
      for (int q = 1; q < NR; ++q) g += it >= pre[q] ? 1 : 0;
      int off = 0, gs = 0;
#pragma unroll
      for (int q = 0; q < NR; ++q)
        if (g == q) {
          pos = rs[q] + it - pre[q];
          off = TAPS == 8 ? (q >> 1) * r * r + (q & 1) * r : 0;
          gs = q;
        }
      sl = kb[pos] + off - v0;
      if constexpr (TAPS == 8) {  // taps k = 4dx + 2dy + dz = 2g + dz
        const float2 ww = *reinterpret_cast<const float2*>(wb + (size_t)pos * 8 + 2 * gs);
        w0v = ww.x;
        w1v = ww.y;
      }
    }
    for (int u0 = 0; u0 < m; u0 += kInFlight) {
      float x[kInFlight];
      // unconditional: lanes >= m hold pos = 0, a valid row
#pragma unroll
      for (int q = 0; q < kInFlight; ++q)
        x[q] = xb[(size_t)__builtin_amdgcn_readlane(pos, u0 + q) * C];
      const int cnt = min(kInFlight, m - u0);
#pragma unroll
      for (int q = 0; q < kInFlight; ++q) {
        if (q < cnt) {
          const int slot = __builtin_amdgcn_readlane(sl, u0 + q);
          if (slot != cur) {
            seg_run_end<TAPS>(tl, cur, lane, p0, p1, a0, a1);
            cur = slot;
            seg_run_begin<TAPS>(tl, cur, lane, p0, p1);
            a0 = 0.0f;
            a1 = 0.0f;
            if constexpr (TAPS == 1) sc = rl_f(vs, slot & 63);
          }
          if constexpr (TAPS == 8) {
            a0 = a0 + rl_f(w0v, u0 + q) * x[q];
            a1 = a1 + rl_f(w1v, u0 + q) * x[q];
          } else {
            a0 = vscale != nullptr ? a0 + x[q] * sc : a0 + x[q];
          }
        }
      }
    }
  }
  seg_run_end<TAPS>(tl, cur, lane, p0, p1, a0, a1);

  // tile -> global, 2 channels x 32 voxels (2 x 128 B) per store instruction
  float* dst;
  size_t cstride, bofs;
  if (part == 0) {
    dst = out + v0;
    cstride = (size_t)V;
    bofs = (size_t)b * C * V;
  } else {  // partial slot: units of tiles before this one beyond their first, + part - 1
    dst = partial;
    cstride = (size_t)kTV;
    bofs = ((size_t)b * slots + (size_t)(u - tile - 1)) * C * kTV;
  }
  const int vi = lane & (kTV - 1), ch = lane / kTV;
  const bool vok = part > 0 || v0 + vi < V;
#pragma unroll 4
  for (int k = 0; k < 64; k += 64 / kTV) {
    const int cc = k + ch, cg = c0 + cc;
    if (cg < C && vok) dst[bofs + (size_t)cg * cstride + vi] = tl[vi * 65 + cc];
  }
}

// out += partial tiles 1 .. P-1 of every crowded tile, in unit order.
// grid = (tiles, ceil(C/64), B), 256 threads.
__global__ void __launch_bounds__(256)
    seg_part_sum_kernel(const int2* __restrict__ tinfo, const float* __restrict__ partial,
                        int C, int V, int tiles, int slots, float* __restrict__ out) {
  const int b = blockIdx.z, tile = blockIdx.x, c0 = blockIdx.y * 64;
  const int2 ti = tinfo[(size_t)b * tiles + tile];
  if (ti.x <= 1) return;
  const int v0 = tile * kTV;
  for (int e = threadIdx.x; e < 64 * kTV; e += 256) {
    const int cc = e / kTV, vi = e - cc * kTV;
    const int cg = c0 + cc, v = v0 + vi;
    if (cg < C && v < V) {
      const size_t o = ((size_t)b * C + cg) * V + v;
      const float* pp = partial + (((size_t)b * slots + ti.y) * C + cg) * kTV + vi;
      const size_t ps = (size_t)C * kTV;  // one partial tile
      float sum = out[o];
      int p = 0;
      for (; p + 8 <= ti.x - 1; p += 8) {  // 8 independent loads in flight, summed in order
        float x[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] = pp[(size_t)(p + q) * ps];
#pragma unroll
        for (int q = 0; q < 8; ++q) sum = sum + x[q];
      }
      for (; p < ti.x - 1; ++p) sum = sum + pp[(size_t)p * ps];
      out[o] = sum;
    }
  }
}

}  // namespace

// --------------------------------------------------------------------------
// host driver
// --------------------------------------------------------------------------

// Upper bound of work units per batch element: one per tile plus one per
// kItems of range items (an item lies in at most 2 tiles per stencil column).
inline int seg_tiles(int V) { return (V + kTV - 1) / kTV; }

// (Round 5 built 2 x 2-column tiles for the trilinear scatter -- a row read by
// 2.25 tiles instead of 4 -- bit-identical to the column tiles and slower:
// the gather is issue-bound; profiles/r05_ab_devox_quad.jsonl.  Removed in
// round 6.)
inline int seg_umax(int n, int V, int taps) {
  return seg_tiles(V) + (int)(((long long)(taps == 8 ? 8 : 1) * n + kItems - 1) / kItems) + 1;
}

// A scatter = plan (sort the items by key, cut the output into work units,
// gather the sorted keys / tap weights) + apply (channels-last rows, unit
// gather, partial sums).  The plan depends only on the keys, so scatters over
// the same points share it (include/pcfm.h, "segment plans").
struct SegPlan {
  int* start;      // B*(VK+1), VK = seg_keys(V, taps)
  float* vinv;     // B*V (per-voxel 1/cnt)
  int* rank;       // B*n
  int* skey;       // B*n
  float* ws8;      // B*n*8 (TAPS == 8)
  int4* units;     // B*umax
  int2* tinfo;     // B*tiles
  int* nunits;     // B
};
struct SegApplyWs {
  float* xs;       // B*n*C
  float* partial;  // B*slots*C*kTV
};

inline size_t seg_plan_bytes(int B, int n, int V, int taps) {
  const int umax = seg_umax(n, V, taps), tiles = seg_tiles(V);
  size_t s = align256((size_t)B * (seg_keys(V, taps) + 1) * 4);
  s += align256((size_t)B * V * 4);
  s += 2 * align256((size_t)B * n * 4);
  if (taps == 8) s += align256((size_t)B * n * 8 * 4);
  s += align256((size_t)B * umax * 16);
  s += align256((size_t)B * tiles * 8);
  s += align256((size_t)B * 4);
  return s;
}
inline size_t seg_apply_bytes(int B, int C, int n, int V, int taps) {
  const int umax = seg_umax(n, V, taps), tiles = seg_tiles(V);
  const size_t part = (size_t)B * (umax - tiles) * std::max(C, 1) * kTV * 4;
  return align256((size_t)B * n * std::max(C, 1) * 4) + align256(part);
}
inline size_t seg_ws_bytes(int B, int C, int n, int V, int taps) {
  return seg_plan_bytes(B, n, V, taps) + seg_apply_bytes(B, C, n, V, taps);
}

struct SegCarver {
  char* p;
  char* take(size_t bytes) {
    char* q = p;
    p += align256(bytes);
    return q;
  }
};
inline SegPlan seg_plan_carve(void* mem, int B, int n, int V, int taps) {
  const int umax = seg_umax(n, V, taps), tiles = seg_tiles(V);
  SegCarver c{(char*)mem};
  SegPlan w;
  w.start = (int*)c.take((size_t)B * (seg_keys(V, taps) + 1) * 4);
  w.vinv = (float*)c.take((size_t)B * V * 4);
  w.rank = (int*)c.take((size_t)B * n * 4);
  w.skey = (int*)c.take((size_t)B * n * 4);
  w.ws8 = taps == 8 ? (float*)c.take((size_t)B * n * 8 * 4) : nullptr;
  w.units = (int4*)c.take((size_t)B * umax * 16);
  w.tinfo = (int2*)c.take((size_t)B * tiles * 8);
  w.nunits = (int*)c.take((size_t)B * 4);
  return w;
}
inline SegApplyWs seg_apply_carve(void* mem, int B, int C, int n, int V, int taps) {
  const int umax = seg_umax(n, V, taps), tiles = seg_tiles(V);
  SegCarver c{(char*)mem};
  SegApplyWs w;
  w.xs = (float*)c.take((size_t)B * n * std::max(C, 1) * 4);
  w.partial = (float*)c.take((size_t)B * (umax - tiles) * std::max(C, 1) * kTV * 4);
  return w;
}

// The plan of a scatter over items with keys at key + b*key_bstride (first n
// used): the stable sort (+ cnt_out [b, V] counts when non-null; 1/cnt when
// avg), the work units and the sorted keys / tap weights (tapw [b, 8, n] for
// TAPS == 8).
template <int TAPS>
inline int seg_plan_build(const int* key, long long key_bstride, bool avg, const float* tapw,
                          int r, int B, int n, int V, int* cnt_out, const SegPlan& w,
                          hipStream_t st) {
  // (A rocPRIM radix sort of the composite keys, kept opt-in through round 5
  // at ~70 us per sort against this kernel's 23 us, was removed in round 6.)
  const int koff = seg_koff(V, TAPS), VK = V + koff;
  PCFM_CHECK_ARG(koff == 0 || (cnt_out == nullptr && !avg),
                 "segment plan: counts of a shifted-key sort");
  int e = allow_big_lds((const void*)seg_sort_kernel);
  if (e) return e;
  hipLaunchKernelGGL(seg_sort_kernel, dim3(seg_sort_parts(VK), B), dim3(1024), seg_sort_lds(VK),
                     st, key, key_bstride, n, VK, seg_sort_span(VK), w.start, cnt_out,
                     avg ? w.vinv : nullptr, w.rank, koff);
  const int tiles = seg_tiles(V), umax = seg_umax(n, V, TAPS);
  hipLaunchKernelGGL(seg_units_kernel<TAPS>, dim3(B), dim3(1024), 0, st, w.start, V, r, tiles,
                     umax, w.units, w.tinfo, w.nunits);
  if (n > 0)
    hipLaunchKernelGGL(seg_plan_rows_kernel, dim3(ceil_div(n, 256), B), dim3(256), 0, st, w.rank,
                       key, key_bstride, TAPS == 8 ? tapw : nullptr, n, w.skey, w.ws8);
  return PCFM_OK;
}

// out[b, c, v] = sum over items i whose key (+ stencil offset) is v of the tap
// term, on a built plan (avg: scaled by the plan's 1/cnt).
template <int TAPS>
inline int seg_apply(const float* in, const SegPlan& w, bool avg, int r, int B, int C, int n,
                     int V, float* out, const SegApplyWs& aw, hipStream_t st) {
  if (C == 0) return PCFM_OK;
  const int tiles = seg_tiles(V), umax = seg_umax(n, V, TAPS), slots = umax - tiles;
  if (n > 0)
    hipLaunchKernelGGL(seg_rows_kernel,
                       dim3(ceil_div(n, kRowsItems), kRowsAllC ? 1 : ceil_div(C, 64), B),
                       dim3(256), 0, st, in, w.rank, nullptr, 0LL, nullptr, C, n, aw.xs, nullptr,
                       nullptr);
  const int gx = ceil_div(umax, kUnitWaves);
  hipLaunchKernelGGL(seg_unit_gather_kernel<TAPS>, dim3(gx, ceil_div(C, 64), B),
                     dim3(kUnitWaves * 64), 0, st, aw.xs, w.skey, w.ws8, w.start,
                     avg ? w.vinv : nullptr, w.units, w.nunits, C, n, V, r, umax, slots, out,
                     aw.partial);
  hipLaunchKernelGGL(seg_part_sum_kernel, dim3(tiles, ceil_div(C, 64), B), dim3(256), 0, st,
                     w.tinfo, aw.partial, C, V, tiles, slots, out);
  return PCFM_OK;
}

// plan + apply in one workspace (seg_ws_bytes): the unshared scatter.
template <int TAPS>
inline int seg_scatter(const float* in, const int* key, long long key_bstride, bool avg,
                       const float* tapw, int r, int B, int C, int n, int V, int* cnt_out,
                       float* out, void* ws, hipStream_t st, const char* what) {
  if (B == 0 || V == 0) return PCFM_OK;
  const SegPlan w = seg_plan_carve(ws, B, n, V, TAPS);
  const SegApplyWs aw =
      seg_apply_carve((char*)ws + seg_plan_bytes(B, n, V, TAPS), B, C, n, V, TAPS);
  int e = seg_plan_build<TAPS>(key, key_bstride, avg, tapw, r, B, n, V, cnt_out, w, st);
  if (e) return e;
  e = seg_apply<TAPS>(in, w, avg, r, B, C, n, V, out, aw, st);
  if (e) return e;
  return check_launch(what);
}

}  // namespace pcfm
