// 3x3x3 voxel convolution (PVConv's Conv3d, stride 1, padding 1) as an
// implicit GEMM on the bf16 matrix cores, with fp32-class accuracy from a
// three-term split ("bf16x3").
//
// Why: MI355X has no TF32/xf32 path; its fp32-input MFMA runs at 1/16 of the
// bf16 rate (cdna_hip_programming.md, "FP32-input MFMA").  The reference runs
// these convolutions through cuDNN with PyTorch's default allow_tf32 = True,
// i.e. with 10-bit-mantissa inputs.  Here every fp32 operand x is split into
// hi = bf16(x), lo = bf16(x - hi) (16 significant bits together) and
//     a*b ~= ah*bh + ah*bl + al*bh        (the al*bl term, ~2^-16, is dropped)
// with all products accumulated in fp32 by the MFMA.  Per product the
// relative error is ~2^-16: ~30x tighter than TF32, at 3 bf16 MFMAs = 3/16 of
// the fp32-MFMA cost.
//
// GEMM view (NCDHW fp32 tensors, V = R^3 voxels per sample):
//   Y[b, m, v] = sum_{tap, k} W'[tap, m, k] * X[b, k, v + off(tap)]  (+ bias[m])
// forward:        m = out channel, k = in channel, W'[tap, co, ci] = W[co, ci, tap]
// backward-data:  m = in channel,  k = out channel, X = dY,
//                 W'[tap, ci, co] = W[co, ci, 26 - tap]   (off(26 - t) = -off(t))
// A operand = weight tile [m][k], B operand = input tile [voxel][k] staged in
// LDS as bf16 hi/lo rows; D[m][voxel] leaves with lanes along voxels, i.e.
// coalesced into the NCDHW output.  Out-of-grid neighbours read as 0 (padding).
#include <algorithm>
#include <cstdlib>
#include <mutex>

#include "mfma_x3.hpp"

namespace pcfm {
namespace {

// W [Cout][Cin][27] fp32 -> W' [27][M][K] bf16 hi, lo (see header), rows of K
// interleaved per 32-channel group (split_off)
__global__ void __launch_bounds__(256)
    conv3_wsplit_kernel(const float* __restrict__ w, int cout, int cin, int transpose,
                        uint16_t* __restrict__ wh) {
  const size_t total = (size_t)27 * cout * cin;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  // i indexes the destination [tap][m][k]
  const int M = transpose ? cin : cout, K = transpose ? cout : cin;
  const int tap = (int)(i / ((size_t)M * K));
  const int rem = (int)(i - (size_t)tap * M * K);
  const int m = rem / K, k = rem - m * K;
  const float v = transpose ? w[((size_t)k * cin + m) * 27 + (26 - tap)]
                            : w[((size_t)m * cin + k) * 27 + tap];
  uint32_t hi, lo;
  split_bf16(v, hi, lo);
  const size_t o = split_off((size_t)tap * M + m, k, K);  // interleaved image (pcfm_common.hpp)
  wh[o] = (uint16_t)hi;
  wh[o + kSplitLo] = (uint16_t)lo;
}

// ---------------------------------------------------------------------------
// Occupancy of a voxelized grid (PVConv's first convolution reads the
// voxelization's output, exactly zero in every voxel no point falls into, and
// its input gradient is read back only at occupied voxels): from the
// voxelization's counts cnt [b][V] (> 0 = occupied),
//   tmask [b][V / 256]: bit t < 27 = tap t of the 256-voxel tile's forward
//     GEMM reads an occupied voxel (v + off(t) in the volume); bit 31 = the
//     tile holds an occupied voxel;
//   cmask [b][V / 64]: bit p < 9 = some voxel of the 64-voxel chunk shifted by
//     (dx, dy, dz), p = 3 (dx + 1) + dy + 1, dz = -1..1, is occupied, i.e. the
//     weight gradient's (pair, chunk) step has a nonzero X operand;
//   kmask [b][V / 16]: bit t < 27 = some voxel of the 16-voxel group shifted by
//     tap t is occupied, i.e. the weight gradient's 16-voxel K-slice of tap t
//     has a nonzero X operand (the rest of its products are exact zeros).
// grid = (V / 256, b), 256 threads (a thread = a voxel, a wave = a chunk).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
    conv3_occupancy_kernel(const int* __restrict__ cnt, int R, uint32_t* __restrict__ tmask,
                           uint32_t* __restrict__ cmask, uint32_t* __restrict__ kmask) {
  __shared__ uint32_t sm;
  const int V = R * R * R, R2 = R * R;
  const int b = blockIdx.y, t = threadIdx.x;
  const int v = blockIdx.x * 256 + t;
  const int x = v / R2, y = (v / R) % R, z = v % R;
  const int* __restrict__ c = cnt + (size_t)b * V;
  uint32_t taps = 0, pairs = 0;
#pragma unroll
  for (int tap = 0; tap < 27; ++tap) {
    const int dx = tap / 9 - 1, dy = (tap / 3) % 3 - 1, dz = tap % 3 - 1;
    const int xx = x + dx, yy = y + dy, zz = z + dz;
    if ((unsigned)xx < (unsigned)R && (unsigned)yy < (unsigned)R && (unsigned)zz < (unsigned)R &&
        c[xx * R2 + yy * R + zz] > 0) {
      taps |= 1u << tap;
      pairs |= 1u << (tap / 3);
    }
  }
  uint32_t k16 = taps;  // 16-voxel group OR of the tap bits
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) k16 |= __shfl_xor(k16, o);
  if ((t & 15) == 0) kmask[(size_t)b * (V / 16) + v / 16] = k16;
  if (c[v] > 0) taps |= 1u << 31;
  if (t == 0) sm = 0;
  __syncthreads();
  // chunk (wave) OR of the pair bits, block OR of the tap bits
  uint32_t w = pairs;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) w |= __shfl_xor(w, o);
  if ((t & 63) == 0) cmask[(size_t)b * (V / 64) + v / 64] = w;
  atomicOr(&sm, taps);
  __syncthreads();
  if (t == 0) tmask[(size_t)b * (V / 256) + blockIdx.x] = sm;
}

// ---------------------------------------------------------------------------
// Chunk lists of a voxelized grid (from the voxelization's counts), for the
// list form of the LDS-DMA GEMM.  A chunk is 32 consecutive voxels (a z-row at
// r = 32): list 0 = the chunks holding an occupied voxel (cnt > 0: where
// PVConv's first convolution's input gradient is read back, vox.cu:86-110),
// list 1 = the chunks holding a voxel with an occupied voxel in its 3x3x3
// neighbourhood (outside them that convolution's forward output is exactly
// its bias: its input is 0 there).  Whole chunks keep the GEMM's B-row fetches
// and output stores 128-B runs (voxel-granular lists measured slower: short
// scattered runs).  Entries are global chunk indices (b V + v) / 32, ascending
// (deterministic).  Lists 2 / 3: the occupied / active voxels themselves,
// global voxel indices b V + v, ascending (the voxel-granular forms).
// Buffer layout: pcfm_conv3d_vlist_bytes.
// ---------------------------------------------------------------------------
constexpr int kChunk = 32;

__device__ __forceinline__ void vlist_flags(const int* __restrict__ c, int v, int R, bool& occ,
                                            bool& act) {
  const int R2 = R * R;
  const int x = v / R2, y = (v / R) % R, z = v % R;
  occ = c[v] > 0;
  act = false;
#pragma unroll
  for (int tap = 0; tap < 27; ++tap) {
    const int xx = x + tap / 9 - 1, yy = y + (tap / 3) % 3 - 1, zz = z + tap % 3 - 1;
    act = act || ((unsigned)xx < (unsigned)R && (unsigned)yy < (unsigned)R &&
                  (unsigned)zz < (unsigned)R && c[xx * R2 + yy * R + zz] > 0);
  }
}

// chunk flags of this thread's chunk (32 consecutive lanes = one chunk); o, a:
// the thread's own voxel's flags
__device__ __forceinline__ void chunk_flags(const int* __restrict__ cnt, long long g, int R,
                                            bool& occ, bool& act, bool& o, bool& a) {
  const int V = R * R * R;
  vlist_flags(cnt + (g / V) * V, (int)(g % V), R, o, a);
  const int sh = threadIdx.x & 32;
  occ = ((__ballot(o) >> sh) & 0xFFFFFFFFull) != 0ull;
  act = ((__ballot(a) >> sh) & 0xFFFFFFFFull) != 0ull;
}
__device__ __forceinline__ void chunk_flags(const int* __restrict__ cnt, long long g, int R,
                                            bool& occ, bool& act) {
  bool o, a;
  chunk_flags(cnt, g, R, occ, act, o, a);
}

// grid = B V / 256 tiles (8 chunks each), 256 threads: per-tile chunk counts
// (lists 0, 1 -> tcount[2][tiles]) and voxel counts (lists 2, 3 -> tcount2[2][tiles])
__global__ void __launch_bounds__(256)
    conv3_vlist_count_kernel(const int* __restrict__ cnt, int R, int tiles,
                             int* __restrict__ tcount, int* __restrict__ tcount2) {
  __shared__ int ws[2][8];
  __shared__ int wv[2][4];
  const int t = threadIdx.x;
  const long long g = (long long)blockIdx.x * 256 + t;
  bool occ, act, o, a;
  chunk_flags(cnt, g, R, occ, act, o, a);
  if ((t & 31) == 0) {
    ws[0][t >> 5] = occ ? 1 : 0;
    ws[1][t >> 5] = act ? 1 : 0;
  }
  // occupied / active voxels (lists 2, 3): per-wave ballot counts
  const int n2 = __popcll(__ballot(o)), n3 = __popcll(__ballot(a));
  if ((t & 63) == 0) {
    wv[0][t >> 6] = n2;
    wv[1][t >> 6] = n3;
  }
  __syncthreads();
  if (t < 2) {
    int n = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) n += ws[t][q];
    tcount[t * tiles + blockIdx.x] = n;
  } else if (t < 4) {
    const int k = t - 2;
    tcount2[k * tiles + blockIdx.x] = ((wv[k][0] + wv[k][1]) + wv[k][2]) + wv[k][3];
  }
}

// one block: exclusive scans of the two per-tile count rows (in place) and
// the totals
__global__ void __launch_bounds__(1024)
    conv3_vlist_scan_kernel(int* __restrict__ tcount, int tiles, int* __restrict__ counts,
                            int rows) {
  __shared__ int wsum[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int k = 0; k < rows; ++k) {
    int* row = tcount + (size_t)k * tiles;
    int carry = 0;
    for (int t0 = 0; t0 < tiles; t0 += 1024) {
      const int i = t0 + t;
      const int c = i < tiles ? row[i] : 0;
      int x = c;
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
        ofs += g < w ? wsum[g] : 0;
        total += wsum[g];
      }
      if (i < tiles) row[i] = ofs + x - c;
      carry += total;
      __syncthreads();
    }
    if (t == 0) counts[k] = carry;
  }
}

// grid = tiles, 256 threads: each tile writes its listed chunks and voxels at
// its offsets
__global__ void __launch_bounds__(256)
    conv3_vlist_write_kernel(const int* __restrict__ cnt, int R, int tiles,
                             const int* __restrict__ toff, int* __restrict__ list0,
                             int* __restrict__ list1, const int* __restrict__ toff2,
                             int* __restrict__ list2, int* __restrict__ list3,
                             uint32_t* __restrict__ bits2, uint32_t* __restrict__ bits3) {
  __shared__ int ws[2][8];
  __shared__ int wv[2][4];
  const int t = threadIdx.x;
  const long long g = (long long)blockIdx.x * 256 + t;
  bool occ, act, o, a;
  chunk_flags(cnt, g, R, occ, act, o, a);
  if ((t & 31) == 0) {
    ws[0][t >> 5] = occ ? 1 : 0;
    ws[1][t >> 5] = act ? 1 : 0;
  }
  const unsigned long long m2 = __ballot(o), m3 = __ballot(a);
  if ((t & 63) == 0) {
    wv[0][t >> 6] = __popcll(m2);
    wv[1][t >> 6] = __popcll(m3);
  }
  if ((t & 31) == 0) {  // the lists' voxel bitmaps (bit g & 31 of word g >> 5)
    bits2[g >> 5] = (uint32_t)(m2 >> (t & 32));
    bits3[g >> 5] = (uint32_t)(m3 >> (t & 32));
  }
  __syncthreads();
  // lists 2 / 3: the occupied / active voxels in voxel order
  if (o) {
    int p = toff2[blockIdx.x];
    for (int u = 0; u < (t >> 6); ++u) p += wv[0][u];
    p += __builtin_amdgcn_mbcnt_hi((unsigned)(m2 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m2, 0u));
    list2[p] = (int)g;
  }
  if (a) {
    int p = toff2[tiles + blockIdx.x];
    for (int u = 0; u < (t >> 6); ++u) p += wv[1][u];
    p += __builtin_amdgcn_mbcnt_hi((unsigned)(m3 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m3, 0u));
    list3[p] = (int)g;
  }
  if ((t & 31) == 0) {
    const int q = t >> 5, chunk = blockIdx.x * 8 + q;
    int p0 = toff[blockIdx.x], p1 = toff[tiles + blockIdx.x];
    for (int u = 0; u < q; ++u) {
      p0 += ws[0][u];
      p1 += ws[1][u];
    }
    if (occ) list0[p0] = chunk;
    if (act) list1[p1] = chunk;
  }
}

// y[b][m][v] = value (bias[m], or 0 without bias) in the chunks NOT in list
// `which` -- the complement the list form of the GEMM does not write.
// grid = B V / 256, 256 threads.
__global__ void __launch_bounds__(256)
    conv3_fill_unlisted_kernel(const int* __restrict__ cnt, int R, int M, int which,
                               const float* __restrict__ bias, float* __restrict__ y,
                               const uint32_t* __restrict__ vbits) {
  const int V = R * R * R;
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  if (vbits != nullptr) {  // over a voxel list (2 / 3): every voxel not in it
    if ((vbits[g >> 5] >> (g & 31)) & 1u) return;
  } else {
    bool occ, act;
    chunk_flags(cnt, g, R, occ, act);
    if (which == 0 ? occ : act) return;
  }
  const int b = (int)(g / V), v = (int)(g % V);
  float* __restrict__ yb = y + (size_t)b * M * V + v;
  for (int m = 0; m < M; ++m)
    nt_st(bias != nullptr ? bias[m] : 0.0f, yb + (size_t)m * V);
}

// ---------------------------------------------------------------------------
// Channels-last split of the GEMM's B operand, done once per convolution
// instead of once per tap: X fp32 [B][C][V] -> hi, lo bf16 [B][V][C], rows
// interleaved per 32-channel group (split_off).
// grid = (V / 64, C / 64, B), 256 threads; a 64 x 64 LDS transpose tile.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
    conv3_split_cl_kernel(const float* __restrict__ x, int C, int V, uint16_t* __restrict__ xh) {
  __shared__ float tile[64][65];
  const int v0 = blockIdx.x * 64, c0 = blockIdx.y * 64, b = blockIdx.z;
  const int t = threadIdx.x;
  const float* __restrict__ src = x + ((size_t)b * C + c0) * V + v0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = i * 4 + (t >> 6), v = t & 63;
    tile[c][v] = src[(size_t)c * V + v];
  }
  __syncthreads();
  const int v = t >> 2, cg = (t & 3) * 16;
  float f[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) f[q] = tile[cg + q][v];
  const size_t o = split_off((size_t)b * V + v0 + v, c0 + cg, C);
  store_split<16>(f, xh + o, xh + o + kSplitLo);
}

// ---------------------------------------------------------------------------
// Forward / backward-data implicit GEMM over the channels-last split input.
// grid = (V / TN) * (M / TM) * B (1-D); K-steps s = tap * (K / KT) + channel chunk.
// A = pre-split weights W'[tap][m][k], B = pre-split input rows xs[b][v][k]:
// every staging access is a 16-B copy (no per-tap split arithmetic).  KT = 64
// channels per step: 48 MFMAs per wave between barriers (TM = TN = 128).
// LDS rows are KT + 8 bf16 (144 B): conflict-free ds_read_b128 fragments.
// ---------------------------------------------------------------------------
template <int TM, int TN, int KT>
struct TileK {
  static constexpr int LDR = KT + 8;
  static constexpr int SI = TM / 64, SJ = TN / 64;
  static constexpr int A_ELEMS = TM * LDR, B_ELEMS = TN * LDR;
  static constexpr int BUF = 2 * A_ELEMS + 2 * B_ELEMS;
  static constexpr int CPR = KT / 8;               // 16-B chunks per row
  static constexpr int QA = TM * CPR / 256;        // A chunks per thread (per image)
  static constexpr int QB = TN * CPR / 256;        // B chunks per thread (per image)
};

template <int TM, int TN, int KT>
__device__ __forceinline__ void tile_mfma_k(const uint16_t* buf, int wr, int wc, int r, int h,
                                            f32x16 (&acc)[TM / 64][TN / 64]) {
  using T = TileK<TM, TN, KT>;
  const uint16_t* sAh = buf;
  const uint16_t* sAl = buf + T::A_ELEMS;
  const uint16_t* sBh = buf + 2 * T::A_ELEMS;
  const uint16_t* sBl = sBh + T::B_ELEMS;
#pragma unroll
  for (int kk = 0; kk < KT / 16; ++kk) {
    bf16x8 ah[T::SI], al[T::SI], bh[T::SJ], bl[T::SJ];
#pragma unroll
    for (int i = 0; i < T::SI; ++i) {
      const int o = (wr * (TM / 2) + i * 32 + r) * T::LDR + kk * 16 + 8 * h;
      ah[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sAh + o));
      al[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sAl + o));
    }
#pragma unroll
    for (int j = 0; j < T::SJ; ++j) {
      const int o = (wc * (TN / 2) + j * 32 + r) * T::LDR + kk * 16 + 8 * h;
      bh[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sBh + o));
      bl[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sBl + o));
    }
    // product-major order: consecutive MFMAs write different accumulators
#pragma unroll
    for (int i = 0; i < T::SI; ++i)
#pragma unroll
      for (int j = 0; j < T::SJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < T::SI; ++i)
#pragma unroll
      for (int j = 0; j < T::SJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < T::SI; ++i)
#pragma unroll
      for (int j = 0; j < T::SJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
  }
}

template <int TM, int TN, int KT>
__global__ void __launch_bounds__(256)
    conv3_igemm_cl_kernel(const uint16_t* __restrict__ xh, const uint16_t* __restrict__ xl,
                          const uint16_t* __restrict__ wh, const uint16_t* __restrict__ wl,
                          const float* __restrict__ bias, float* __restrict__ y, int K, int M,
                          int R, int S, float* __restrict__ part) {
  using T = TileK<TM, TN, KT>;
  __shared__ __attribute__((aligned(16))) uint16_t lds[T::BUF];
  const int V = R * R * R, R2 = R * R;
  // 1-D grid of (m tile, voxel tile, b) items, m fastest, dealt to the 8 XCDs
  // in contiguous runs (T1 remap): an XCD sweeps a contiguous slab of the grid,
  // so the 27 taps' neighbour rows of concurrently resident blocks overlap in
  // its L2 instead of streaming from the Infinity Cache.
  int id = (int)blockIdx.x;
  {
    const int nwg = (int)gridDim.x, q = nwg / 8, rr = nwg % 8, xcd = id % 8;
    id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + id / 8;
  }
  const int nmt = M / TM, nvt = V / TN;
  const int items = (int)gridDim.x / S;  // split-K: S K-ranges per output tile, split outermost
  const int sp = id / items;
  id -= sp * items;
  const int m0 = (id % nmt) * TM;
  id /= nmt;
  const int v0 = (id % nvt) * TN, b = id / nvt;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1, r = lane & 31, h = lane >> 5;
  const uint16_t* __restrict__ xbh = xh + (size_t)b * V * 2 * K;
  const uint16_t* __restrict__ xbl = xl + (size_t)b * V * 2 * K;
  const int nck = K / KT, nall = 27 * nck;
  const int s0 = (int)((long long)nall * sp / S), nsteps = (int)((long long)nall * (sp + 1) / S) - s0;
  // chunk q of this thread: row (t + 256 q) / CPR, 8-channel column (t % CPR) * 8
  const int col = (t % T::CPR) * 8;
  int bv[T::QB], bx[T::QB], by[T::QB], bz[T::QB];
#pragma unroll
  for (int q = 0; q < T::QB; ++q) {
    bv[q] = v0 + (t + 256 * q) / T::CPR;
    bx[q] = bv[q] / R2;
    by[q] = (bv[q] / R) % R;
    bz[q] = bv[q] % R;
  }

  StageVec<T::QA> rah, ral;
  StageVec<T::QB> rbh, rbl;
  auto load = [&](int s) {
    const int c0 = (s / 27) * KT, tap = s - (s / 27) * 27;  // chunk-major (L2 reuse)
#pragma unroll
    for (int q = 0; q < T::QA; ++q) {
      const int row = (t + 256 * q) / T::CPR;
      const size_t g = split_off((size_t)tap * M + m0 + row, c0 + col, K);
      sv_put<T::QA>(rah, q, *reinterpret_cast<const uint4*>(wh + g));
      sv_put<T::QA>(ral, q, *reinterpret_cast<const uint4*>(wl + g));
    }
    const int dx = tap / 9 - 1, dy = (tap / 3) % 3 - 1, dz = tap % 3 - 1;
    const int doff = dx * R2 + dy * R + dz;
#pragma unroll
    for (int q = 0; q < T::QB; ++q) {
      const bool inb = (unsigned)(bx[q] + dx) < (unsigned)R &&
                       (unsigned)(by[q] + dy) < (unsigned)R && (unsigned)(bz[q] + dz) < (unsigned)R;
      const size_t o = split_off((size_t)(inb ? bv[q] + doff : bv[q]), c0 + col, K);
      const uint4 hv = *reinterpret_cast<const uint4*>(xbh + o);
      const uint4 lv = *reinterpret_cast<const uint4*>(xbl + o);
      sv_put<T::QB>(rbh, q, inb ? hv : uint4{0u, 0u, 0u, 0u});
      sv_put<T::QB>(rbl, q, inb ? lv : uint4{0u, 0u, 0u, 0u});
    }
  };
  auto store = [&](uint16_t* buf) {
#pragma unroll
    for (int q = 0; q < T::QA; ++q) {
      uint16_t* d = buf + ((t + 256 * q) / T::CPR) * T::LDR + col;
      *reinterpret_cast<uint4*>(d) = sv_get<T::QA>(rah, q);
      *reinterpret_cast<uint4*>(d + T::A_ELEMS) = sv_get<T::QA>(ral, q);
    }
#pragma unroll
    for (int q = 0; q < T::QB; ++q) {
      uint16_t* d = buf + 2 * T::A_ELEMS + ((t + 256 * q) / T::CPR) * T::LDR + col;
      *reinterpret_cast<uint4*>(d) = sv_get<T::QB>(rbh, q);
      *reinterpret_cast<uint4*>(d + T::B_ELEMS) = sv_get<T::QB>(rbl, q);
    }
  };

  f32x16 acc[T::SI][T::SJ];
#pragma unroll
  for (int i = 0; i < T::SI; ++i)
#pragma unroll
    for (int j = 0; j < T::SJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  load(s0);
  store(lds);
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    if (s + 1 < nsteps) load(s0 + s + 1);
    tile_mfma_k<TM, TN, KT>(lds, wr, wc, r, h, acc);
    __syncthreads();
    if (s + 1 < nsteps) store(lds);
    __syncthreads();
  }
  // S == 1: y (+ bias); else this split's partial, summed in split order by
  // conv3_ksum_kernel (deterministic)
  const int nb = items / (nmt * nvt);  // batch elements
  float* __restrict__ yb =
      S == 1 ? y + (size_t)b * M * V : part + ((size_t)sp * nb + b) * M * V;
  float biasv[T::SI][16];
#pragma unroll
  for (int i = 0; i < T::SI; ++i)
    load_bias16(S == 1 ? bias : nullptr, m0 + wr * (TM / 2) + i * 32, h, M, biasv[i]);
#pragma unroll
  for (int i = 0; i < T::SI; ++i)
#pragma unroll
    for (int j = 0; j < T::SJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wr * (TM / 2) + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int v = v0 + wc * (TN / 2) + j * 32 + r;
        yb[(size_t)m * V + v] = acc[i][j][e] + biasv[i][e];
      }
}

// y[b][m][v] = bias[m] + sum_sp part[sp][b][m][v], float4 per thread
__global__ void __launch_bounds__(256)
    conv3_ksum_kernel(const float* __restrict__ part, const float* __restrict__ bias, int S, int M,
                      int V, long long total4, float* __restrict__ y) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total4) return;
  const float4* p4 = reinterpret_cast<const float4*>(part);
  float4 a = p4[i];
  for (int sp = 1; sp < S; ++sp) {
    const float4 q = p4[(size_t)sp * total4 + i];
    a.x += q.x;
    a.y += q.y;
    a.z += q.z;
    a.w += q.w;
  }
  if (bias != nullptr) {
    const float bb = bias[(int)((i * 4 / V) % M)];  // V % 4 == 0: a float4 is one (b, m) row
    a.x += bb;
    a.y += bb;
    a.z += bb;
    a.w += bb;
  }
  reinterpret_cast<float4*>(y)[i] = a;
}

// ---------------------------------------------------------------------------
// Forward / backward-data implicit GEMM, LDS-DMA pipelined form (the large
// grids: r = 32 and r = 16).  128 (m) x 256 (voxel) tile, 8 waves of 64 x 64,
// K-steps of 32 channels, THREE LDS stages filled by global_load_lds_dwordx4
// (cdna_hip_programming.md section 5 "Async global->LDS copy"): the loads of
// step s+2 are in flight while step s computes; one raw s_barrier per step,
// counted s_waitcnt vmcnt (never 0 inside the loop).  An LDS-DMA writes
// lane-linear 16-B pieces, so the bank swizzle is applied on the SOURCE side:
// physical chunk p of row r holds logical k-chunk p ^ ((r >> 2) & 3), which
// makes the ds_read_b128 fragment reads conflict-free (64-B rows).  A
// neighbour outside the grid reads from a zero row (the padding).
// ---------------------------------------------------------------------------
constexpr int kGM = 128, kGN = 256, kGStages = 3;

// K-step geometry of the LDS-DMA kernel: KT = 32 (64-B rows, 48 KiB stages,
// one block per CU) or KT = 16 (32-B rows, 24 KiB stages, two blocks per CU)
// GN: voxels per block tile (256: 8 waves, one block per CU; 128: 4 waves and
// two stages, two independent blocks per CU)
template <int KT, int GN = kGN>
struct GK {
  static constexpr int NW = 2 * (GN / 64);     // waves: 2 (m) x GN / 64 (voxels)
  static constexpr int RB = KT * 2;            // bytes per LDS row (hi or lo)
  static constexpr int CPR = RB / 16;          // 16-B chunks per row
  static constexpr int RPP = 1024 / RB;        // rows per 1-KiB LDS-DMA piece
  static constexpr int A = kGM * RB, B = GN * RB;  // bytes per image
  static constexpr int STAGE = 2 * A + 2 * B;
  static constexpr int APW = 2 * A / 1024 / NW, BPW = 2 * B / 1024 / NW;  // pieces per wave
  static constexpr int API = A / 1024, BPI = B / 1024;                  // pieces per image
  // physical chunk p of row r holds logical chunk p ^ swz(r): conflict-free
  // ds_read_b128 fragment reads
  static __device__ __forceinline__ int swz(int row) {
    return KT == 32 ? (row >> 2) & 3 : (row >> 3) & 1;
  }
};

__device__ __forceinline__ void glds16(const void* g, uint8_t* l) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                   (void __attribute__((address_space(3)))*)l, 16, 0, 0);
}

// One step's MFMA operands of a wave (64 x 64 of the 128 x 256 tile):
// F[kk] = {A hi 0, A hi 1, A lo 0, A lo 1, B hi 0, B hi 1, B lo 0, B lo 1}
template <int KT, int GN = kGN>
__device__ __forceinline__ void glds_frags(const uint8_t* lds, int buf, int wr, int wc, int r,
                                           int h, bf16x8 (&F)[KT / 16][8]) {
  using G = GK<KT, GN>;
  const uint8_t* base = lds + buf * G::STAGE;
#pragma unroll
  for (int kk = 0; kk < KT / 16; ++kk) {
    const int kc = 2 * kk + h;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = wr * 64 + i * 32 + r;
      const int off = row * G::RB + ((kc ^ G::swz(row)) << 4);
      F[kk][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(base + off));
      F[kk][2 + i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(base + G::A + off));
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wc * 64 + j * 32 + r;
      const int off = 2 * G::A + row * G::RB + ((kc ^ G::swz(row)) << 4);
      F[kk][4 + j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(base + off));
      F[kk][6 + j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(base + G::B + off));
    }
  }
}

template <int KT>
__device__ __forceinline__ void glds_mfma(const bf16x8 (&F)[KT / 16][8], f32x16 (&acc)[2][2]) {
#pragma unroll
  for (int kk = 0; kk < KT / 16; ++kk) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[kk][i], F[kk][4 + j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[kk][i], F[kk][6 + j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(F[kk][2 + i], F[kk][4 + j], acc[i][j], 0, 0, 0);
  }
}

template <int KT, int GN = kGN, int NST = kGStages>
__global__ void __launch_bounds__(GN * 2)  // GK<KT, GN>::NW = GN / 32 waves
    conv3_igemm_glds_kernel(const uint16_t* __restrict__ xh, const uint16_t* __restrict__ xl,
                            const uint16_t* __restrict__ wh, const uint16_t* __restrict__ wl,
                            const uint16_t* __restrict__ zrow, const float* __restrict__ bias,
                            float* __restrict__ y, int K, int M, int R, int S,
                            float* __restrict__ part, const uint32_t* __restrict__ tmask,
                            int mmode, const int* __restrict__ vlist = nullptr,
                            const int* __restrict__ vcount = nullptr, int lg = 5,
                            const uint32_t* __restrict__ obits = nullptr) {
  using G = GK<KT, GN>;
  __shared__ __attribute__((aligned(16))) uint8_t lds[NST * G::STAGE];
  const int V = R * R * R, R2 = R * R;
  const int nmt = M / kGM, nvt = V / GN;
  // List form (S == 1, conv3_vlist_*): the block's GN output voxels are the
  // CPT listed runs of 2^lg voxels [lt CPT, lt CPT + CPT) -- global run
  // indices (b V + v) >> lg whose result is wanted, ascending: 32-voxel chunks
  // (lg 5) or single voxels (lg 0) -- instead of a contiguous range; the B rows
  // of every tap are their neighbours (a padding entry reads zero rows and
  // stores nothing).  Only the first nmt x ceil(count / CPT) blocks
  // (device-side count) work, dealt to the XCDs as the dense grid is; the rest
  // leave at once, before any barrier.
  const bool lmode = vlist != nullptr;
  const int CPT = GN >> lg, lmask = (1 << lg) - 1;
  int lcount = 0;
  int nwg = (int)gridDim.x, id = (int)blockIdx.x;
  if (lmode) {
    lcount = __builtin_amdgcn_readfirstlane(vcount[0]);
    nwg = nmt * ((lcount + CPT - 1) / CPT);
    if (id >= nwg) return;
  }
  {
    const int q = nwg / 8, rr = nwg % 8, xcd = id % 8;
    id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + id / 8;
  }
  const int nb = (int)gridDim.x / (S * nmt * nvt);  // batch elements
  const int m0 = (id % nmt) * kGM;
  id /= nmt;
  const int lt = id;  // list tile (list form)
  const int v0 = (id % nvt) * GN;
  id /= nvt;
  const int b = id % nb, sp = id / nb;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w / (GN / 64), wc = w % (GN / 64), r = lane & 31, h = lane >> 5;
  // Empty-voxel skipping (S == 1; conv3_occupancy_kernel's tile masks):
  // mmode 1 (forward of a conv over a voxelized grid): only the taps whose
  // shifted tile holds an occupied voxel -- every other tap's B rows are exact
  // zeros, so skipping it leaves the accumulators' bits unchanged; mmode 2
  // (backward-data into a voxelized grid): only tiles that hold an occupied
  // voxel (the gradient is read back there only); the others are written 0.
  const uint32_t kAll = 0x7FFFFFFu;
  uint32_t mask = kAll;
  if (mmode != 0 && !lmode) {
    const uint32_t mm = __builtin_amdgcn_readfirstlane(tmask[(size_t)b * (V >> 8) + (v0 >> 8)]);
    mask = mmode == 1 ? (mm & kAll) : ((mm >> 31) ? kAll : 0u);
  }
  const int na = __builtin_popcount(mask);
  // split-K (small grids, r = 8): this block's K-steps [k0, k1) of na * K / KT
  const int nall = na * (K / KT);
  const int k0 = (int)((long long)nall * sp / S), k1 = (int)((long long)nall * (sp + 1) / S);
  const int nsteps = k1 - k0;
  // K-step order: channel chunk major, the active taps of a chunk in tap order.
  // (ichunk, itap) is the step last issued (iseq); issue() advances one step
  // at a time in scalar registers (masks apply only with S == 1, so k0 = 0
  // unless every tap is active)
  const int first = mask != 0u ? __builtin_ctz(mask) : 0;
  int iseq = 0;
  int ichunk = na > 0 ? k0 / na : 0;
  int itap = mask == kAll ? k0 % 27 : first;
  const size_t bV = (size_t)b * V;
  const int prow = lane / G::CPR, pch = lane % G::CPR;  // this lane's place in a piece

  // A pieces: I = APW w + q -> image I / API, rows (I % API) * RPP + lane / CPR.
  // Per-piece element offsets are fixed; a step adds the uniform tap / chunk offset.
  const uint16_t* abase[G::APW];
#pragma unroll
  for (int q = 0; q < G::APW; ++q) {
    const int I = G::APW * w + q;
    const int row = (I % G::API) * G::RPP + prow;
    abase[q] = ((I / G::API) ? wl : wh) + (size_t)(m0 + row) * 2 * K + ((pch ^ G::swz(row)) << 3);
  }
  // B pieces: I = BPW w + q -> image I / BPI (waves 0-3: hi, 4-7: lo)
  const uint16_t* bbase[G::BPW];
  const uint16_t* zbase[G::BPW];
  // bit t: tap t's neighbour of the piece's voxel is inside the volume (all 0 for
  // padding).  Built once, so a step selects its source with a bit test instead
  // of three range checks (which hipcc compiled to exec-mask branches per piece)
  uint32_t bval[G::BPW];
#pragma unroll
  for (int q = 0; q < G::BPW; ++q) {
    const int I = G::BPW * w + q;
    const int row = (I % G::BPI) * G::RPP + prow;
    long long gv = (long long)bV + v0 + row;  // global row b V + v, -1: padding
    if (lmode) {
      const int e = lt * CPT + (row >> lg);
      gv = e < lcount ? ((long long)vlist[e] << lg) + (row & lmask) : -1;
    }
    const int v = gv >= 0 ? (int)(gv % V) : 0;
    const int cofs = (pch ^ G::swz(row)) << 3;
    bbase[q] = ((I / G::BPI) ? xl : xh) + (size_t)(gv >= 0 ? gv : 0) * 2 * K + cofs;
    zbase[q] = zrow + cofs;
    const int x = v / R2, yy = (v / R) % R, z = v % R;
    // per axis: bit (d + 1) set when coordinate + d is inside [0, R)
    const uint32_t ax = (x > 0 ? 1u : 0u) | 2u | (x + 1 < R ? 4u : 0u);
    const uint32_t ay = (yy > 0 ? 1u : 0u) | 2u | (yy + 1 < R ? 4u : 0u);
    const uint32_t az = (z > 0 ? 1u : 0u) | 2u | (z + 1 < R ? 4u : 0u);
    uint32_t m = 0u;
#pragma unroll
    for (int t = 0; t < 27; ++t)
      m |= (((ax >> (t / 9)) & (ay >> ((t / 3) % 3)) & (az >> (t % 3))) & 1u) << t;
    // obits (the forward over a voxelized input): a neighbour without a point
    // has an all-zero row, so it is read from the zero row instead (same bits:
    // zeros either way) -- the gather then fetches only occupied rows
    if (obits != nullptr && gv >= 0) {
      uint32_t keep = 0u;
#pragma unroll
      for (int t = 0; t < 27; ++t) {
        const long long gn = gv + (t / 9 - 1) * R2 + ((t / 3) % 3 - 1) * R + (t % 3 - 1);
        const uint32_t word = ((m >> t) & 1u) ? obits[gn >> 5] : 0u;
        keep |= ((word >> (gn & 31)) & 1u) << t;
      }
      m = keep;
    }
    bval[q] = gv >= 0 ? m : 0u;
  }

  auto issue = [&](int sl, int buf) {
    // channel-chunk-major: the 27 taps of one chunk are consecutive, so the
    // neighbour rows they re-read stay in L2 (tap-major measured slower)
    {
      const bool adv = sl != iseq;
      const uint32_t rest = mask & ~((2u << itap) - 1u);
      const int nt = rest != 0u ? __builtin_ctz(rest) : first;
      ichunk += (adv && rest == 0u) ? 1 : 0;
      itap = adv ? nt : itap;
      iseq = sl;
    }
    const int c0 = ichunk * KT, tap = itap;
    // the chunk's place in an interleaved row (split_off; a KT-chunk never
    // straddles a 32-channel group)
    const int cof = ((c0 >> 5) << 6) + (c0 & 31);
    uint8_t* base = lds + buf * G::STAGE;
    const size_t aofs = (size_t)tap * M * 2 * K + cof;
#ifndef PCFM_EXP_CNOA
#pragma unroll
    for (int q = 0; q < G::APW; ++q) {
      const int I = G::APW * w + q;
      glds16(abase[q] + aofs, base + (I / G::API) * G::A + (I % G::API) * 1024);
    }
#endif
    const int dx = tap / 9 - 1, dy = (tap / 3) % 3 - 1, dz = tap % 3 - 1;
    const long long bofs = (long long)(dx * R2 + dy * R + dz) * 2 * K + cof;
#ifdef PCFM_EXP_CNOB
    if (aofs == (size_t)-1)
#endif
#pragma unroll
    for (int q = 0; q < G::BPW; ++q) {
      const int I = G::BPW * w + q;
      // branch-free select of the source row (a divergent ?: on the pointer
      // compiled to an exec-mask branch around every piece)
      const unsigned long long src = (unsigned long long)(bbase[q] + bofs);
      const unsigned long long zsrc = (unsigned long long)zbase[q];
      const bool inb = (bval[q] >> tap) & 1u;
      const uint32_t slo = inb ? (uint32_t)src : (uint32_t)zsrc;
      const uint32_t shi = inb ? (uint32_t)(src >> 32) : (uint32_t)(zsrc >> 32);
      glds16((const void*)(((unsigned long long)shi << 32) | slo),
             base + 2 * G::A + (I / G::BPI) * G::B + (I % G::BPI) * 1024);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  if (nsteps > 0) {  // an all-skipped tile writes bias (forward) / 0 (backward-data)
#ifndef PCFM_CONV_GLDS_NOPF
  // Fragment registers double-buffered across steps: after the barrier of
  // step s the waves read step s+1's fragments while step s's 24 MFMAs run,
  // so the LDS read latency of a step hides behind the previous step's
  // matrix work (the single-buffered form exposed it at every step: 2 waves
  // per SIMD cannot cover it).  Stage s's LDS buffer is refilled (stage s+3)
  // once every wave holds its fragments: lgkmcnt(0) + barrier.
  bf16x8 F0[KT / 16][8], F1[KT / 16][8];
  issue(0, 0);
  if (nsteps > 1) issue(1, 1);
  if (nsteps > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::APW + G::BPW) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (NST == 3 && nsteps > 2) issue(2, 2);
  glds_frags<KT, GN>(lds, 0, wr, wc, r, h, F0);
  // step s with the prefetch of step s+1 (s + 1 < nsteps)
  auto step = [&](int s, bf16x8 (&Fc)[KT / 16][8], bf16x8 (&Fn)[KT / 16][8]) {
    // stage s+1 landed (own pieces; with three stages, stage s+2's stay in flight)
    if (NST == 3 && s + 2 < nsteps)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::APW + G::BPW) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's stage-s reads done
    __builtin_amdgcn_s_barrier();
#ifndef PCFM_CONV_DMA_LATE
#define PCFM_CONV_DMA_LATE 4  // MFMAs per LDS-DMA piece; 0: the burst after the barrier
#endif
#if PCFM_CONV_DMA_LATE > 0
    // LDS-DMA issue (~60-185 cycles per piece) between the MFMAs instead of in
    // a burst after the barrier, where both waves of a SIMD issue theirs at the
    // same time and the MFMA pipe idles: 0.711 -> 0.694 ms (C128 R32 fwd),
    // 0.368 -> 0.357 ms (C256 R16), tools/conv_ab.py on MI355X; 4 MFMAs per
    // piece (over-asking the 16 left after the fragment reads): 0.680 / 0.348 ms
    glds_frags<KT, GN>(lds, (s + 1) % NST, wr, wc, r, h, Fn);
#ifndef PCFM_EXP_CNOMFMA
    glds_mfma<KT>(Fc, acc);
#else
    acc[0][0][0] += (float)Fc[0][0][0];
#endif
    // unconditional (same basic block as the MFMAs, so the scheduler can place
    // the pieces between them): past the last step it reloads the final
    // step's data into the buffer step s just drained (never read again)
#ifndef PCFM_EXP_CNODMA
    // the buffer step s just drained (its fragments were read in step s - 1)
    issue(min(s + NST, nsteps - 1), s % NST);
#endif
#pragma unroll
    for (int g = 0; g < 4 * (KT / 16); ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
#pragma unroll
    for (int g = 0; g < G::APW + G::BPW; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, PCFM_CONV_DMA_LATE, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8 * (KT / 16), 0);
#else
    static_assert(NST == 3, "the burst-issue schedule needs three stages");
#ifndef PCFM_EXP_NOLOAD
    if (s + 3 < nsteps) issue(s + 3, s % kGStages);
#endif
    glds_frags<KT, GN>(lds, (s + 1) % kGStages, wr, wc, r, h, Fn);
    glds_mfma<KT>(Fc, acc);
    // reads of step s+1 interleaved with the first MFMAs of step s (two
    // ds_read_b128 per MFMA gap are free, microarch guide "LDS")
#pragma unroll
    for (int g = 0; g < 4 * (KT / 16); ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 12 * (KT / 16) - 4 * (KT / 16), 0);
#endif
  };
  int s = 0;
  for (; s + 2 < nsteps; s += 2) {
    step(s, F0, F1);
    step(s + 1, F1, F0);
  }
  if (s + 1 < nsteps) {
    step(s, F0, F1);
    glds_mfma<KT>(F1, acc);
  } else {
    glds_mfma<KT>(F0, acc);
  }
  // the interleaved schedule issues (redundant) pieces in the last steps too:
  // none may still be writing LDS when the wave ends
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
  issue(0, 0);
  if (nsteps > 1) issue(1, 1);
  for (int s = 0; s < nsteps; ++s) {
    // stage s landed (this wave's pieces of it): leave stage s+1's in flight
    if (s + 1 < nsteps) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::APW + G::BPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // everyone's stage s landed; stage s-1 reads done
#ifndef PCFM_EXP_NOLOAD
    if (s + 2 < nsteps) issue(s + 2, (s + 2) % kGStages);
#endif
    const uint8_t* base = lds + (s % kGStages) * G::STAGE;
#pragma unroll
    for (int kk = 0; kk < KT / 16; ++kk) {
      const int kc = 2 * kk + h;
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wr * 64 + i * 32 + r;
        const int off = row * G::RB + ((kc ^ G::swz(row)) << 4);
        ah[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(base + off));
        al[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(base + G::A + off));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = wc * 64 + j * 32 + r;
        const int off = 2 * G::A + row * G::RB + ((kc ^ G::swz(row)) << 4);
        bh[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(base + off));
        bl[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(base + G::B + off));
      }
#ifdef PCFM_EXP_NOMFMA
      acc[0][0][kk] += (float)(ah[0][0] + al[0][1] + ah[1][2] + al[1][3] + bh[0][4] + bl[0][5] +
                               bh[1][6] + bl[1][7]);
      continue;
#endif
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
    }
  }
#endif
  }
  float* __restrict__ yb = S == 1 ? y + (size_t)b * M * V : part + ((size_t)sp * nb + b) * M * V;
  float biasv[2][16];
#pragma unroll
  for (int i = 0; i < 2; ++i) load_bias16(S == 1 ? bias : nullptr, m0 + wr * 64 + i * 32, h, M, biasv[i]);
  // this lane's output column per j: dense y[b][m][v0 + col], list y[g / V][m][g % V]
  float* ycol[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = wc * 64 + j * 32 + r;
    if (lmode) {
      const int e = lt * CPT + (col >> lg);
      const long long g = e < lcount ? ((long long)vlist[e] << lg) + (col & lmask) : -1;
      ycol[j] = g >= 0 ? y + (size_t)(g / V) * M * V + (size_t)(g % V) : nullptr;
    } else {
      ycol[j] = yb + v0 + col;
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wr * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (ycol[j] != nullptr) {
#ifndef PCFM_CONV_CACHED_STORE  // streamed: same-box bench 33.70 -> 33.57 ms/step
          nt_st(acc[i][j][e] + biasv[i][e], ycol[j] + (size_t)m * V);
#else
          ycol[j][(size_t)m * V] = acc[i][j][e] + biasv[i][e];
#endif
        }
      }
}

// LDS-DMA as inline asm: hipcc does not see it, so it inserts no vmcnt(0)
// before the step's LDS reads (it does for __builtin_amdgcn_global_load_lds
// here, which serialises the prefetch with the compute); completion is waited
// for by hand.  M0 is set and restored inside the statement.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void glds16_asm(const void* g, uint32_t lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(lds)
      : "memory");
}

// ---------------------------------------------------------------------------
// Small-grid form (r <= 8, the split-K launches): a 256-voxel tile's 27 taps
// read rows of ONE window of the channels-last input, voxels [v0 - H, v0 + 256
// + H) with H = r^2 + r + 1 (416 rows at r = 8), so the window is staged once
// per 32-channel chunk and every tap reads its B fragments at row offset
// H + dx r^2 + dy r + dz of it.  conv3_igemm_glds_kernel instead DMAs the
// tile's 256 shifted rows at every tap: at r = 8 its 6 LDS-DMA pieces per wave
// per step (issue cost, MI355X_MICROARCH.md) against 24 MFMAs set the pace.
// Here a step moves only the weight slice (2 pieces per wave).  A neighbour
// outside the volume (the window holds the linear-index neighbour there) is
// zeroed in registers per lane and tap (the 27-bit validity masks of the
// LDS-DMA kernel).  Same tile, waves, split-K partition (whole chunks per
// split), step order (chunk-major, taps 0..26) and MFMA order as
// conv3_igemm_glds_kernel, whose zero rows give the same zero products: the
// results are bit-identical to it (tests/test_gpu_conv3d.py).
// ---------------------------------------------------------------------------
constexpr int kWinRowsMax = 416;  // 256 + 2 (r^2 + r + 1) rounded up to 16 rows (r = 8)
#ifndef PCFM_CONV_WIN_STAGES
#define PCFM_CONV_WIN_STAGES 3  // 6: 56.0 vs 53.0 us at C256 r = 8 (tools/conv_ab.py)
#endif
constexpr int kWinStages = PCFM_CONV_WIN_STAGES;  // weight slices in flight + 1

__host__ __device__ constexpr int win_rows(int r) {
  return ((kGN + 2 * (r * r + r + 1)) + 15) / 16 * 16;
}

__global__ void __launch_bounds__(512)
    conv3_igemm_win_kernel(const uint16_t* __restrict__ xh, const uint16_t* __restrict__ wh,
                           const float* __restrict__ bias, float* __restrict__ y, int K, int M,
                           int R, int S, float* __restrict__ part) {
  using G = GK<32, kGN>;
  constexpr int kAStage = 2 * G::A;                 // weight slice hi | lo: 16 KiB
  constexpr int kWinImg = kWinRowsMax * G::RB;      // 26 KiB per image
  constexpr int NS = kWinStages;                    // weight ring depth
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t* win = lds;                               // [hi | lo] window images
  uint8_t* aring = lds + 2 * kWinImg;               // kGStages weight stages
  const int V = R * R * R, R2 = R * R, H = R2 + R + 1, WR = win_rows(R);
  const int nmt = M / kGM, nvt = V / kGN;
  int id = (int)blockIdx.x;
  {
    const int nwg = (int)gridDim.x, q = nwg / 8, rr = nwg % 8, xcd = id % 8;
    id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + id / 8;
  }
  const int nb = (int)gridDim.x / (S * nmt * nvt);
  const int m0 = (id % nmt) * kGM;
  id /= nmt;
  const int v0 = (id % nvt) * kGN;
  id /= nvt;
  const int b = id % nb, sp = id / nb;
  const int nch = K / 32;                             // 32-channel chunks
  const int ch0 = nch * sp / S, ch1 = nch * (sp + 1) / S;  // whole chunks (nch % S == 0)
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w / 4, wc = w % 4, r = lane & 31, h = lane >> 5;
  const int prow = lane / G::CPR, pch = lane % G::CPR;
  const size_t bV = (size_t)b * V;
  const uint32_t lds_win = lds_addr(win), lds_ring = lds_addr(aring);

  // weight pieces of this wave: I = 2 w + q (image I / API), as the LDS-DMA kernel
  const uint16_t* abase[G::APW];
#pragma unroll
  for (int q = 0; q < G::APW; ++q) {
    const int I = G::APW * w + q;
    const int row = (I % G::API) * G::RPP + prow;
    abase[q] = wh + (kSplitLo * (I / G::API)) + (size_t)(m0 + row) * 2 * K +
               ((pch ^ G::swz(row)) << 3);
  }
  // this lane's two B columns (j): tap validity, and their window row H + col
  uint32_t bval[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int v = v0 + wc * 64 + j * 32 + r;
    const int x = v / R2, yy = (v / R) % R, z = v % R;
    const uint32_t ax = (x > 0 ? 1u : 0u) | 2u | (x + 1 < R ? 4u : 0u);
    const uint32_t ay = (yy > 0 ? 1u : 0u) | 2u | (yy + 1 < R ? 4u : 0u);
    const uint32_t az = (z > 0 ? 1u : 0u) | 2u | (z + 1 < R ? 4u : 0u);
    uint32_t m = 0u;
#pragma unroll
    for (int tp = 0; tp < 27; ++tp)
      m |= (((ax >> (tp / 9)) & (ay >> ((tp / 3) % 3)) & (az >> (tp % 3))) & 1u) << tp;
    bval[j] = m;
  }

  auto issue_a = [&](int c0, int tap, int slot) {
    const int cof = ((c0 >> 5) << 6) + (c0 & 31);
    const size_t aofs = (size_t)tap * M * 2 * K + cof;
#pragma unroll
    for (int q = 0; q < G::APW; ++q) {
      const int I = G::APW * w + q;
      glds16_asm(abase[q] + aofs,
                 lds_ring + slot * kAStage + (I / G::API) * G::A + (I % G::API) * 1024);
    }
  };
  // the window of chunk c0: WR rows x 2 images in 1-KiB pieces (16 rows), dealt
  // round-robin to the waves; rows outside the batch volume are clamped (their
  // products are masked)
  const int wpieces = 2 * (WR / 16);
  auto issue_win = [&](int c0) {
    const int cof = ((c0 >> 5) << 6) + (c0 & 31);
    for (int P = w; P < wpieces; P += 8) {  // wave-uniform loop
      const int img = P / (WR / 16), pr = P % (WR / 16);
      const int row = pr * 16 + prow;
      const int gv = min(max(v0 - H + row, 0), V - 1);
      const uint16_t* src =
          xh + kSplitLo * img + (bV + gv) * 2 * K + cof + ((pch ^ G::swz(row)) << 3);
      glds16_asm(src, lds_win + img * kWinImg + pr * 1024);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  for (int ch = ch0; ch < ch1; ++ch) {
    const int c0 = ch * 32;
    if (ch > ch0) {
      // every wave is done with the previous chunk's window and weight stages
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    issue_win(c0);
#pragma unroll
    for (int q = 0; q < NS - 1; ++q) issue_a(c0, q, q);
    // B fragments (from the window, which stays put during the chunk) read one
    // step ahead: step s + 1's while step s's MFMAs run
    auto read_b = [&](int s, bf16x8 (&Bf)[2][4]) {
      const int dx = s / 9 - 1, dy = (s / 3) % 3 - 1, dz = s % 3 - 1;
      const int toff = H + dx * R2 + dy * R + dz;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int kc = 2 * kk + h;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int row = wc * 64 + j * 32 + r + toff;
          const int off = row * G::RB + ((kc ^ G::swz(row)) << 4);
          uint4 u0 = *reinterpret_cast<const uint4*>(win + off);
          uint4 u1 = *reinterpret_cast<const uint4*>(win + kWinImg + off);
          const uint32_t mk = ((bval[j] >> s) & 1u) ? 0xFFFFFFFFu : 0u;
          u0.x &= mk; u0.y &= mk; u0.z &= mk; u0.w &= mk;
          u1.x &= mk; u1.y &= mk; u1.z &= mk; u1.w &= mk;
          Bf[kk][j] = __builtin_bit_cast(bf16x8, u0);
          Bf[kk][2 + j] = __builtin_bit_cast(bf16x8, u1);
        }
      }
    };
    auto step = [&](int s, const bf16x8 (&Bc)[2][4], bf16x8 (&Bn)[2][4]) {
      // this wave's pieces of step s (and the window) landed; step s + 1's stay
      // in flight; the barrier makes everyone's visible and ends the reads of
      // step s - 1, whose stage step s + 2 refills
      // this wave's weight pieces of step s landed, the later ones issued so far
      // (min(NS - 2, 26 - s) steps) stay in flight
      switch (min(NS - 2, 26 - s)) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::APW) : "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G::APW) : "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * G::APW) : "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * G::APW) : "memory"); break;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (s + NS - 1 < 27) issue_a(c0, s + NS - 1, (s + NS - 1) % NS);
      const uint8_t* ab = aring + (s % NS) * kAStage;
      if (s + 1 < 27) read_b(s + 1, Bn);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int kc = 2 * kk + h;
        bf16x8 ah[2], al[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int row = wr * 64 + i * 32 + r;
          const int off = row * G::RB + ((kc ^ G::swz(row)) << 4);
          ah[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(ab + off));
          al[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(ab + G::A + off));
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], Bc[kk][j], acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], Bc[kk][2 + j], acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], Bc[kk][j], acc[i][j], 0, 0, 0);
      }
    };
    // the window landed (this wave's pieces: everything but step 1's weights),
    // then everyone's: step 0's B fragments
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 1) * G::APW) : "memory");
    __builtin_amdgcn_s_barrier();
    bf16x8 B0[2][4], B1[2][4];
    read_b(0, B0);
    int s = 0;
    for (; s + 1 < 27; s += 2) {
      step(s, B0, B1);
      step(s + 1, B1, B0);
    }
    step(s, B0, B1);  // s = 26
  }
  float* __restrict__ yb = S == 1 ? y + (size_t)b * M * V : part + ((size_t)sp * nb + b) * M * V;
  float biasv[2][16];
#pragma unroll
  for (int i = 0; i < 2; ++i) load_bias16(S == 1 ? bias : nullptr, m0 + wr * 64 + i * 32, h, M, biasv[i]);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wr * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        nt_st(acc[i][j][e] + biasv[i][e], yb + (size_t)m * V + v0 + wc * 64 + j * 32 + r);
      }
}

// ---------------------------------------------------------------------------
// Forward / backward-data, SLAB form (r = 32, 16; dense unsplit launches).
// Same tile (128 m x 256 voxels, 8 waves of 64 x 64), K-steps (32 channels,
// chunk-major, taps 0..26 in order: the accumulation order of
// conv3_igemm_glds_kernel, so the results are bit-identical) and A operand
// (three-stage LDS-DMA ring of the weight slice) as the LDS-DMA kernel above.
// The difference is the B operand.  There every step DMAs the tile's 256 input
// rows shifted by its tap: 32 KiB per step, 2/3 of the bytes moved and 4 of the
// 6 DMA pieces a wave issues per step (each piece costs 60-185 issue cycles,
// MI355X_MICROARCH.md).  The 256 voxels of a tile are YT = 256 / R whole
// z-rows of one x-plane, so the nine taps of one dx read rows of ONE 2-D slab
// of the plane x + dx: y in [y0 - 1, y0 + YT], z in [-1, R] (zero rows at the
// borders), 340 / 324 rows x 32 channels (hi | lo), 44 KiB.  The slab is
// staged once per (chunk, dx) -- double-buffered, its 42-44 pieces spread one
// per wave-step over the previous slab's nine steps -- and a tap (dy, dz) reads
// its fragments at row offset dy (R + 2) + dz.  Per step a wave issues 2 A
// pieces + 1 slab piece instead of 6, and the block moves 21 KiB instead of 48.
// ---------------------------------------------------------------------------
template <int R_>
struct SlabGeo {
  static constexpr int R = R_, R2 = R * R, V = R * R * R;
  static constexpr int YT = 256 / R;                 // z-rows (y) per tile: 8 / 16
  static constexpr int SZ = R + 2, SY = YT + 2;      // slab extent in z and y
  static constexpr int NS = SY * SZ;                 // 340 / 324 rows
  static constexpr int NSP = (NS + 15) / 16 * 16;    // whole 16-row pieces
  static constexpr int PPI = NSP / 16;               // pieces per image (22 / 21)
  static constexpr int PIECES = 2 * PPI;             // hi + lo
  static constexpr int WQ = (PIECES + 7) / 8;        // slab pieces per wave (6)
  static constexpr int IMG = NSP * 64;               // bytes of one image (64-B rows)
  static constexpr int SLAB = 2 * IMG;
  static constexpr int ASTAGE = GK<32>::STAGE - 2 * GK<32>::B;  // A hi | lo: 16 KiB
  static constexpr int LDS = 3 * ASTAGE + 2 * SLAB;
  static_assert(R * YT == 256 && LDS <= 160 * 1024 && WQ <= 9, "slab geometry");
};

template <int R_>
__global__ void __launch_bounds__(512)
    conv3_igemm_slab_kernel(const uint16_t* __restrict__ xh, const uint16_t* __restrict__ wh,
                            const uint16_t* __restrict__ zrow, const float* __restrict__ bias,
                            float* __restrict__ y, int K, int M) {
  using G = GK<32>;
  using SG = SlabGeo<R_>;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t* aring = lds;                       // 3 x (A hi | A lo)
  uint8_t* slabs = lds + 3 * SG::ASTAGE;      // 2 x (slab hi | slab lo)
  constexpr int R = SG::R, R2 = SG::R2, V = SG::V;
  const int nmt = M / kGM, nvt = V / 256;
  int id = (int)blockIdx.x;
  {
    const int nwg = (int)gridDim.x, q = nwg / 8, rr = nwg % 8, xcd = id % 8;
    id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + id / 8;
  }
  const int m0 = (id % nmt) * kGM;
  id /= nmt;
  const int v0 = (id % nvt) * 256;
  const int b = id / nvt;
  const int x0 = v0 / R2, y0 = (v0 % R2) / R;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w / 4, wc = w % 4, r = lane & 31, h = lane >> 5;
  const int nck = K / 32, T = 27 * nck;
  const int prow = lane / G::CPR, pch = lane % G::CPR;
  const uint16_t* __restrict__ wl = wh + kSplitLo;

  // A pieces (as the LDS-DMA kernel): I = APW w + q -> image I / API, rows (I % API) * RPP + prow
  const uint16_t* abase[G::APW];
#pragma unroll
  for (int q = 0; q < G::APW; ++q) {
    const int I = G::APW * w + q;
    const int row = (I % G::API) * G::RPP + prow;
    abase[q] = ((I / G::API) ? wl : wh) + (size_t)(m0 + row) * 2 * K + ((pch ^ G::swz(row)) << 3);
  }
  // this lane's B fragment rows at tap (0, 0): slab row (yl + 1) SZ + z + 1
  int brow[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = wc * 64 + j * 32 + r;
    brow[j] = (col / R + 1) * SG::SZ + (col % R) + 1;
  }
  const size_t bV = (size_t)b * V;

  // slab sl = (chunk, dx) -> slab buffer sbuf; q: this wave's piece
  // piece q of this wave (I = w + 8 q; a wave with no piece q re-issues its
  // piece 0: same bytes) of slab sl -> slab buffer sbuf.  Lane -> slab row
  // 16 P + prow (y' = y0 - 1 + row / SZ, z' = row % SZ - 1), physical chunk pch;
  // rows outside the volume or past the slab's NS rows read the zero row.
  // Recomputed per step (a per-q table indexed by the runtime q went to scratch)
  auto slab_piece = [&](int sl, int q, int sbuf) {
    int I = w + 8 * q;
    if (I >= SG::PIECES) I = w;
    const int img = I / SG::PPI, P = I % SG::PPI;
    const int row = 16 * P + prow;
    const int ys = row / SG::SZ, zs = row - ys * SG::SZ;
    const int yy = y0 - 1 + ys, zz = zs - 1;
    const int c0 = (sl / 3) * 32, xx = x0 + sl % 3 - 1;
    const bool ok = (unsigned)xx < (unsigned)R && row < SG::NS && (unsigned)yy < (unsigned)R &&
                    (unsigned)zz < (unsigned)R;
    const int cofs = img * 32 + ((pch ^ G::swz(row)) << 3);
    // the plane's first row (uniform; an out-of-volume plane is never read)
    const uint16_t* plane = xh + (bV + (size_t)(xx < 0 ? 0 : xx) * R2) * 2 * K + 2 * c0;
    const unsigned long long src = (unsigned long long)(plane + (yy * R + zz) * 2 * K + cofs);
    const unsigned long long zs64 = (unsigned long long)(zrow + (cofs & 31));
    const uint32_t slo = ok ? (uint32_t)src : (uint32_t)zs64;
    const uint32_t shi = ok ? (uint32_t)(src >> 32) : (uint32_t)(zs64 >> 32);
    glds16((const void*)(((unsigned long long)shi << 32) | slo),
           slabs + sbuf * SG::SLAB + img * SG::IMG + P * 1024);
  };
  auto a_pieces = [&](int s, int buf) {
    const int c0 = (s / 27) * 32, tap = s % 27;
    const int cof = ((c0 >> 5) << 6) + (c0 & 31);
    const size_t aofs = (size_t)tap * M * 2 * K + cof;
#pragma unroll
    for (int q = 0; q < G::APW; ++q) {
      const int I = G::APW * w + q;
      glds16(abase[q] + aofs, aring + buf * SG::ASTAGE + (I / G::API) * G::A + (I % G::API) * 1024);
    }
  };
  // fragments of a step: A from ring slot `ring`, B from slab buffer `sbuf` at
  // the offset of the slab's tap u = 3 (dy + 1) + dz + 1
  auto frags = [&](int ring, int u, int sbuf, bf16x8 (&F)[2][8]) {
    const uint8_t* ab = aring + ring * SG::ASTAGE;
    const int toff = (u / 3 - 1) * SG::SZ + (u % 3 - 1);
    const uint8_t* sb = slabs + sbuf * SG::SLAB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int kc = 2 * kk + h;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wr * 64 + i * 32 + r;
        const int off = row * G::RB + ((kc ^ G::swz(row)) << 4);
        F[kk][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(ab + off));
        F[kk][2 + i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(ab + G::A + off));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = brow[j] + toff;
        const int off = row * G::RB + ((kc ^ G::swz(row)) << 4);
        F[kk][4 + j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sb + off));
        F[kk][6 + j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sb + SG::IMG + off));
      }
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  const int nslab = 3 * nck;  // even (nck even: the launcher's condition)
  // prologue: slab 0 whole, A of steps 0..2
#pragma unroll
  for (int q = 0; q < SG::WQ; ++q) slab_piece(0, q, 0);
  a_pieces(0, 0);
  a_pieces(1, 1);
  a_pieces(2, 2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  bf16x8 F[2][2][8];
  frags(0, 0, 0, F[0]);
  // step s: its fragments are in Fc; read step s + 1's (past the end: unused),
  // run step s's MFMAs, DMA A of step s + 3 into ring s % 3 and one piece of
  // the next slab.  Every step issues exactly APW + 1 pieces (the extra ones
  // re-issue data that is already there or never read again), so the wait at
  // the next step's top is one immediate.
  auto step = [&](int s, bf16x8 (&Fc)[2][8], bf16x8 (&Fn)[2][8]) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::APW + 1) : "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    const int sl = s / 9, u = s - 9 * sl;
    const int un = u == 8 ? 0 : u + 1;
    frags((s + 1) % 3, un, (sl + (u == 8 ? 1 : 0)) & 1, Fn);
    glds_mfma<32>(Fc, acc);
    a_pieces(min(s + 3, T - 1), s % 3);
    slab_piece(min(sl + 1, nslab - 1), min(u, SG::WQ - 1), (sl + 1) & 1);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
#pragma unroll
    for (int g = 0; g < G::APW + 1; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 16 - 4 * (G::APW + 1), 0);
  };
  for (int s = 0; s < T; s += 2) {  // T = 27 nck is even (nck even)
    step(s, F[0], F[1]);
    step(s + 1, F[1], F[0]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may outlive the wave

  float* __restrict__ yb = y + (size_t)b * M * V;
  float biasv[2][16];
#pragma unroll
  for (int i = 0; i < 2; ++i) load_bias16(bias, m0 + wr * 64 + i * 32, h, M, biasv[i]);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float* ycol = yb + v0 + wc * 64 + j * 32 + r;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wr * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        nt_st(acc[i][j][e] + biasv[i][e], ycol + (size_t)m * V);
      }
    }
}

// (Measured and removed: a BRICK form -- 256 output voxels a 2x4x32 / 2x8x16
// brick whose halo sits in LDS once per 16-channel chunk, all 27 taps read from
// it: 1.25x slower, 12 MFMAs per wave between barriers -- and a PING-PONG form
// of the LDS-DMA kernel, waves 0-3 and 4-7 half a step apart: 1.5x slower.
// DESIGN.md section 7; both removed in round 6.)

// ---------------------------------------------------------------------------
// Weight gradient over the channels-last split operands (the forward's split
// input xs and the backward-data pass's split dY): per tap a GEMM reducing over
// voxels, dW[co][ci] = sum_v dY[v][co] * X[v + off][ci], both operands
// row-major [voxel][channel], so the LDS images are the global rows as they lie
// ([64 voxels][128 channels], T10 swizzle) and the MFMA operands (8 consecutive
// voxels per lane) come from ds_read_b64_tr_b16.  Rows whose neighbour is out of
// the grid are zero (padding).  Same 1-D item order, XCD deal and partial
// layout as conv3_wgrad_kernel; 48 MFMAs per wave per 64-voxel step.
// ---------------------------------------------------------------------------
constexpr int kWV = 64;  // voxels per K-step

__global__ void __launch_bounds__(256)
    conv3_wgrad_cl_kernel(const uint16_t* __restrict__ xh, const uint16_t* __restrict__ xl,
                          const uint16_t* __restrict__ gh, const uint16_t* __restrict__ gl,
                          int B, int cin, int cout, int R, int S, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * kWV * 256];
  uint8_t* iAh = lds;
  uint8_t* iAl = lds + kWV * 256;
  uint8_t* iBh = lds + 2 * kWV * 256;
  uint8_t* iBl = lds + 3 * kWV * 256;
  const int V = R * R * R, R2 = R * R;
  const int nco = cout / kMT;
  int id = (int)blockIdx.x;
  {
    const int nwg = (int)gridDim.x, q = nwg / 8, rr = nwg % 8, xcd = id % 8;
    id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + id / 8;
  }
  const int tap = id % 27;
  id /= 27;
  const int sp = id % S;
  id /= S;
  const int co0 = (id % nco) * kMT;
  const int ci0 = (id / nco) * kMT;
  const long long nsteps = (long long)B * V / kWV;
  const long long k0 = nsteps * sp / S, k1 = nsteps * (sp + 1) / S;
  const int dx = tap / 9 - 1, dy_ = (tap / 3) % 3 - 1, dz = tap % 3 - 1;
  const int off = dx * R2 + dy_ * R + dz;

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int ch = t & 15;  // 16-B chunk of the 128-channel row

  StageVec<4> rah, ral, rbh, rbl;
  auto load = [&](long long ks) {
    const long long gv0 = ks * kWV;
    const int b = (int)(gv0 / V), v0 = (int)(gv0 - (long long)b * V);
    const size_t rowA = (size_t)b * V;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = (t >> 4) + 16 * q;
      const int v = v0 + row;
      const size_t ga = split_off(rowA + v, co0 + ch * 8, cout);
      sv_put<4>(rah, q, *reinterpret_cast<const uint4*>(gh + ga));
      sv_put<4>(ral, q, *reinterpret_cast<const uint4*>(gl + ga));
      const int xq = v / R2, yq = (v / R) % R, zq = v % R;
      const bool inb = (unsigned)(xq + dx) < (unsigned)R && (unsigned)(yq + dy_) < (unsigned)R &&
                       (unsigned)(zq + dz) < (unsigned)R;
      const size_t gb = split_off(rowA + (inb ? v + off : v), ci0 + ch * 8, cin);
      const uint4 hv = *reinterpret_cast<const uint4*>(xh + gb);
      const uint4 lv = *reinterpret_cast<const uint4*>(xl + gb);
      sv_put<4>(rbh, q, inb ? hv : uint4{0u, 0u, 0u, 0u});
      sv_put<4>(rbl, q, inb ? lv : uint4{0u, 0u, 0u, 0u});
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int o = swz256((t >> 4) + 16 * q, ch);
      *reinterpret_cast<uint4*>(iAh + o) = sv_get<4>(rah, q);
      *reinterpret_cast<uint4*>(iAl + o) = sv_get<4>(ral, q);
      *reinterpret_cast<uint4*>(iBh + o) = sv_get<4>(rbh, q);
      *reinterpret_cast<uint4*>(iBl + o) = sv_get<4>(rbl, q);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  if (k0 < k1) {
    load(k0);
    store();
  }
  __syncthreads();
  for (long long ks = k0; ks < k1; ++ks) {
#ifndef PCFM_EXP_WG_NOLOAD
    if (ks + 1 < k1) load(ks + 1);
#endif
#pragma unroll
    for (int kk = 0; kk < kWV / 16; ++kk) {
      bf16x8 ah[2], al[2], bh[2], bl[2];
#ifdef PCFM_EXP_WG_NOLDSREAD
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ah[i] = __builtin_bit_cast(bf16x8, sv_get<4>(rah, i));
        al[i] = __builtin_bit_cast(bf16x8, sv_get<4>(ral, i));
        bh[i] = __builtin_bit_cast(bf16x8, sv_get<4>(rbh, i));
        bl[i] = __builtin_bit_cast(bf16x8, sv_get<4>(rbl, i));
      }
#else
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ah[i] = tr_operand(iAh, kk, wr * 64 + i * 32, lane);
        al[i] = tr_operand(iAl, kk, wr * 64 + i * 32, lane);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bh[j] = tr_operand(iBh, kk, wc * 64 + j * 32, lane);
        bl[j] = tr_operand(iBl, kk, wc * 64 + j * 32, lane);
      }
#endif
#ifdef PCFM_EXP_WG_NOMFMA
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j][kk] += (float)ah[i][kk] + (float)bh[j][kk] + (float)al[i][kk] + (float)bl[j][kk];
      continue;
#endif
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
    }
#ifndef PCFM_EXP_WG_NOLOAD
    __syncthreads();
    if (ks + 1 < k1) store();
    __syncthreads();
#endif
  }
  float* pb = part + ((size_t)sp * 27 + tap) * cout * cin;
  const int h = lane >> 5, r = lane & 31;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = co0 + wr * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int ci = ci0 + wc * 64 + j * 32 + r;
        pb[(size_t)co * cin + ci] = acc[i][j][e];
      }
}

// ---------------------------------------------------------------------------
// Weight gradient, three taps per block.  The three taps (dx, dy, dz = -1..1)
// of one (dx, dy) read the SAME dY rows and X rows shifted by one voxel, so a
// block stages dY[v0, v0 + 64) and X[v0 + off - 1, v0 + off + 65) once (66
// rows: the z halo) and its 12 waves -- (dz, 64x64 quadrant) each -- read their
// X operand at row offset 1 + dz.  Global loads and LDS writes per tap drop 3x
// against conv3_wgrad_cl_kernel.  A voxel whose tap leaves the volume has its
// X operand elements zeroed in registers: a lane's 8 K-elements are 8
// consecutive voxels of one z-row (R % 8 == 0), so only x/y validity and the
// first / last element for dz = -1 / +1 matter.  Double-buffered LDS (2 x 65
// KiB), one barrier per step; partials in conv3_wgrad_cl_kernel's layout.
// ---------------------------------------------------------------------------
constexpr int kW3Threads = 768;
constexpr int kW3ARows = kWV;                       // dY rows per step
constexpr int kW3BRows = kWV + 4;                   // X rows: z halo (66), padded to 4-row pieces
constexpr int kW3AImg = kW3ARows * 256;             // bytes of one hi/lo image
constexpr int kW3BImg = kW3BRows * 256;
constexpr int kW3Buf = 2 * kW3AImg + 2 * kW3BImg;   // Ah | Al | Bh | Bl
constexpr int kW3APieces = kW3ARows / 4, kW3BPieces = kW3BRows / 4;  // 1-KiB LDS-DMA pieces
constexpr int kW3Pieces = 2 * kW3APieces + 2 * kW3BPieces;           // 66 per step
constexpr int kW3Q = (kW3Pieces + kW3Threads / 64 - 1) / (kW3Threads / 64);

// tr_operand with an arbitrary first row (row0 + 8 * (lane / 32) ...)
__device__ __forceinline__ bf16x8 tr_operand_rows(const uint8_t* img, int row0, int col0,
                                                  int lane) {
  const int g = lane >> 4, i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;
  const int row = row0 + 8 * (g >> 1) + q4;
  const int col = col0 + (g & 1) * 16 + 4 * p4;
  const v4s_tr x0 = tr_read16(img, swz256(row, col >> 3) + 8 * (p4 & 1));
  const v4s_tr x1 = tr_read16(img, swz256(row + 4, col >> 3) + 8 * (p4 & 1));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ __forceinline__ bf16x8 mask_k8(bf16x8 v, uint32_t m0, uint32_t m12, uint32_t m3) {
  uint4 u = __builtin_bit_cast(uint4, v);
  u.x &= m0;
  u.y &= m12;
  u.z &= m12;
  u.w &= m3;
  return __builtin_bit_cast(bf16x8, u);
}

// Chunk lists of the masked weight gradient: for each (pair, split sp), the
// 64-voxel chunks c = sp, sp + S, sp + 2S, ... whose X operand for that pair is
// nonzero (conv3_occupancy_kernel's cmask), in increasing order -- exactly the
// chunks the unmasked kernel visits, minus those whose products are all exact
// zeros.  grid = (9, S), 64 threads; list row stride `cap`.
__global__ void __launch_bounds__(64)
    conv3_wgrad_lists_kernel(const uint32_t* __restrict__ cmask, int nchunk, int S, int cap,
                             int* __restrict__ lists, int* __restrict__ counts) {
  const int pair = blockIdx.x, sp = blockIdx.y, lane = threadIdx.x;
  int* __restrict__ out = lists + (size_t)(pair * S + sp) * cap;
  int n = 0;
  for (int j0 = 0; sp + (long long)j0 * S < nchunk; j0 += 64) {
    const long long c = sp + (long long)(j0 + lane) * S;
    const bool act = c < nchunk && ((cmask[c] >> pair) & 1u);
    const unsigned long long bal = __ballot(act);
    if (act) out[n + __popcll(bal & ((1ull << lane) - 1ull))] = (int)c;
    n += __popcll(bal);
  }
  if (lane == 0) counts[pair * S + sp] = n;
}

// (Measured, round 5: issuing the next step's pieces between the MFMA groups of
// the step, kW3Q / 4 per 16-voxel K-slice behind sched_barriers, instead of in
// one burst at the step's start: 2.09 vs 2.04 ms/step, same box -- the issue
// burst is not what holds the MFMA pipe at 0.56 busy.)
// kmask (with lists; conv3_occupancy_kernel): a wave skips the 16-voxel
// K-slices whose X rows for its tap are all empty -- products that are exact
// zeros, so the partials keep their bits.  The block's mask words are staged
// in LDS behind the two buffers before the first DMA (a global load inside the
// loop would be waited for with vmcnt(0), draining the DMA pieces in flight).
__global__ void __launch_bounds__(kW3Threads)
    conv3_wgrad3_kernel(const uint16_t* __restrict__ xh, const uint16_t* __restrict__ xl,
                        const uint16_t* __restrict__ gh, const uint16_t* __restrict__ gl,
                        int B, int cin, int cout, int R, int S, float* __restrict__ part,
                        const int* __restrict__ lists, const int* __restrict__ counts, int cap,
                        const uint32_t* __restrict__ kmask) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  // 12 waves = 3 per SIMD at 168 VGPRs each: the CU's whole register file, so
  // no other kernel's wave shares a CU with this block
  static_assert(kW3Threads == 768, "three waves per SIMD");
  PCFM_CLAIM_VGPRS(167);
  const int V = R * R * R, R2 = R * R;
  const int nco = cout / kMT;
  int id = (int)blockIdx.x;
  {
    const int nwg = (int)gridDim.x, q = nwg / 8, rr = nwg % 8, xcd = id % 8;
    id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + id / 8;
  }
  const int pair = id % 9;
  id /= 9;
  const int sp = id % S;
  id /= S;
  const int co0 = (id % nco) * kMT;
  const int ci0 = (id / nco) * kMT;
  // split sp takes the 64-voxel chunks sp, sp + S, ... (of all B * V / 64), or
  // with lists those of them whose X operand is nonzero for this pair
  const int cpb = V / kWV, nchunk = B * cpb;
  const int* __restrict__ lst = lists != nullptr ? lists + (size_t)(pair * S + sp) * cap : nullptr;
  const int nst = lists != nullptr ? counts[pair * S + sp]
                                   : (sp < nchunk ? (nchunk - sp + S - 1) / S : 0);
  const int dx = pair / 3 - 1, dy_ = pair % 3 - 1;
  const int off = dx * R2 + dy_ * R;

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);  // 0..11
  const int dz = w / 4 - 1;
  const int wr = (w >> 1) & 1, wc = w & 1;
  const int h = lane >> 5;

  // LDS-DMA pieces of this wave: I = w + 12 q; lane -> (row 4P + lane / 16,
  // physical chunk lane % 16 = logical chunk ^ swizzle): the swz256 image is
  // produced by choosing the source chunk.  The lane's part of each source
  // address (its row within the step's rows, its chunk, hi / lo) is fixed:
  // built once here, so a step adds one uniform row base (and for X clamps the
  // row) instead of a 64-bit split_off per piece.
  int prow_[kW3Q], pofs[kW3Q];
#pragma unroll
  for (int q = 0; q < kW3Q; ++q) {
    const int I = w + (kW3Threads / 64) * q;
    const bool isA = I < 2 * kW3APieces;
    const int I2 = isA ? I : I - 2 * kW3APieces;
    const int np = isA ? kW3APieces : kW3BPieces;
    const int img = I2 / np, P = I2 % np;
    const int row = 4 * P + (lane >> 4);
    const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
    const int c = (isA ? co0 : ci0) + ch * 8;
    prow_[q] = row;
    // dY pieces: the whole in-step offset (the row is never clamped)
    pofs[q] = ((c >> 5) << 6) + (c & 31) + (img ? kSplitLo : 0) + (isA ? row * 2 * cout : 0);
  }
  // piece q of the step at (b, v0) into buf
  auto issue_q = [&](int q, int b, int v0, uint8_t* buf) {
    const size_t base = (size_t)b * V;
    const int I = w + (kW3Threads / 64) * q;
    if (I < 2 * kW3APieces) {
      const uint16_t* ga = gh + (base + v0) * 2 * cout;  // dY rows of the step
      const int img = I / kW3APieces, P = I % kW3APieces;
      glds16_asm(ga + pofs[q], lds_addr(buf + img * kW3AImg + P * 1024));
    } else if (I < kW3Pieces) {
      const uint16_t* xb = xh + base * 2 * cin;
      const int g0 = v0 + off - 1;  // X row of the halo's first row
      const int I2 = I - 2 * kW3APieces;
      const int img = I2 / kW3BPieces, P = I2 % kW3BPieces;
      const int gv = min(max(g0 + prow_[q], 0), V - 1);  // out-of-volume rows are masked at use
      glds16_asm(xb + ((size_t)gv * 2 * cin + pofs[q]),
                 lds_addr(buf + 2 * kW3AImg + img * kW3BImg + P * 1024));
    }
  };
  auto issue = [&](int b, int v0, uint8_t* buf) {
#pragma unroll
    for (int q = 0; q < kW3Q; ++q) issue_q(q, b, v0, buf);
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  auto chunk_of = [&](int st) { return lst != nullptr ? lst[st] : sp + st * S; };
  const int lgR = 31 - __builtin_clz(R);  // R is a power of two here
  // the 4 K-slice mask words of every listed chunk (kmask: with lists only)
  uint32_t* kms = reinterpret_cast<uint32_t*>(lds + 2 * kW3Buf);
  const bool skip = kmask != nullptr && lst != nullptr;
  if (skip) {
    for (int i = t; i < 4 * nst; i += kW3Threads) {
      const int c = lst[i >> 2];
      kms[i] = kmask[(size_t)(c / cpb) * (V / 16) + (size_t)(c % cpb) * (kWV / 16) + (i & 3)];
    }
    __syncthreads();
  }
  const int mytap = pair * 3 + (dz + 1);
  int cnext = nst > 0 ? chunk_of(0) : 0;
  if (nst > 0) issue(cnext / cpb, (cnext % cpb) * kWV, lds);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int st = 0; st < nst; ++st) {
    __builtin_amdgcn_s_barrier();  // step st landed everywhere; step st-1 reads done
    const uint8_t* cur = lds + (st & 1) * kW3Buf;
    const int v0 = (cnext % cpb) * kWV;
    const bool more = st + 1 < nst;
    if (more) cnext = chunk_of(st + 1);
    const int nb = cnext / cpb, nv0 = (cnext % cpb) * kWV;
    uint8_t* nbuf = lds + ((st + 1) & 1) * kW3Buf;
#ifndef PCFM_EXP_WG_NOLOAD
    if (more) issue(nb, nv0, nbuf);
#endif
    const uint8_t* iAh = cur;
    const uint8_t* iAl = cur + kW3AImg;
    const uint8_t* iBh = cur + 2 * kW3AImg;
    const uint8_t* iBl = iBh + kW3BImg;
    uint32_t kw = 0xFu;  // K-slices of this step with a nonzero X operand (bit kk)
    if (skip) {
      const uint4 q = *reinterpret_cast<const uint4*>(kms + 4 * st);
      kw = ((q.x >> mytap) & 1u) | (((q.y >> mytap) & 1u) << 1) | (((q.z >> mytap) & 1u) << 2) |
           (((q.w >> mytap) & 1u) << 3);
      kw = __builtin_amdgcn_readfirstlane(kw);
    }
#pragma unroll
    for (int kk = 0; kk < kWV / 16; ++kk) {
      if (!((kw >> kk) & 1u)) continue;  // wave-uniform: exact-zero products skipped
      // validity of this lane's 8 voxels for tap (dx, dy, dz)
      const int vk = v0 + kk * 16 + 8 * h;
      const int xq = vk >> (2 * lgR), yq = (vk >> lgR) & (R - 1), z0 = vk & (R - 1);
      const bool xyok = (unsigned)(xq + dx) < (unsigned)R && (unsigned)(yq + dy_) < (unsigned)R;
      const uint32_t mall = xyok ? 0xFFFFFFFFu : 0u;
      const uint32_t m0 = (dz < 0 && z0 == 0) ? (mall & 0xFFFF0000u) : mall;
      const uint32_t m3 = (dz > 0 && z0 + 8 == R) ? (mall & 0x0000FFFFu) : mall;
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ah[i] = tr_operand_rows(iAh, kk * 16, wr * 64 + i * 32, lane);
        al[i] = tr_operand_rows(iAl, kk * 16, wr * 64 + i * 32, lane);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bh[j] = mask_k8(tr_operand_rows(iBh, kk * 16 + 1 + dz, wc * 64 + j * 32, lane), m0, mall,
                        m3);
        bl[j] = mask_k8(tr_operand_rows(iBl, kk * 16 + 1 + dz, wc * 64 + j * 32, lane), m0, mall,
                        m3);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // step ks+1 landed (this wave's pieces)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  const int tap = pair * 3 + (dz + 1);
  float* pb = part + ((size_t)sp * 27 + tap) * cout * cin;
  const int r = lane & 31;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = co0 + wr * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int ci = ci0 + wc * 64 + j * 32 + r;
        pb[(size_t)co * cin + ci] = acc[i][j][e];
      }
}

// dw[co][ci][tap] = sum_s part[s][tap][co][ci], in split order.  A block owns
// 64 consecutive (co, ci) pairs x 27 taps: partial rows are read coalesced
// (64 pairs of one tap), the [64][27] result goes out through LDS as one
// contiguous run of dw.  grid = ceil(cout * cin / 64), 256 threads.
__global__ void __launch_bounds__(256)
    conv3_wgrad_reduce_kernel(const float* __restrict__ part, int cout, int cin, int S,
                              float* __restrict__ dw) {
  __shared__ float tile[64 * 27];
  const size_t pairs = (size_t)cout * cin;
  const size_t cc0 = (size_t)blockIdx.x * 64;
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const size_t cc = cc0 + cl;
  const size_t ps = 27 * pairs;  // one split's partial
  // this thread's taps grp, grp + 4, ... (7 at most) accumulate side by side:
  // per split q all their partials are loaded before any is added, two splits
  // per round (each tap's sum keeps the split order)
  constexpr int kT = 7;
  float sum[kT];
#pragma unroll
  for (int k = 0; k < kT; ++k) sum[k] = 0.0f;
  if (cc < pairs) {
    const float* p = part + cc;
    auto tap_of = [&](int k) { return min(grp + 4 * k, 26); };
    int q = 0;
    for (; q + 2 <= S; q += 2) {
      float a[2][kT];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int k = 0; k < kT; ++k)
          a[u][k] = p[(size_t)(q + u) * ps + (size_t)tap_of(k) * pairs];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int k = 0; k < kT; ++k) sum[k] = sum[k] + a[u][k];
    }
    for (; q < S; ++q)
#pragma unroll
      for (int k = 0; k < kT; ++k) sum[k] = sum[k] + p[(size_t)q * ps + (size_t)tap_of(k) * pairs];
  }
#pragma unroll
  for (int k = 0; k < kT; ++k)
    if (grp + 4 * k < 27) tile[cl * 27 + grp + 4 * k] = sum[k];
  __syncthreads();
  const size_t n = (min(pairs, cc0 + 64) - cc0) * 27;
  for (size_t e = threadIdx.x; e < n; e += 256) dw[cc0 * 27 + e] = tile[e];
}

#ifndef PCFM_WGRAD_OCC
#define PCFM_WGRAD_OCC 4
#endif
#ifndef PCFM_WGRAD3_BLOCKS
#define PCFM_WGRAD3_BLOCKS 2  // blocks per CU the three-tap split aims for
#endif
bool conv3_wgrad3_ok(int R) {
#ifdef PCFM_WGRAD_NO3
  return false;
#else
  return R >= 8 && (R & (R - 1)) == 0;  // 8-voxel z runs, shift-decoded voxel index
#endif
}

int conv3_wgrad_splits(int B, int cin, int cout, int R) {
  if (conv3_wgrad3_ok(R)) {
    // one 768-thread block per CU: pick the split minimising
    // (rounds of blocks over the CUs) x (K-steps per block), i.e. no lone tail round
    const long long items = 9LL * (cout / kMT) * (cin / kMT);
    const long long steps = (long long)B * R * R * R / kWV;
    const long long smax = std::min(64LL, std::max(1LL, steps / 8));
    // model: ~4 us per K-step; each split adds its partial (27 cout cin fp32),
    // written then read by the reduce, at ~5 TB/s
    const double part_us = 2.0 * 27.0 * cout * cin * 4.0 / 5.0e6;
    long long best = 1;
    double best_cost = -1.0;
    for (long long s = 1; s <= smax; ++s) {
      const long long rounds = (items * s + kCUs - 1) / kCUs;
      const double cost = 4.0 * rounds * ((steps + s - 1) / s) + part_us * s;
      if (best_cost < 0 || cost < best_cost) best = s, best_cost = cost;
    }
    return (int)best;
  }
  const long long tiles = 27LL * (cout / kMT) * (cin / kMT);
  const long long steps = (long long)B * R * R * R / kWV;
  // blocks per CU the split aims for (one block's staging overlaps another's MFMAs)
  long long s = std::max(1LL, ((long long)PCFM_WGRAD_OCC * kCUs + tiles - 1) / tiles);
  s = std::min(s, std::max(1LL, steps / 8));  // keep >= 8 K-steps per block
  return (int)std::min(s, 64LL);
}

bool conv3_shape_ok(int b, int cin, int cout, int r) {
  if (b < 0 || cin <= 0 || cout <= 0 || r <= 0 || r > 1024) return false;
  const long long v = (long long)r * r * r;
  return cin % 64 == 0 && cout % kMT == 0 && v % kNT == 0 && v < (1LL << 31);
}

}  // namespace
}  // namespace pcfm

using namespace pcfm;

extern "C" size_t pcfm_conv3d_weight_bytes(int cout, int cin) {
  if (cout <= 0 || cin <= 0) return 0;
  return (size_t)2 * 27 * cout * cin * sizeof(uint16_t);
}

extern "C" int pcfm_conv3d_prep_weight(const float* w, int cout, int cin, int transpose,
                                       void* wsplit, void* stream) {
  PCFM_CHECK_ARG(cout > 0 && cin > 0 && (transpose ? cout : cin) % 32 == 0,
                 "conv3d_prep_weight: unsupported size cout=%d cin=%d (the GEMM's K %% 32 == 0)", cout,
                 cin);
  const size_t total = (size_t)27 * cout * cin;
  uint16_t* wh = (uint16_t*)wsplit;
  hipLaunchKernelGGL(conv3_wsplit_kernel, dim3(ceil_div((long long)total, 256)), dim3(256), 0,
                     (hipStream_t)stream, w, cout, cin, transpose ? 1 : 0, wh);
  return check_launch("conv3d_prep_weight");
}

extern "C" int pcfm_conv3d_supported(int b, int cin, int cout, int r) {
  return conv3_shape_ok(b, cin, cout, r) ? 1 : 0;
}

#ifndef PCFM_CONV_KT
#define PCFM_CONV_KT 64
#endif

// One 256-B zero buffer per device (the LDS-DMA source of out-of-grid rows).
static const uint16_t* zero_row() {
  static std::mutex mu;
  static const uint16_t* rows[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (rows[dev] == nullptr) {
    void* p = nullptr;
    if (hipMalloc(&p, 256) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, 256) != hipSuccess) return nullptr;
    rows[dev] = (const uint16_t*)p;
  }
  return rows[dev];
}

static size_t split_bytes_al(int b, int cin, int r) {
  return ((size_t)2 * b * r * r * r * cin * sizeof(uint16_t) + 255) / 256 * 256;
}

extern "C" size_t pcfm_conv3d_igemm_workspace_bytes(int b, int cin, int cout, int r) {
  if (!conv3_shape_ok(b, cin, cout, r) || cin % 64 != 0) return 0;
  return split_bytes_al(b, cin, r) + pcfm_conv3d_igemm_cl_workspace_bytes(b, cin, cout, r);
}

extern "C" int pcfm_conv3d_igemm(const float* x, const void* wsplit, const float* bias, int b,
                                 int cin, int cout, int r, float* y, void* ws, size_t ws_bytes,
                                 void* stream) {
  PCFM_CHECK_ARG(conv3_shape_ok(b, cin, cout, r),
                 "conv3d_igemm: unsupported shape b=%d cin=%d cout=%d r=%d (need cin %% 64, "
                 "cout %% %d, r^3 %% %d == 0)",
                 b, cin, cout, r, kMT, kNT);
  if (b == 0) return PCFM_OK;
  const size_t need = pcfm_conv3d_igemm_workspace_bytes(b, cin, cout, r);
  PCFM_CHECK_ARG(ws_bytes >= need, "conv3d_igemm: workspace %zu < %zu bytes", ws_bytes, need);
  const int rc = pcfm_conv3d_split(x, b, cin, r, ws, stream);
  const size_t so = split_bytes_al(b, cin, r);
  return rc != PCFM_OK ? rc
                       : pcfm_conv3d_igemm_cl(ws, wsplit, bias, b, cin, cout, r, y,
                                              (uint8_t*)ws + so, ws_bytes - so, stream);
}

static size_t wgrad_partial_bytes(int b, int cin, int cout, int r) {
  return (size_t)conv3_wgrad_splits(b, cin, cout, r) * 27 * cout * cin * sizeof(float);
}

extern "C" size_t pcfm_conv3d_wgrad_workspace_bytes(int b, int cin, int cout, int r) {
  if (b <= 0 || !conv3_shape_ok(b, cin, cout, r) || cin % kMT != 0) return 0;
  // split-operand partials, plus room for split(x) and split(grad_y) when the
  // fp32 entry point (pcfm_conv3d_wgrad) makes them itself
  const size_t v = (size_t)r * r * r;
  return wgrad_partial_bytes(b, cin, cout, r) + 4 * (size_t)b * v * (cin + cout);
}

extern "C" int pcfm_conv3d_wgrad(const float* x, const float* grad_y, int b, int cin, int cout,
                                 int r, float* grad_w, void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(b > 0 && conv3_shape_ok(b, cin, cout, r) && cin % kMT == 0,
                 "conv3d_wgrad: unsupported shape b=%d cin=%d cout=%d r=%d", b, cin, cout, r);
  const size_t need = pcfm_conv3d_wgrad_workspace_bytes(b, cin, cout, r);
  PCFM_CHECK_ARG(ws_bytes >= need, "conv3d_wgrad: workspace %zu < %zu bytes", ws_bytes, need);
  const size_t v = (size_t)r * r * r;
  char* xs = (char*)ws + wgrad_partial_bytes(b, cin, cout, r);
  char* gys = xs + 4 * (size_t)b * v * cin;
  int rc = pcfm_conv3d_split(x, b, cin, r, xs, stream);
  if (rc == PCFM_OK) rc = pcfm_conv3d_split(grad_y, b, cout, r, gys, stream);
  if (rc == PCFM_OK)
    rc = pcfm_conv3d_wgrad_cl(xs, gys, b, cin, cout, r, grad_w, ws,
                              wgrad_partial_bytes(b, cin, cout, r), stream);
  return rc;
}

extern "C" size_t pcfm_conv3d_split_bytes(int b, int c, int r) {
  if (b <= 0 || c <= 0 || c % 64 != 0 || r <= 0 || ((long long)r * r * r) % 64 != 0) return 0;
  return (size_t)2 * b * r * r * r * c * sizeof(uint16_t);
}

extern "C" int pcfm_conv3d_split(const float* x, int b, int c, int r, void* xs, void* stream) {
  PCFM_CHECK_ARG(pcfm_conv3d_split_bytes(b, c, r) > 0, "conv3d_split: bad shape b=%d c=%d r=%d",
                 b, c, r);
  const int V = r * r * r;
  uint16_t* xh = (uint16_t*)xs;
  hipLaunchKernelGGL(conv3_split_cl_kernel, dim3(V / 64, c / 64, b), dim3(256), 0,
                     (hipStream_t)stream, x, c, V, xh);
  return check_launch("conv3d_split");
}

// split-K count of the 64 x 64 tile path (small grids: r = 8): enough blocks
// to fill the chip, >= 8 K-steps each
static int igemm_splits(int b, int cin, int cout, int r) {
  const int V = r * r * r;
  const long long blocks = (long long)(V / 64) * (cout / 64) * b;
  const long long nall = 27LL * (cin / PCFM_CONV_KT);
  long long s = std::max(1LL, (4LL * kCUs + blocks - 1) / blocks);
  s = std::min(s, std::max(1LL, nall / 8));
  return (int)std::min(s, 8LL);
}

static bool igemm_big(int b, int cout, int r) {
  const int V = r * r * r;
  const long long big_blocks = (long long)(V / 128) * (cout / 128) * b;
  return big_blocks >= 2 * kCUs;
}

#ifndef PCFM_CONV_GLDS_MINV
#define PCFM_CONV_GLDS_MINV 512  // 4096: r = 8 on the 64x64-tile kernel instead
#endif
// LDS-DMA kernel applies (128 x 256 tiles); small grids (r = 8) split K so
// that about one block per CU runs, >= 8 K-steps per split, ordered reduce.
static bool glds_ok(int cout, int r) {
  const int V = r * r * r;
  return V % kGN == 0 && V >= PCFM_CONV_GLDS_MINV && cout % kGM == 0;
}

static int glds_splits(int b, int cin, int cout, int r) {
  const int V = r * r * r;
  const long long items = (long long)(V / kGN) * (cout / kGM) * b;
  const long long nall = 27LL * (cin / 16);  // K-steps at KT = 16 (the shorter bound)
  long long s = std::max(1LL, (long long)kCUs / std::max(1LL, items));
  s = std::min(s, std::max(1LL, nall / 16));
  return (int)std::min(s, 8LL);
}

extern "C" size_t pcfm_conv3d_igemm_cl_workspace_bytes(int b, int cin, int cout, int r) {
  if (!conv3_shape_ok(b, cin, cout, r)) return 0;
  if (b == 0) return 1;
#ifndef PCFM_CONV_NOGLDS
  if (glds_ok(cout, r)) {
    const int S = glds_splits(b, cin, cout, r);
    return S == 1 ? 1 : (size_t)S * b * cout * r * r * r * sizeof(float);
  }
#endif
  if (igemm_big(b, cout, r)) return 1;
  const int S = igemm_splits(b, cin, cout, r);
  return S == 1 ? 1 : (size_t)S * b * cout * r * r * r * sizeof(float);
}



// Slab form of the dense r = 32 / 16 launches (PCFM_CONV_SLAB=0: the LDS-DMA
// kernel that refetches B per tap)
static bool conv_slab() {
  const char* e = getenv("PCFM_CONV_SLAB");  // read per call: tests compare both forms
  return e == nullptr || e[0] != '0';
}

// Window form of the small-grid split-K launches (PCFM_CONV_WIN=0: the
// LDS-DMA kernel that refetches B per tap)
static bool conv_win() {
  const char* e = getenv("PCFM_CONV_WIN");  // read per call: tests compare both forms
  return e == nullptr || e[0] != '0';
}


// List-form tile in voxels, per direction (env PCFM_LIST_GN_FWD / _BWD = 256 or
// 128, read per call: A/B runs).  The backward-data's list (the occupied
// voxels, 12 % at r = 32, 21 % at r = 16) fills only ~120 / ~110 blocks of
// 256 voxels -- half the CUs idle -- so it takes 128-voxel tiles: 0.89 -> 0.70
// ms/step; the forward's longer list (30 % / 50 %) is slower on them (1.17 ->
// 1.34), profiles/r06_ab_list_gn128.jsonl.  PCFM_LIST_NST: 3 / 2 LDS-DMA
// stages at 128 (2: two blocks per CU; measured slower, 0.85 ms).
static int list_gn(int which) {
  const char* e = getenv(which == 0 ? "PCFM_LIST_GN_BWD" : "PCFM_LIST_GN_FWD");
  if (e != nullptr) return atoi(e) == 128 ? 128 : 256;
  return which == 0 ? 128 : 256;
}
static int list_nst() {
  const char* e = getenv("PCFM_LIST_NST");
  return e != nullptr && atoi(e) == 2 ? 2 : 3;
}

static int igemm_cl(const void* xs, const void* wsplit, const float* bias, int b, int cin,
                    int cout, int r, float* y, void* ws, size_t ws_bytes, void* stream,
                    const uint32_t* tmask, int mmode, const int* vlist = nullptr,
                    const int* vcount = nullptr, int lg = 5, const uint32_t* obits = nullptr,
                    int lgn = 256) {
  PCFM_CHECK_ARG(conv3_shape_ok(b, cin, cout, r),
                 "conv3d_igemm_cl: unsupported shape b=%d cin=%d cout=%d r=%d", b, cin, cout, r);
  if (b == 0) return PCFM_OK;
  const int V = r * r * r;
  const uint16_t* wh = (const uint16_t*)wsplit;
  const uint16_t* xh = (const uint16_t*)xs;
  const uint16_t* xl = xh + kSplitLo;  // interleaved hi / lo (split_off)
  hipStream_t st = (hipStream_t)stream;
  const long long big_blocks = (long long)(V / 128) * (cout / 128) * b;
#ifndef PCFM_CONV_NOGLDS
  if (glds_ok(cout, r)) {
    const int S = glds_splits(b, cin, cout, r);
    const long long glds_blocks = (long long)(V / kGN) * (cout / kGM) * b * S;
    const size_t need = pcfm_conv3d_igemm_cl_workspace_bytes(b, cin, cout, r);
    PCFM_CHECK_ARG(S == 1 || (ws != nullptr && ws_bytes >= need),
                   "conv3d_igemm_cl: workspace %zu < %zu bytes", ws_bytes, need);
    float* part = S == 1 ? nullptr : (float*)ws;
    const uint16_t* zrow = zero_row();  // 64 B of zeros: the padding row
    if (zrow == nullptr) {
      set_error("conv3d_igemm_cl: zero-row allocation failed");
      return (int)hipErrorOutOfMemory;
    }
#ifndef PCFM_CONV_GK
#define PCFM_CONV_GK 32  // 16: two blocks per CU, measured 1.15-1.18x slower
#endif
    // tile masks apply to unsplit launches only (a split's K range is a fixed
    // share of all 27 taps)
    const int mm = S == 1 && tmask != nullptr ? mmode : 0;
    const int* vl = S == 1 ? vlist : nullptr;  // the list form is unsplit
    const int* vc = S == 1 ? vcount : nullptr;
    if (S == 1 && mm == 0 && vl == nullptr && cin % 64 == 0 && (r == 32 || r == 16) &&
        conv_slab()) {  // cin % 64: an even number of 32-channel chunks (the step loop's pairs)
      const int e = r == 32 ? allow_big_lds((const void*)conv3_igemm_slab_kernel<32>)
                            : allow_big_lds((const void*)conv3_igemm_slab_kernel<16>);
      if (e) return e;
      if (r == 32)
        hipLaunchKernelGGL(conv3_igemm_slab_kernel<32>, dim3((unsigned)glds_blocks), dim3(512),
                           SlabGeo<32>::LDS, st, xh, wh, zrow, bias, y, cin, cout);
      else
        hipLaunchKernelGGL(conv3_igemm_slab_kernel<16>, dim3((unsigned)glds_blocks), dim3(512),
                           SlabGeo<16>::LDS, st, xh, wh, zrow, bias, y, cin, cout);
      return check_launch("conv3d_igemm_cl");
    }
    if (mm == 0 && vl == nullptr && cin % 32 == 0 && r <= 8 && win_rows(r) <= kWinRowsMax &&
        (cin / 32) % S == 0 && conv_win()) {
      const size_t lds = 2 * (size_t)kWinRowsMax * 64 + (size_t)kWinStages * 2 * kGM * 64;
      const int e = allow_big_lds((const void*)conv3_igemm_win_kernel);
      if (e) return e;
      hipLaunchKernelGGL(conv3_igemm_win_kernel, dim3((unsigned)glds_blocks), dim3(512), lds, st,
                         xh, wh, bias, y, cin, cout, r, S, part);
      if (S > 1) {
        const long long total4 = (long long)b * cout * V / 4;
        hipLaunchKernelGGL(conv3_ksum_kernel, dim3((unsigned)ceil_div(total4, 256)), dim3(256), 0,
                           st, (const float*)part, bias, S, cout, V, total4, y);
      }
      return check_launch("conv3d_igemm_cl");
    }
    if (vl != nullptr && cin % 32 == 0 && lgn == 128) {
      // list form on 128-voxel tiles (list_gn): twice the blocks
      const long long lblocks = (long long)(V / 128) * (cout / kGM) * b;
      if (list_nst() == 2)
        hipLaunchKernelGGL((conv3_igemm_glds_kernel<32, 128, 2>), dim3((unsigned)lblocks),
                           dim3(256), 0, st, xh, xl, wh, wh + kSplitLo, zrow, bias, y, cin, cout,
                           r, S, part, tmask, mm, vl, vc, lg, obits);
      else
        hipLaunchKernelGGL((conv3_igemm_glds_kernel<32, 128, 3>), dim3((unsigned)lblocks),
                           dim3(256), 0, st, xh, xl, wh, wh + kSplitLo, zrow, bias, y, cin, cout,
                           r, S, part, tmask, mm, vl, vc, lg, obits);
      return check_launch("conv3d_igemm_cl");
    }
    if (PCFM_CONV_GK == 16 || cin % 32 != 0)
      hipLaunchKernelGGL(conv3_igemm_glds_kernel<16>, dim3((unsigned)glds_blocks), dim3(512), 0,
                         st, xh, xl, wh, wh + kSplitLo, zrow, bias, y, cin, cout, r, S, part, tmask,
                         mm, vl, vc, lg, S == 1 ? obits : nullptr);
    else
      hipLaunchKernelGGL(conv3_igemm_glds_kernel<32>, dim3((unsigned)glds_blocks), dim3(512), 0,
                         st, xh, xl, wh, wh + kSplitLo, zrow, bias, y, cin, cout, r, S, part, tmask,
                         mm, vl, vc, lg, S == 1 ? obits : nullptr);
    if (S > 1) {
      const long long total4 = (long long)b * cout * V / 4;
      hipLaunchKernelGGL(conv3_ksum_kernel, dim3((unsigned)ceil_div(total4, 256)), dim3(256), 0,
                         st, (const float*)part, bias, S, cout, V, total4, y);
    }
    return check_launch("conv3d_igemm_cl");
  }
#endif
  if (big_blocks >= 2 * kCUs) {
    hipLaunchKernelGGL((conv3_igemm_cl_kernel<128, 128, PCFM_CONV_KT>),
                       dim3((V / 128) * (cout / 128) * b), dim3(256), 0, st, xh, xl, wh, wh + kSplitLo,
                       bias, y, cin, cout, r, 1, nullptr);
  } else {
    const int S = igemm_splits(b, cin, cout, r);
    const size_t need = pcfm_conv3d_igemm_cl_workspace_bytes(b, cin, cout, r);
    PCFM_CHECK_ARG(S == 1 || (ws != nullptr && ws_bytes >= need),
                   "conv3d_igemm_cl: workspace %zu < %zu bytes", ws_bytes, need);
    const int items = (V / 64) * (cout / 64) * b;
    hipLaunchKernelGGL((conv3_igemm_cl_kernel<64, 64, PCFM_CONV_KT>), dim3(items * S), dim3(256),
                       0, st, xh, xl, wh, wh + kSplitLo, bias, y, cin, cout, r, S, (float*)ws);
    if (S > 1) {
      const long long total4 = (long long)b * cout * V / 4;
      hipLaunchKernelGGL(conv3_ksum_kernel, dim3((unsigned)ceil_div(total4, 256)), dim3(256), 0,
                         st, (const float*)ws, bias, S, cout, V, total4, y);
    }
  }
  return check_launch("conv3d_igemm_cl");
}

extern "C" int pcfm_conv3d_igemm_cl(const void* xs, const void* wsplit, const float* bias, int b,
                                    int cin, int cout, int r, float* y, void* ws,
                                    size_t ws_bytes, void* stream) {
  return igemm_cl(xs, wsplit, bias, b, cin, cout, r, y, ws, ws_bytes, stream, nullptr, 0);
}

extern "C" int pcfm_conv3d_igemm_cl_occ(const void* xs, const void* wsplit, const float* bias,
                                        int b, int cin, int cout, int r, const unsigned* tmask,
                                        int mode, float* y, void* ws, size_t ws_bytes,
                                        void* stream) {
  PCFM_CHECK_ARG(tmask != nullptr && (mode == 1 || mode == 2) && (r * r * r) % 256 == 0,
                 "conv3d_igemm_cl_occ: need a tile mask, mode 1 or 2 and r^3 %% 256 == 0 "
                 "(mode=%d r=%d)", mode, r);
  return igemm_cl(xs, wsplit, bias, b, cin, cout, r, y, ws, ws_bytes, stream,
                  (const uint32_t*)tmask, mode);
}

extern "C" size_t pcfm_conv3d_occupancy_bytes(int b, int r) {
  const long long v = (long long)r * r * r;
  if (b <= 0 || r <= 0 || v % 256 != 0) return 0;
  return (size_t)b * (v / 256 + v / 64 + v / 16) * sizeof(uint32_t);
}

extern "C" int pcfm_conv3d_occupancy(const int* cnt, int b, int r, unsigned* masks,
                                     void* stream) {
  PCFM_CHECK_ARG(pcfm_conv3d_occupancy_bytes(b, r) > 0,
                 "conv3d_occupancy: bad shape b=%d r=%d (r^3 %% 256 == 0)", b, r);
  const int V = r * r * r;
  hipLaunchKernelGGL(conv3_occupancy_kernel, dim3(V / 256, b), dim3(256), 0, (hipStream_t)stream,
                     cnt, r, (uint32_t*)masks, (uint32_t*)masks + (size_t)b * (V / 256),
                     (uint32_t*)masks + (size_t)b * (V / 256 + V / 64));
  return check_launch("conv3d_occupancy");
}

// Buffer: int32 counts[4] | pad to 64 | per-tile counts / offsets [2][tiles] |
// list 0 [B V / 32] | list 1 [B V / 32] | per-tile counts / offsets of lists 2, 3
// [2][tiles] | list 2 [B V] (the occupied voxels, global indices b V + v) |
// list 3 [B V] (the voxels with an occupied voxel in their 3x3x3 neighbourhood)
// | bitmaps of lists 2, 3 [2][B V / 32] (bit v & 31 of word v >> 5).
extern "C" size_t pcfm_conv3d_vlist_bytes(int b, int r) {
  const long long v = (long long)r * r * r;
  if (b <= 0 || r <= 0 || v % 256 != 0 || (long long)b * v >= (1LL << 31)) return 0;
  const long long tiles = (long long)b * v / 256;
  return (size_t)(64 + 4 * tiles + 4 * (long long)b * v / kChunk + 2 * (long long)b * v) *
         sizeof(int);
}

extern "C" int pcfm_conv3d_vlist(const int* cnt, int b, int r, int* lists, void* stream) {
  PCFM_CHECK_ARG(pcfm_conv3d_vlist_bytes(b, r) > 0,
                 "conv3d_vlist: bad shape b=%d r=%d (r^3 %% 256 == 0, b r^3 < 2^31)", b, r);
  const int V = r * r * r, tiles = b * (V / 256);
  hipStream_t st = (hipStream_t)stream;
  int* tc = lists + 64;
  int* l0 = tc + 2 * tiles;
  int* tc2 = l0 + 2 * ((size_t)b * V / kChunk);
  int* l2 = tc2 + 2 * tiles;
  hipLaunchKernelGGL(conv3_vlist_count_kernel, dim3(tiles), dim3(256), 0, st, cnt, r, tiles, tc,
                     tc2);
  hipLaunchKernelGGL(conv3_vlist_scan_kernel, dim3(1), dim3(1024), 0, st, tc, tiles, lists, 2);
  hipLaunchKernelGGL(conv3_vlist_scan_kernel, dim3(1), dim3(1024), 0, st, tc2, tiles, lists + 2,
                     2);
  uint32_t* bits = (uint32_t*)(l2 + 2 * (size_t)b * V);
  hipLaunchKernelGGL(conv3_vlist_write_kernel, dim3(tiles), dim3(256), 0, st, cnt, r, tiles, tc,
                     l0, l0 + (size_t)b * V / kChunk, (const int*)tc2, l2, l2 + (size_t)b * V,
                     bits, bits + (size_t)b * V / kChunk);
  return check_launch("conv3d_vlist");
}

// The list forms over single voxels (lists 2 / 3) instead of 32-voxel chunks
// (lists 0 / 1): env PCFM_LIST_VOX bit 0 = backward-data (which 0), bit 1 =
// forward (which 1); default 3; read per call (A/B runs).  At the C2 stages an
// occupied chunk holds 27 % (r = 32) / 36 % (r = 16) occupied voxels, and a
// listed forward chunk 49 % / 61 % active voxels.
static int list_vox() {
  const char* e = getenv("PCFM_LIST_VOX");
  return e == nullptr ? 3 : (atoi(e) & 3);
}

extern "C" int pcfm_conv3d_igemm_cl_list(const void* xs, const void* wsplit, const float* bias,
                                         int b, int cin, int cout, int r, const int* cnt,
                                         const int* lists, int which, float* y, void* ws,
                                         size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(cnt != nullptr && lists != nullptr && (which == 0 || which == 1) &&
                     pcfm_conv3d_vlist_bytes(b, r) > 0,
                 "conv3d_igemm_cl_list: need counts, lists, which 0 / 1 and r^3 %% 256 == 0 "
                 "(which=%d b=%d r=%d)", which, b, r);
  PCFM_CHECK_ARG(conv3_shape_ok(b, cin, cout, r),
                 "conv3d_igemm_cl_list: unsupported shape b=%d cin=%d cout=%d r=%d", b, cin, cout,
                 r);
  const int V = r * r * r, tiles = b * (V / 256);
#ifndef PCFM_CONV_NOGLDS
  const bool listed = glds_ok(cout, r) && glds_splits(b, cin, cout, r) == 1;
#else
  const bool listed = false;
#endif
  if (!listed)  // no list form for this shape: the dense GEMM (every voxel)
    return igemm_cl(xs, wsplit, bias, b, cin, cout, r, y, ws, ws_bytes, stream, nullptr, 0);
  const bool vox = (list_vox() >> which) & 1;
  const int* l = vox ? lists + 64 + 4 * tiles + 2 * ((size_t)b * V / kChunk) +
                           (size_t)which * b * V
                     : lists + 64 + 2 * tiles + (size_t)which * b * V / kChunk;
  hipStream_t st = (hipStream_t)stream;
  const uint32_t* vbits =
      vox ? (const uint32_t*)(lists + 64 + 4 * tiles + 2 * ((size_t)b * V / kChunk) +
                              2 * (size_t)b * V) +
                (size_t)which * b * V / kChunk
          : nullptr;
  hipLaunchKernelGGL(conv3_fill_unlisted_kernel, dim3(tiles), dim3(256), 0, st, cnt, r, cout,
                     which, bias, y, vbits);
  const int e = check_launch("conv3d_igemm_cl_list");
  if (e) return e;
  // the forward reads occupied neighbour rows only (list 2's bitmap; env
  // PCFM_LIST_ZROW=0: every in-volume row, A/B)
  const char* zr = getenv("PCFM_LIST_ZROW");
  const uint32_t* obits =
      which == 1 && (zr == nullptr || zr[0] != '0')
          ? (const uint32_t*)(lists + 64 + 4 * tiles + 2 * ((size_t)b * V / kChunk) +
                              2 * (size_t)b * V)
          : nullptr;
  return igemm_cl(xs, wsplit, bias, b, cin, cout, r, y, ws, ws_bytes, stream, nullptr, 0, l,
                  vox ? lists + 2 + which : lists + which, vox ? 0 : 5, obits,
                  vox ? list_gn(which) : 256);
}

static int wgrad_cap(int b, int r, int S) {
  const long long nchunk = (long long)b * r * r * r / kWV;
  return (int)((nchunk + S - 1) / S);
}

static int wgrad_cl(const void* xs, const void* gys, int b, int cin, int cout, int r,
                    const uint32_t* cmask, float* grad_w, void* ws, size_t ws_bytes,
                    void* stream, const uint32_t* kmask = nullptr) {
  PCFM_CHECK_ARG(b > 0 && conv3_shape_ok(b, cin, cout, r) && cin % kMT == 0,
                 "conv3d_wgrad_cl: unsupported shape b=%d cin=%d cout=%d r=%d", b, cin, cout, r);
  const size_t need = wgrad_partial_bytes(b, cin, cout, r);
  PCFM_CHECK_ARG(ws_bytes >= need, "conv3d_wgrad_cl: workspace %zu < %zu bytes", ws_bytes, need);
  const int S = conv3_wgrad_splits(b, cin, cout, r);
  const int V = r * r * r;
  hipStream_t st = (hipStream_t)stream;
  const int tiles = 27 * (cout / kMT) * (cin / kMT);
  const uint16_t* xh = (const uint16_t*)xs;
  const uint16_t* gh = (const uint16_t*)gys;
  if (conv3_wgrad3_ok(r)) {
    const int e = allow_big_lds((const void*)conv3_wgrad3_kernel);
    if (e) return e;
    int* lists = nullptr;
    int* counts = nullptr;
    const int cap = wgrad_cap(b, r, S);
    if (cmask != nullptr) {
      const size_t lb = (size_t)9 * S * cap * sizeof(int), cb = (size_t)9 * S * sizeof(int);
      PCFM_CHECK_ARG(ws_bytes >= need + lb + cb,
                     "conv3d_wgrad_cl_occ: workspace %zu < %zu bytes", ws_bytes, need + lb + cb);
      lists = (int*)((char*)ws + need);
      counts = (int*)((char*)ws + need + lb);
      hipLaunchKernelGGL(conv3_wgrad_lists_kernel, dim3(9, S), dim3(64), 0, st, cmask,
                         b * (V / kWV), S, cap, lists, counts);
    }
    const size_t lds = 2 * (size_t)kW3Buf + (kmask != nullptr ? (size_t)cap * 16 : 0);
    PCFM_CHECK_ARG(lds <= (size_t)kLdsBytesMax, "conv3d_wgrad_cl_occ: %d listed chunks per split "
                   "exceed the LDS", cap);
    hipLaunchKernelGGL(conv3_wgrad3_kernel, dim3(tiles / 3 * S), dim3(kW3Threads), lds, st,
                       xh, xh + kSplitLo, gh, gh + kSplitLo, b, cin, cout, r,
                       S, (float*)ws, lists, counts, cap, kmask);
  } else {
    hipLaunchKernelGGL(conv3_wgrad_cl_kernel, dim3(tiles * S), dim3(256), 0, st, xh,
                       xh + kSplitLo, gh, gh + kSplitLo, b, cin, cout, r, S,
                       (float*)ws);
  }
  hipLaunchKernelGGL(conv3_wgrad_reduce_kernel, dim3(ceil_div((long long)cout * cin, 64)),
                     dim3(256), 0, st, (const float*)ws, cout, cin, S, grad_w);
  return check_launch("conv3d_wgrad_cl");
}

extern "C" int pcfm_conv3d_wgrad_cl(const void* xs, const void* gys, int b, int cin, int cout,
                                    int r, float* grad_w, void* ws, size_t ws_bytes,
                                    void* stream) {
  return wgrad_cl(xs, gys, b, cin, cout, r, nullptr, grad_w, ws, ws_bytes, stream);
}

extern "C" size_t pcfm_conv3d_wgrad_occ_workspace_bytes(int b, int cin, int cout, int r) {
  if (b <= 0 || !conv3_shape_ok(b, cin, cout, r) || cin % kMT != 0) return 0;
  const int S = conv3_wgrad_splits(b, cin, cout, r);
  return wgrad_partial_bytes(b, cin, cout, r) +
         (size_t)9 * S * (wgrad_cap(b, r, S) + 1) * sizeof(int);
}

extern "C" int pcfm_conv3d_wgrad_cl_occ(const void* xs, const void* gys, int b, int cin,
                                        int cout, int r, const unsigned* masks, float* grad_w,
                                        void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(masks != nullptr && (r * r * r) % 256 == 0,
                 "conv3d_wgrad_cl_occ: need the occupancy masks and r^3 %% 256 == 0 (r=%d)", r);
  const int V = r * r * r;
  // the chunk masks follow the tile masks in pcfm_conv3d_occupancy's buffer
  const uint32_t* cmask = (const uint32_t*)masks + (size_t)b * (V / 256);
  // the K-slice masks follow the chunk masks (PCFM_WGRAD_KSKIP=0: none, A/B knob)
  const char* ks = std::getenv("PCFM_WGRAD_KSKIP");
  const uint32_t* kmask = (ks != nullptr && ks[0] == '0') ? nullptr : cmask + (size_t)b * (V / 64);
  return wgrad_cl(xs, gys, b, cin, cout, r, cmask, grad_w, ws, ws_bytes, stream, kmask);
}
