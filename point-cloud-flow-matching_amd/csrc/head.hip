// Per-point head of the flow model (models.py:62-153, 546-601 in the
// reference): the Linear layers of VelocityNetWithContext / ShapeEncoder run
// under bf16 autocast on rows = B*N points (160000 at the bench config).
//
// Weight gradient of such a Linear:  dW[m][n] = sum_r dY[r][m] * X[r][n]
// with R = 160000 and M, N <= 512 -- a GEMM whose reduction axis is the long
// one.  The library GEMM runs it as a handful of output tiles with the whole
// K = R each (16 x 128x128 tiles on 256 CUs, ~160 TFLOP/s measured); here the
// row axis is split over the grid (split-K, every CU busy), each block
// accumulates a 128 x 128 fp32 tile with v_mfma_f32_32x32x16_bf16, and an
// ordered reduce adds the partials (deterministic) and rounds to bf16 -- the
// dtype autocast's mm returns for the reference's layer.
//
// Operand staging: both operands are row-major [r][col] with the reduction
// index r on the slow axis, so the LDS image is the global tile as it is
// ([64 rows][128 cols] bf16, 16-B chunks XOR-swizzled within a 256-B row) and
// the MFMA operands (8 consecutive r per lane) come out of gfx950's
// transposing LDS read ds_read_b64_tr_b16 (cdna_hip_programming.md T10).
#include <algorithm>
#include <cstdlib>

#include "pcfm_common.hpp"

namespace pcfm {
namespace {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8h __attribute__((ext_vector_type(8)));
typedef float f32x16h __attribute__((ext_vector_type(16)));

constexpr int kRT = 64;    // rows (reduction) per K-step
constexpr int kTile = 128; // output tile edge

// byte offset of 16-B chunk `ch` (0..15) of LDS row `row` (256-B rows),
// the T10 (b) swizzle: conflict-free ds_write_b128 rows and tr_b16 reads
__device__ __forceinline__ int swz(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ v4s tr_read(const uint8_t* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s*)(base + off));
}

// One 64-row x 128-col bf16 tile of a row-major matrix into 4 uint4 per thread
// (rows >= R and columns >= ncols are zero).  MODE 2: ld % 8 == 0, 16-B
// aligned base and the tile's 128 columns all in range (one 16-B load per
// chunk); MODE 1: ld even, 4-B aligned base (32-bit loads); MODE 0: 16-bit loads.
template <int MODE>
__device__ __forceinline__ void load_tile(const uint16_t* __restrict__ src, int ld, int ncols,
                                          long long r0, long long R, int c0, int t,
                                          uint4 (&v)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = t + 256 * q;
    const int row = c >> 4, ch = c & 15;
    const long long gr = r0 + row;
    const bool rok = gr < R;
    const long long grc = rok ? gr : R - 1;
    if (MODE == 2) {
      uint4 x = *reinterpret_cast<const uint4*>(src + (size_t)grc * ld + c0 + ch * 8);
      if (!rok) x = uint4{0u, 0u, 0u, 0u};
      v[q] = x;
    } else {
      const uint16_t* rp = src + (size_t)grc * ld;
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int col = c0 + ch * 8 + 2 * e;
        uint32_t x = 0u;
        if (MODE == 1) {
          if (col < ncols) x = *reinterpret_cast<const uint32_t*>(rp + col);
          if (col + 1 >= ncols) x &= 0xFFFFu;
        } else {
          if (col < ncols) x = rp[col];
          if (col + 1 < ncols) x |= (uint32_t)rp[col + 1] << 16;
        }
        w[e] = rok ? x : 0u;
      }
      v[q] = uint4{w[0], w[1], w[2], w[3]};
    }
  }
}

__device__ __forceinline__ void store_tile(uint8_t* img, int t, const uint4 (&v)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = t + 256 * q;
    *reinterpret_cast<uint4*>(img + swz(c >> 4, c & 15)) = v[q];
  }
}

// 3 waves per SIMD (140 VGPRs, accumulators out of AGPRs) and 3 blocks per CU:
// the compiler's own choice was 120 VGPRs + 64 AGPRs, 2 waves per SIMD.
// tools/rows_ab.py on MI355X (R = 160000): 512x512 0.173 -> 0.160 ms,
// 512x384 0.197 -> 0.119 ms, 6x512 0.047 -> 0.042 ms; 4 waves spill (0.22 ms)
#ifndef PCFM_RW_W4
#define PCFM_RW_W4 3
#endif
#define RW_WAVES __attribute__((amdgpu_waves_per_eu(PCFM_RW_W4, PCFM_RW_W4)))
// grid = (tiles_m * tiles_n, S), 256 threads (2 x 2 waves of 64 x 64).
// part[s][M][N] fp32 = sum over split s's rows of A[r][m] * B[r][n].
template <int MA, int MB>
__global__ void __launch_bounds__(256) RW_WAVES
    rows_wgrad_kernel(const uint16_t* __restrict__ A, int lda, const uint16_t* __restrict__ B,
                      int ldb, long long R, int M, int N, int S, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * kRT * 256];
  uint8_t* imgA = lds;
  uint8_t* imgB = lds + kRT * 256;
  const int tm = (M + kTile - 1) / kTile;
#ifndef PCFM_RW_NOXCD
  // XCD-contiguous deal: consecutive blocks go round-robin to the 8 XCDs, so
  // give each XCD a contiguous run of (split, tile) items -- the tiles of one
  // split read the same A / B row chunks and now share that XCD's L2
  int bx, sp;
  {
    const int tiles = (int)gridDim.x;
    const int tot = tiles * (int)gridDim.y;
    int id = (int)(blockIdx.x + tiles * blockIdx.y);
    const int q = tot / 8, rr = tot % 8, xcd = id % 8;
    id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + id / 8;
    bx = id % tiles;
    sp = id / tiles;
  }
#else
  const int bx = blockIdx.x, sp = blockIdx.y;
#endif
  const int m0 = (bx % tm) * kTile, n0 = (bx / tm) * kTile;
  const long long nsteps = (R + kRT - 1) / kRT;
  const long long k0 = nsteps * sp / S, k1 = nsteps * (sp + 1) / S;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int g = lane >> 4, i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;

  f32x16h acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  uint4 ra[4], rb[4];
  if (k0 < k1) {
    load_tile<MA>(A, lda, M, k0 * kRT, R, m0, t, ra);
    load_tile<MB>(B, ldb, N, k0 * kRT, R, n0, t, rb);
    store_tile(imgA, t, ra);
    store_tile(imgB, t, rb);
  }
  __syncthreads();
  for (long long ks = k0; ks < k1; ++ks) {
    if (ks + 1 < k1) {
      load_tile<MA>(A, lda, M, (ks + 1) * kRT, R, m0, t, ra);
      load_tile<MB>(B, ldb, N, (ks + 1) * kRT, R, n0, t, rb);
    }
#pragma unroll
    for (int kk = 0; kk < kRT / 16; ++kk) {
      bf16x8h a[2], b[2];
      const int row = kk * 16 + 8 * (g >> 1) + q4;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int col = wr * 64 + i * 32 + (g & 1) * 16 + 4 * p4;
        const int off0 = swz(row, col >> 3) + 8 * (p4 & 1);
        const int off1 = swz(row + 4, col >> 3) + 8 * (p4 & 1);
        const v4s x0 = tr_read(imgA, off0), x1 = tr_read(imgA, off1);
        a[i] = __builtin_bit_cast(bf16x8h, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = wc * 64 + j * 32 + (g & 1) * 16 + 4 * p4;
        const int off0 = swz(row, col >> 3) + 8 * (p4 & 1);
        const int off1 = swz(row + 4, col >> 3) + 8 * (p4 & 1);
        const v4s y0 = tr_read(imgB, off0), y1 = tr_read(imgB, off1);
        b[j] = __builtin_bit_cast(bf16x8h, __builtin_shufflevector(y0, y1, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (ks + 1 < k1) {
      store_tile(imgA, t, ra);
      store_tile(imgB, t, rb);
    }
    __syncthreads();
  }
  float* pb = part + (size_t)sp * M * N;
  const int h = lane >> 5, r = lane & 31;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wr * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int n = n0 + wc * 64 + j * 32 + r;
        if (m < M && n < N) pb[(size_t)m * N + n] = acc[i][j][e];
      }
}

// out[i] = bf16(sum_{s < S} part[s][i]) in split order (deterministic).
__global__ void __launch_bounds__(256)
    rows_wgrad_reduce_kernel(const float* __restrict__ part, size_t total, int S,
                             uint16_t* __restrict__ out) {
  // 64 outputs per block, 4 thread groups over the splits, fixed combine order
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const size_t i = (size_t)blockIdx.x * 64 + cl;
  float sum = 0.0f;
  if (i < total) {
    int q = grp;
    // 4 of the group's partials loaded before they are added (same order)
    for (; q + 12 < S; q += 16) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = part[(size_t)(q + 4 * u) * total + i];
#pragma unroll
      for (int u = 0; u < 4; ++u) sum = sum + v[u];
    }
    for (; q < S; q += 4) sum = sum + part[(size_t)q * total + i];
  }
  red[grp][cl] = sum;
  __syncthreads();
  if (grp == 0 && i < total)
    out[i] = __builtin_bit_cast(
        uint16_t, (__bf16)(((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl]));
}

// blocks per CU the split count aims at (dev knob PCFM_RW_BPC, measurement)
inline long long rows_wgrad_bpc() {
  static const long long v = [] {
    const char* e = std::getenv("PCFM_RW_BPC");
    return e != nullptr ? std::max(1LL, std::atoll(e)) : 3LL;
  }();
  return v;
}

int rows_wgrad_splits(long long R, int M, int N) {
  const long long tiles = (long long)((M + kTile - 1) / kTile) * ((N + kTile - 1) / kTile);
  const long long steps = (R + kRT - 1) / kRT;
  long long s = std::max(1LL, (rows_wgrad_bpc() * kCUs + tiles - 1) / tiles);
  s = std::min(s, std::max(1LL, steps / 8));  // >= 8 K-steps per block
  return (int)std::min(s, 256LL);
}

bool rows_ok(long long R, int M, int N, int lda, int ldb) {
  return R >= 0 && M > 0 && N > 0 && lda >= M && ldb >= N;
}

}  // namespace
}  // namespace pcfm

using namespace pcfm;

extern "C" size_t pcfm_rows_wgrad_workspace_bytes(long long rows, int m, int n) {
  if (!rows_ok(rows, m, n, m, n) || rows == 0) return 0;
  return (size_t)rows_wgrad_splits(rows, m, n) * m * n * sizeof(float);
}

extern "C" int pcfm_rows_wgrad_bf16(const void* a, int lda, const void* b, int ldb,
                                    long long rows, int m, int n, void* out, void* ws,
                                    size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(rows_ok(rows, m, n, lda, ldb),
                 "rows_wgrad_bf16: bad shape rows=%lld m=%d n=%d lda=%d ldb=%d", rows, m, n,
                 lda, ldb);
  hipStream_t st = (hipStream_t)stream;
  const size_t total = (size_t)m * n;
  if (rows == 0) {
    const hipError_t e = hipMemsetAsync(out, 0, total * sizeof(uint16_t), st);
    if (e != hipSuccess) {
      set_error("rows_wgrad_bf16: hipMemsetAsync: %s", hipGetErrorString(e));
      return (int)e;
    }
    return PCFM_OK;
  }
  const size_t need = pcfm_rows_wgrad_workspace_bytes(rows, m, n);
  PCFM_CHECK_ARG(ws_bytes >= need, "rows_wgrad_bf16: workspace %zu < %zu bytes", ws_bytes, need);
  const int S = rows_wgrad_splits(rows, m, n);
  const int tiles = ((m + kTile - 1) / kTile) * ((n + kTile - 1) / kTile);
  const uint16_t* A = (const uint16_t*)a;
  const uint16_t* B = (const uint16_t*)b;
  const auto mode = [](const void* p, int ld, int cols) {
    const uintptr_t u = (uintptr_t)p;
    if (ld % 8 == 0 && cols % kTile == 0 && (u & 15) == 0) return 2;
    return (ld % 2 == 0 && (u & 3) == 0) ? 1 : 0;
  };
  const int ma = mode(a, lda, m), mb = mode(b, ldb, n);
  const dim3 grid(tiles, S), blk(256);
  float* part = (float*)ws;
#define PCFM_ROWS_LAUNCH(X, Y)                                                              \
  if (ma == X && mb == Y)                                                                   \
    hipLaunchKernelGGL((rows_wgrad_kernel<X, Y>), grid, blk, 0, st, A, lda, B, ldb, rows, m, \
                       n, S, part);
  PCFM_ROWS_LAUNCH(2, 2)
  PCFM_ROWS_LAUNCH(2, 1)
  PCFM_ROWS_LAUNCH(2, 0)
  PCFM_ROWS_LAUNCH(1, 2)
  PCFM_ROWS_LAUNCH(1, 1)
  PCFM_ROWS_LAUNCH(1, 0)
  PCFM_ROWS_LAUNCH(0, 2)
  PCFM_ROWS_LAUNCH(0, 1)
  PCFM_ROWS_LAUNCH(0, 0)
#undef PCFM_ROWS_LAUNCH
  hipLaunchKernelGGL(rows_wgrad_reduce_kernel, dim3(ceil_div((long long)total, 64)), dim3(256),
                     0, st, (const float*)ws, total, S, (uint16_t*)out);
  return check_launch("rows_wgrad_bf16");
}

// ---------------------------------------------------------------------------
// Max over the point axis of a (B, N, C) bf16 tensor with its argmax -- the
// ShapeEncoder's global pooling h.max(dim=1) (reference models.py:156-187).
// Lowest index on ties.  Stage 1: grid (P, B), 4 waves stride the part's rows,
// lanes hold channel pairs (128 channels per pass); stage 2: per (b, c) over the P parts in order.
// ---------------------------------------------------------------------------
namespace pcfm {
namespace {

__device__ __forceinline__ bool max_better(float v, int i, float m, int mi) {
  // NaN propagates as the maximum (torch.max); ties -> lower index
  if (v != v) return m == m || i < mi;
  return v > m || (v == m && i < mi);
}

__global__ void __launch_bounds__(256)
    rows_max_part_kernel(const uint16_t* __restrict__ h, int N, int C, float* __restrict__ pv,
                         int* __restrict__ pi) {
  __shared__ float sv[4][128];
  __shared__ int si[4][128];
  const int b = blockIdx.y, p = blockIdx.x, P = gridDim.x;
  const int chunk = (N + P - 1) / P, n0 = min(N, p * chunk), n1 = min(N, n0 + chunk);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int cb = 0; cb < C; cb += 128) {
    const int c = cb + 2 * lane;  // channel pair (c, c + 1); C is even
    float m0 = -INFINITY, m1 = -INFINITY;
    int i0 = N, i1 = N;
    if (c < C) {
      for (int r = n0 + wave; r < n1; r += 4) {
        const uint32_t u = *reinterpret_cast<const uint32_t*>(h + ((size_t)b * N + r) * C + c);
        const float v0 = __uint_as_float(u << 16), v1 = __uint_as_float(u & 0xFFFF0000u);
        if (max_better(v0, r, m0, i0)) { m0 = v0; i0 = r; }
        if (max_better(v1, r, m1, i1)) { m1 = v1; i1 = r; }
      }
    }
    sv[wave][2 * lane] = m0;
    sv[wave][2 * lane + 1] = m1;
    si[wave][2 * lane] = i0;
    si[wave][2 * lane + 1] = i1;
    __syncthreads();
    if (threadIdx.x < 128) {
      const int k = threadIdx.x, ck = cb + k;
      float m = sv[0][k];
      int mi = si[0][k];
      for (int w = 1; w < 4; ++w)
        if (max_better(sv[w][k], si[w][k], m, mi)) { m = sv[w][k]; mi = si[w][k]; }
      if (ck < C) {
        pv[((size_t)b * P + p) * C + ck] = m;
        pi[((size_t)b * P + p) * C + ck] = mi;
      }
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256)
    rows_max_final_kernel(const float* __restrict__ pv, const int* __restrict__ pi, int P, int C,
                          uint16_t* __restrict__ val, int* __restrict__ idx) {
  const int b = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float m = -INFINITY;
  int mi = 0x7FFFFFFF;
  for (int p = 0; p < P; ++p) {
    const float v = pv[((size_t)b * P + p) * C + c];
    const int i = pi[((size_t)b * P + p) * C + c];
    if (max_better(v, i, m, mi)) { m = v; mi = i; }
  }
  val[(size_t)b * C + c] = (uint16_t)(__float_as_uint(m) >> 16);
  idx[(size_t)b * C + c] = mi;
}

constexpr int kMaxParts = 32;

// ---------------------------------------------------------------------------
// Column sums over the rows of a (B, rows, C) tensor, bf16 or fp32, into fp32
// (B, C): the bias gradients of the per-point Linears (dY.sum(0)) and the
// gradient of a per-cloud row broadcast over the points.  Stage 1: block p of
// batch b sums rows [p*rows/P, (p+1)*rows/P), threads on (row lane, column
// pair) so every row is one coalesced stream; stage 2 adds the P partials in
// order (deterministic).
// ---------------------------------------------------------------------------
// stage-1 blocks per batch element: >= 256 rows each, ~2048 blocks in all, <= 256
inline int colsum_parts(int b, long long rows) {
  const long long want = std::max(1LL, (2048LL + b - 1) / b);
  return (int)std::max(1LL, std::min({(rows + 255) / 256, want, 256LL}));
}

template <bool BF16>
__global__ void __launch_bounds__(256)
    colsum_part_kernel(const void* __restrict__ x, long long rows, int C, float* __restrict__ part) {
  const int b = blockIdx.y, p = blockIdx.x, P = gridDim.x;
  const int pairs = C / 2;
  const int rl = threadIdx.x / pairs, cp = threadIdx.x % pairs;
  const int rstep = 256 / pairs;  // pairs <= 256
  const long long r0 = rows * p / P, r1 = rows * (p + 1) / P;
  __shared__ float red[256 * 2];
  float s0 = 0.0f, s1 = 0.0f;
  auto ld = [&](long long r) {
    const size_t o = ((size_t)b * rows + r) * C + 2 * cp;
    if constexpr (BF16) {
      const uint32_t q = *reinterpret_cast<const uint32_t*>(
          reinterpret_cast<const uint16_t*>(x) + o);
      return make_float2(__uint_as_float(q << 16), __uint_as_float(q & 0xFFFF0000u));
    } else {
      return *reinterpret_cast<const float2*>(reinterpret_cast<const float*>(x) + o);
    }
  };
  if (rl < rstep) {
    long long r = r0 + rl;
    // 8 rows' loads in flight before they are added, in the same row order (one
    // dependent load per add kept a thread latency-bound: 0.84 TB/s)
    for (; r + 7 * rstep < r1; r += 8 * rstep) {
      float2 q[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) q[u] = ld(r + u * rstep);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s0 += q[u].x;
        s1 += q[u].y;
      }
    }
    for (; r < r1; r += rstep) {
      const float2 q = ld(r);
      s0 += q.x;
      s1 += q.y;
    }
  }
  red[2 * threadIdx.x] = s0;
  red[2 * threadIdx.x + 1] = s1;
  __syncthreads();
  if (threadIdx.x < pairs) {  // row lanes in a fixed order
    float a0 = 0.0f, a1 = 0.0f;
    for (int l = 0; l < rstep; ++l) {
      a0 += red[2 * (l * pairs + threadIdx.x)];
      a1 += red[2 * (l * pairs + threadIdx.x) + 1];
    }
    float* o = part + ((size_t)b * P + p) * C + 2 * threadIdx.x;
    o[0] = a0;
    o[1] = a1;
  }
}

// grid (ceil(C / 64), B): 4 thread groups take every 4th partial, combined in order
__global__ void __launch_bounds__(256)
    colsum_final_kernel(const float* __restrict__ part, int P, int C, float* __restrict__ out) {
  __shared__ float red[4][64];
  const int b = blockIdx.y, cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float s = 0.0f;
  if (c < C) {
    int p = grp;
    // 4 of the group's partials loaded before they are added (same order)
    for (; p + 12 < P; p += 16) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = part[((size_t)b * P + p + 4 * u) * C + c];
#pragma unroll
      for (int u = 0; u < 4; ++u) s += v[u];
    }
    for (; p < P; p += 4) s += part[((size_t)b * P + p) * C + c];
  }
  red[grp][cl] = s;
  __syncthreads();
  if (grp == 0 && c < C) out[(size_t)b * C + c] = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
}

// ContextNet's t-gate blend (models.py:533-541) fused with the (B, C, N) ->
// (B, N, C) permute of head_out:  out[b][n][c] = a[b] * head[b][c][n] +
// (1 - a[b]) * glb[b][c];  backward dhead[b][c][n] = a[b] * dout[b][n][c].
// 64 x 64 tiles through LDS; grid (ceil(N/64), ceil(C/64), B), 256 threads.
template <bool FWD>
__global__ void __launch_bounds__(256)
    tgate_kernel(const float* __restrict__ src, const float* __restrict__ glb,
                 const float* __restrict__ alpha, int C, int N, float* __restrict__ dst) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z, n0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const float a = alpha[b];
  if (FWD) {  // read head rows (c, n contiguous), write out rows (n, c contiguous)
    for (int r = ty; r < 64; r += 4) {
      const int c = c0 + r, n = n0 + tx;
      tile[r][tx] = (c < C && n < N) ? src[((size_t)b * C + c) * N + n] : 0.0f;
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
      const int n = n0 + r, c = c0 + tx;
      if (n < N && c < C)
        dst[((size_t)b * N + n) * C + c] =
            __builtin_fmaf(a, tile[tx][r], (1.0f - a) * glb[(size_t)b * C + c]);
    }
  } else {  // read dout rows (n, c contiguous), write dhead rows (c, n contiguous)
    for (int r = ty; r < 64; r += 4) {
      const int n = n0 + r, c = c0 + tx;
      tile[r][tx] = (n < N && c < C) ? src[((size_t)b * N + n) * C + c] : 0.0f;
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
      const int c = c0 + r, n = n0 + tx;
      if (c < C && n < N) dst[((size_t)b * C + c) * N + n] = a * tile[tx][r];
    }
  }
}

}  // namespace
}  // namespace pcfm

extern "C" int pcfm_tgate_fwd(const float* head, const float* glb, const float* alpha, int b,
                              int c, int n, float* out, void* stream) {
  PCFM_CHECK_ARG(b >= 0 && c > 0 && n >= 0 && b < 65536, "tgate_fwd: bad shape b=%d c=%d n=%d", b,
                 c, n);
  if (b == 0 || n == 0) return PCFM_OK;
  hipLaunchKernelGGL(tgate_kernel<true>, dim3(ceil_div(n, 64), ceil_div(c, 64), b), dim3(256), 0,
                     (hipStream_t)stream, head, glb, alpha, c, n, out);
  return check_launch("tgate_fwd");
}

extern "C" int pcfm_tgate_bwd(const float* dout, const float* alpha, int b, int c, int n,
                              float* dhead, void* stream) {
  PCFM_CHECK_ARG(b >= 0 && c > 0 && n >= 0 && b < 65536, "tgate_bwd: bad shape b=%d c=%d n=%d", b,
                 c, n);
  if (b == 0 || n == 0) return PCFM_OK;
  hipLaunchKernelGGL(tgate_kernel<false>, dim3(ceil_div(n, 64), ceil_div(c, 64), b), dim3(256), 0,
                     (hipStream_t)stream, dout, nullptr, alpha, c, n, dhead);
  return check_launch("tgate_bwd");
}

extern "C" size_t pcfm_rows_colsum_workspace_bytes(int b, long long rows, int c) {
  if (b <= 0 || rows < 0 || c <= 0 || c % 2 != 0 || c > 512) return 0;
  return (size_t)b * colsum_parts(b, rows) * c * sizeof(float);
}

extern "C" int pcfm_rows_colsum(const void* x, int bf16, int b, long long rows, int c, float* out,
                                void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(pcfm_rows_colsum_workspace_bytes(b, rows, c) > 0 && b < 65536,
                 "rows_colsum: bad shape b=%d rows=%lld c=%d (c even, <= 512)", b, rows, c);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_rows_colsum_workspace_bytes(b, rows, c),
                 "rows_colsum: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  const int P = colsum_parts(b, rows);
  if (bf16)
    hipLaunchKernelGGL(colsum_part_kernel<true>, dim3(P, b), dim3(256), 0, st, x, rows, c, part);
  else
    hipLaunchKernelGGL(colsum_part_kernel<false>, dim3(P, b), dim3(256), 0, st, x, rows, c, part);
  hipLaunchKernelGGL(colsum_final_kernel, dim3(ceil_div(c, 64), b), dim3(256), 0, st,
                     (const float*)part, P, c, out);
  return check_launch("rows_colsum");
}

extern "C" size_t pcfm_rows_max_workspace_bytes(int b, int n, int c) {
  if (b <= 0 || n <= 0 || c <= 0 || c % 2 != 0) return 0;
  return (size_t)b * kMaxParts * c * (sizeof(float) + sizeof(int));
}

extern "C" int pcfm_rows_max_bf16(const void* h, int b, int n, int c, void* values, int* indices,
                                  void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(pcfm_rows_max_workspace_bytes(b, n, c) > 0,
                 "rows_max_bf16: bad shape b=%d n=%d c=%d (c even, n > 0)", b, n, c);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_rows_max_workspace_bytes(b, n, c),
                 "rows_max_bf16: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* pv = (float*)ws;
  int* pi = (int*)(pv + (size_t)b * kMaxParts * c);
  hipLaunchKernelGGL(rows_max_part_kernel, dim3(kMaxParts, b), dim3(256), 0, st,
                     (const uint16_t*)h, n, c, pv, pi);
  hipLaunchKernelGGL(rows_max_final_kernel, dim3(ceil_div(c, 256), b), dim3(256), 0, st,
                     (const float*)pv, (const int*)pi, kMaxParts, c, (uint16_t*)values, indices);
  return check_launch("rows_max_bf16");
}
