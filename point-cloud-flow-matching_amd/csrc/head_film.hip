// Row kernels of the per-point head trunk (reference models.py:62-79 FiLMBlock,
// :107-116 trunk loop, :135/:594 per-batch embedding), bf16 autocast
// semantics of the reference's train step:
//
//   h_1 = input Linear(x)            (bf16)
//   block i:  y = LayerNorm(h_i)     (fp32; autocast runs layer_norm in fp32)
//             u = y * sp1[b] + shift[b]     sp1 = bf16(1 + scale), shift bf16,
//                                           (scale, shift) = affine(emb[b]) -- per batch
//             a = bf16(SiLU(u))             (the blk Linear's autocast input cast)
//             g = Linear(a)                 (bf16, library GEMM)
//             h_{i+1} = u + g               (fp32)
//   out:      a_out = bf16(SiLU(h_last));  v = Linear(a_out)
//
// One wave owns a row (W = 256 * NV channels; lane l holds channels
// 256 j + 4 l + e), so LayerNorm's row statistics are wave reductions and every
// access is a coalesced 1-KB (fp32) / 512-B (bf16) stream per wave.  A block
// owns 256 consecutive rows of ONE batch element, so the per-batch FiLM
// vectors are loaded once per block and the backward's per-batch column sums
// (d sp1, d shift) and global column sums (d gamma, d beta, bias grad of the
// preceding Linear) are per-block register partials, added in a fixed order
// by film_bwd_reduce (deterministic, no atomics).
//
// Forward  (film_fwd<FILM>):  FILM: h -> u (fp32), a (bf16), mean/rstd per row
//                             !FILM (output layer): h -> a = bf16(SiLU(h))
// Backward (film_bwd<FILM>):  FILM: du = dh_next + da * SiLU'(u); LayerNorm /
//                             FiLM backward -> dh (fp32) and bf16(dh)
//                             !FILM: dh = da * SiLU'(h)
// with h given either as a bf16 tensor (h_1) or as u_prev + g_prev, the
// residual sum recomputed instead of stored.  h_1 may carry a per-batch fp32
// bias row hb[b] (the input Linear's columns that see the batch-constant
// embedding, folded out of the GEMM): h_1 = bf16(h16 + hb[b]).
#include <algorithm>

#include "pcfm_common.hpp"

namespace pcfm {
namespace {

// waves-per-SIMD bound of the FiLM backward (measurement knob; 0: none)
#ifndef PCFM_FILM_BWD_WPE
#define PCFM_FILM_BWD_WPE 0
#endif
#if PCFM_FILM_BWD_WPE > 0
#define FILM_BWD_ATTR __attribute__((amdgpu_waves_per_eu(PCFM_FILM_BWD_WPE)))
#else
#define FILM_BWD_ATTR
#endif
constexpr int kRowsPerBlock = 256;  // 4 waves x 64 rows, one batch element
constexpr int kSums = 5;            // d sp1, d shift, d gamma, d beta, d bias_prev

__device__ __forceinline__ float bf2f(uint32_t b) { return __uint_as_float(b << 16); }
__device__ __forceinline__ uint32_t f2bf(float x) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)x);
}

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

template <int NV>
__device__ __forceinline__ void ld_f32(const float* __restrict__ p, int lane, float (&v)[NV][4]) {
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const float4 f = *reinterpret_cast<const float4*>(p + 256 * j + 4 * lane);
    v[j][0] = f.x;
    v[j][1] = f.y;
    v[j][2] = f.z;
    v[j][3] = f.w;
  }
}

template <int NV>
__device__ __forceinline__ void ld_bf16(const uint16_t* __restrict__ p, int lane,
                                        float (&v)[NV][4]) {
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const uint2 q = *reinterpret_cast<const uint2*>(p + 256 * j + 4 * lane);
    v[j][0] = bf2f(q.x & 0xFFFFu);
    v[j][1] = bf2f(q.x >> 16);
    v[j][2] = bf2f(q.y & 0xFFFFu);
    v[j][3] = bf2f(q.y >> 16);
  }
}

template <int NV>
__device__ __forceinline__ void st_f32(float* __restrict__ p, int lane, const float (&v)[NV][4]) {
#pragma unroll
  for (int j = 0; j < NV; ++j)
    *reinterpret_cast<float4*>(p + 256 * j + 4 * lane) =
        make_float4(v[j][0], v[j][1], v[j][2], v[j][3]);
}

template <int NV>
__device__ __forceinline__ void st_bf16(uint16_t* __restrict__ p, int lane,
                                        const float (&v)[NV][4]) {
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    uint2 q;
    q.x = f2bf(v[j][0]) | (f2bf(v[j][1]) << 16);
    q.y = f2bf(v[j][2]) | (f2bf(v[j][3]) << 16);
    *reinterpret_cast<uint2*>(p + 256 * j + 4 * lane) = q;
  }
}

// h of row `row`: bf16 tensor if h16, else u_prev + float(g_prev) (fp32 add)
template <int NV>
__device__ __forceinline__ void load_h(const uint16_t* __restrict__ h16,
                                       const float* __restrict__ uprev,
                                       const uint16_t* __restrict__ gprev, size_t off, int lane,
                                       float (&x)[NV][4], bool has_hb, const float (&hb)[NV][4]) {
  if (h16 != nullptr) {
    ld_bf16<NV>(h16 + off, lane, x);
    if (has_hb) {
#pragma unroll
      for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) x[j][e] = bf2f(f2bf(x[j][e] + hb[j][e]));
    }
  } else {
    float g[NV][4];
    ld_f32<NV>(uprev + off, lane, x);
    ld_bf16<NV>(gprev + off, lane, g);
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) x[j][e] = x[j][e] + g[j][e];
  }
}

// torch's SiLU: x / (1 + exp(-x)); its backward: dy * s * (1 + x * (1 - s))
__device__ __forceinline__ float silu(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float dsilu(float x) {
  const float s = 1.0f / (1.0f + expf(-x));
  return s * (1.0f + x * (1.0f - s));
}

// grid = (ceil(n / rpb), B), 256 threads; a block owns rpb rows.
template <int NV, bool FILM>
__global__ void __launch_bounds__(256)
    film_fwd_kernel(const uint16_t* __restrict__ h16, const float* __restrict__ uprev,
                    const uint16_t* __restrict__ gprev, const float* __restrict__ gamma,
                    const float* __restrict__ beta, const uint16_t* __restrict__ sp1,
                    const uint16_t* __restrict__ shift, const float* __restrict__ hbias, int n,
                    float eps, float* __restrict__ u, uint16_t* __restrict__ a,
                    float* __restrict__ mean_o, float* __restrict__ rstd_o, int rpb) {
  constexpr int W = 256 * NV;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.y;
  const int i0 = blockIdx.x * rpb, i1 = min(n, i0 + rpb);
  float gm[NV][4], bt[NV][4], sp[NV][4], sh[NV][4], hb[NV][4];
  const bool has_hb = hbias != nullptr;
  if (has_hb) ld_f32<NV>(hbias + (size_t)b * W, lane, hb);
  if (FILM) {
    ld_f32<NV>(gamma, lane, gm);
    ld_f32<NV>(beta, lane, bt);
    ld_bf16<NV>(sp1 + (size_t)b * W, lane, sp);
    ld_bf16<NV>(shift + (size_t)b * W, lane, sh);
  }
  for (int i = i0 + wave; i < i1; i += 4) {
    const size_t row = (size_t)b * n + i;
    const size_t off = row * W;
    float x[NV][4];
    load_h<NV>(h16, uprev, gprev, off, lane, x, has_hb, hb);
    float o[NV][4];
    if (FILM) {
      float s = 0.0f;
#pragma unroll
      for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) s += x[j][e];
      const float mean = wave_sum(s) * (1.0f / W);
      float q = 0.0f;
#pragma unroll
      for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = x[j][e] - mean;
          q = __builtin_fmaf(d, d, q);
        }
      const float rstd = rsqrtf(wave_sum(q) * (1.0f / W) + eps);
      float uu[NV][4];
#pragma unroll
      for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float y = __builtin_fmaf(gm[j][e], rstd * (x[j][e] - mean), bt[j][e]);
          uu[j][e] = y * sp[j][e] + sh[j][e];  // unfused (-ffp-contract=off), as the backward
          o[j][e] = silu(uu[j][e]);
        }
      st_f32<NV>(u + off, lane, uu);
      if (lane == 0) {
        mean_o[row] = mean;
        rstd_o[row] = rstd;
      }
    } else {
#pragma unroll
      for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) o[j][e] = silu(x[j][e]);
    }
    st_bf16<NV>(a + off, lane, o);
  }
}

// grid = (chunks = ceil(n / 256), B), 256 threads.  part[B * chunks][5][W].
template <int NV, bool FILM>
__global__ void __launch_bounds__(256) FILM_BWD_ATTR
    film_bwd_kernel(const float* __restrict__ dhn, const uint16_t* __restrict__ da16,
                    const float* __restrict__ u, const uint16_t* __restrict__ h16,
                    const float* __restrict__ uprev, const uint16_t* __restrict__ gprev,
                    const float* __restrict__ mean_i, const float* __restrict__ rstd_i,
                    const float* __restrict__ gamma, const float* __restrict__ beta,
                    const uint16_t* __restrict__ sp1, const uint16_t* __restrict__ shift,
                    const float* __restrict__ hbias, int n, float* __restrict__ dh,
                    uint16_t* __restrict__ dh16, float* __restrict__ part) {
  constexpr int W = 256 * NV;
  __shared__ float red[4][kSums][W];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.y;
  const int i0 = blockIdx.x * kRowsPerBlock, i1 = min(n, i0 + kRowsPerBlock);
  const bool has_hb = hbias != nullptr;
  // u == nullptr: u recomputed from h and the saved row statistics with the
  // forward's own expression (bit-identical), instead of read back (2 of the
  // 11 KB a 512-wide row costs)
  const bool keep_u = u != nullptr;
  // The block's channel constants (gamma, beta, sp1[b], shift[b], hbias[b])
  // live in LDS during the row loop -- in `red`, which is only needed after it
  // -- and are read per row: in registers they took 40 VGPRs and held the
  // kernel to 2-3 waves per SIMD on a latency-bound row stream.
  float* cst = &red[0][0][0];
  for (int c = threadIdx.x; c < W; c += 256) {
    if (FILM) {
      cst[c] = gamma[c];
      cst[W + c] = beta[c];
      cst[2 * W + c] = bf2f(sp1[(size_t)b * W + c]);
      cst[3 * W + c] = keep_u ? 0.0f : bf2f(shift[(size_t)b * W + c]);
    }
    cst[4 * W + c] = has_hb ? hbias[(size_t)b * W + c] : 0.0f;
  }
  __syncthreads();
  float acc[kSums][NV][4];
#pragma unroll
  for (int k = 0; k < kSums; ++k)
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[k][j][e] = 0.0f;
#pragma nounroll
  for (int i = i0 + wave; i < i1; i += 4) {
    const size_t row = (size_t)b * n + i;
    const size_t off = row * W;
    // keeps the constant reads inside the loop (not hoisted back into registers)
    asm volatile("" ::: "memory");
    float da[NV][4], x[NV][4], g[NV][4], hb[NV][4];
    if (has_hb) ld_f32<NV>(cst + 4 * W, lane, hb);
    ld_bf16<NV>(da16 + off, lane, da);
    load_h<NV>(h16, uprev, gprev, off, lane, x, has_hb, hb);
    if (FILM) {
      float gm[NV][4], bt[NV][4], sp[NV][4], sh[NV][4];
      ld_f32<NV>(cst, lane, gm);
      ld_f32<NV>(cst + W, lane, bt);
      ld_f32<NV>(cst + 2 * W, lane, sp);
      if (!keep_u) ld_f32<NV>(cst + 3 * W, lane, sh);
      float du[NV][4], uu[NV][4];
      ld_f32<NV>(dhn + off, lane, du);
      if (keep_u) ld_f32<NV>(u + off, lane, uu);
      const float mean = mean_i[row], rstd = rstd_i[row];
      float s1 = 0.0f, s2 = 0.0f;
      float xh[NV][4], dxh[NV][4];
      if (!keep_u) {
#pragma unroll
        for (int j = 0; j < NV; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            uu[j][e] = __builtin_fmaf(gm[j][e], rstd * (x[j][e] - mean), bt[j][e]) * sp[j][e] +
                       sh[j][e];
      }
#pragma unroll
      for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = du[j][e] + da[j][e] * dsilu(uu[j][e]);
          const float xc = rstd * (x[j][e] - mean);
          const float y = __builtin_fmaf(gm[j][e], xc, bt[j][e]);
          const float dy = d * sp[j][e];
          acc[0][j][e] += d * y;     // d sp1 (= d scale)
          acc[1][j][e] += d;         // d shift
          acc[2][j][e] += dy * xc;   // d gamma
          acc[3][j][e] += dy;        // d beta
          xh[j][e] = xc;
          dxh[j][e] = dy * gm[j][e];
          s1 += dxh[j][e];
          s2 += dxh[j][e] * xc;
        }
      const float m1 = wave_sum(s1) * (1.0f / W), m2 = wave_sum(s2) * (1.0f / W);
#pragma unroll
      for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) g[j][e] = rstd * (dxh[j][e] - m1 - xh[j][e] * m2);
    } else {
#pragma unroll
      for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) g[j][e] = da[j][e] * dsilu(x[j][e]);
    }
    if (dh != nullptr) st_f32<NV>(dh + off, lane, g);
    st_bf16<NV>(dh16 + off, lane, g);
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[4][j][e] += bf2f(f2bf(g[j][e]));  // bias grad of prev Linear
  }
  __syncthreads();  // every wave is done with the constants in `red`
#pragma unroll
  for (int k = 0; k < kSums; ++k)
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[wave][k][256 * j + 4 * lane + e] = acc[k][j][e];
  __syncthreads();
  float* pb = part + ((size_t)b * gridDim.x + blockIdx.x) * kSums * W;
  for (int idx = threadIdx.x; idx < kSums * W; idx += 256) {
    const int k = idx / W, c = idx - k * W;
    pb[idx] = ((red[0][k][c] + red[1][k][c]) + red[2][k][c]) + red[3][k][c];
  }
}

// Stage 1: per-batch sums of the block partials, chunk order fixed (4 thread
// groups take every 4th chunk, combined in group order).  k = 0, 1 go straight
// to dsp1 / dshift [B][W]; k = 2..4 go to perb[k - 2][B][W] for stage 2.
// grid = (ceil(W / 64), 5, B), 256 threads.
__global__ void __launch_bounds__(256)
    film_bwd_reduce_kernel(const float* __restrict__ part, int B, int chunks, int W,
                           float* __restrict__ dsp1, float* __restrict__ dshift,
                           float* __restrict__ perb) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, k = blockIdx.y, b = blockIdx.z;
  float s = 0.0f;
  if (c < W) {
    const float* p = part + ((size_t)b * chunks * kSums + k) * W + c;
    int q = grp;
    // 4 of the group's partials loaded before they are added (same order)
    for (; q + 12 < chunks; q += 16) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = p[(size_t)(q + 4 * u) * kSums * W];
#pragma unroll
      for (int u = 0; u < 4; ++u) s += v[u];
    }
    for (; q < chunks; q += 4) s += p[(size_t)q * kSums * W];
  }
  red[grp][cl] = s;
  __syncthreads();
  if (grp != 0 || c >= W) return;
  s = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
  float* out = k == 0 ? dsp1 : k == 1 ? dshift : perb + (size_t)(k - 2) * B * W;
  if (out != nullptr) out[(size_t)b * W + c] = s;
}

// Stage 2: global sums over the batch (k = 2..4 -> dgamma / dbeta / dbias [W]);
// a null output is skipped.  grid = (ceil(W / 64), 3), 64 threads.
__global__ void __launch_bounds__(64)
    film_bwd_reduce2_kernel(const float* __restrict__ perb, int B, int W,
                            float* __restrict__ dgamma, float* __restrict__ dbeta,
                            float* __restrict__ dbias) {
  const int c = blockIdx.x * 64 + threadIdx.x, k = blockIdx.y;
  float* out = k == 0 ? dgamma : k == 1 ? dbeta : dbias;
  if (c >= W || out == nullptr) return;
  float s = 0.0f;
  for (int b = 0; b < B; ++b) s += perb[((size_t)k * B + b) * W + c];
  out[c] = s;
}

// rows per forward block (env PCFM_FILM_FWD_ROWS, a multiple of 4, default
// 32; read per call: A/B runs)
int film_fwd_rows() {
  const char* e = getenv("PCFM_FILM_FWD_ROWS");
  const int v = e != nullptr ? atoi(e) : 32;
  return v >= 4 && v % 4 == 0 ? v : 32;
}

bool film_ok(int b, int n, int w) {
  return b > 0 && n > 0 && (w == 256 || w == 512) &&
         (long long)b * n * w < (1LL << 40);
}

template <bool FILM>
int launch_fwd(const void* h16, const float* uprev, const void* gprev, const float* gamma,
               const float* beta, const void* sp1, const void* shift, const float* hbias, int b,
               int n, int w, float eps, float* u, void* a, float* mean, float* rstd,
               hipStream_t st) {
  // 32 rows per block (8 per wave): at 256 the B = 8, N = 20000 pass had 632
  // blocks, 2.5 waves per SIMD with one row each in flight -- 0.175 -> 0.154 ms
  // per 512-wide launch, 5.6 -> 6.4 TB/s (profiles/r06_ab_film_rows.jsonl).
  // The backward stays at 256 (its partials are per block; 64 / 128 rows and
  // two rows in flight per wave measured slower there).
  const int rpb = film_fwd_rows();
  const dim3 grid(ceil_div(n, rpb), b), blk(256);
  const uint16_t* H = (const uint16_t*)h16;
  const uint16_t* G = (const uint16_t*)gprev;
  const uint16_t* S1 = (const uint16_t*)sp1;
  const uint16_t* SH = (const uint16_t*)shift;
  uint16_t* A = (uint16_t*)a;
  switch (w) {
    case 256:
      hipLaunchKernelGGL((film_fwd_kernel<1, FILM>), grid, blk, 0, st, H, uprev, G, gamma, beta,
                         S1, SH, hbias, n, eps, u, A, mean, rstd, rpb);
      break;
    default:
      hipLaunchKernelGGL((film_fwd_kernel<2, FILM>), grid, blk, 0, st, H, uprev, G, gamma, beta,
                         S1, SH, hbias, n, eps, u, A, mean, rstd, rpb);
  }
  return check_launch(FILM ? "head_film_fwd" : "head_silu_fwd");
}

template <bool FILM>
int launch_bwd(const float* dhn, const void* da16, const float* u, const void* h16,
               const float* uprev, const void* gprev, const float* mean, const float* rstd,
               const float* gamma, const float* beta, const void* sp1, const void* shift,
               const float* hbias, int b, int n, int w, float* dh, void* dh16, float* dsp1, float* dshift, float* dgamma,
               float* dbeta, float* dbias, float* dbias_b, void* ws, hipStream_t st) {
  const int chunks = ceil_div(n, kRowsPerBlock);
  const dim3 grid(chunks, b), blk(256);
  const uint16_t* DA = (const uint16_t*)da16;
  const uint16_t* H = (const uint16_t*)h16;
  const uint16_t* G = (const uint16_t*)gprev;
  const uint16_t* S1 = (const uint16_t*)sp1;
  const uint16_t* SH = (const uint16_t*)shift;
  uint16_t* D16 = (uint16_t*)dh16;
  float* part = (float*)ws;
  switch (w) {
    case 256:
      hipLaunchKernelGGL((film_bwd_kernel<1, FILM>), grid, blk, 0, st, dhn, DA, u, H, uprev, G,
                         mean, rstd, gamma, beta, S1, SH, hbias, n, dh, D16, part);
      break;
    default:
      hipLaunchKernelGGL((film_bwd_kernel<2, FILM>), grid, blk, 0, st, dhn, DA, u, H, uprev, G,
                         mean, rstd, gamma, beta, S1, SH, hbias, n, dh, D16, part);
  }
  float* perb = part + (size_t)b * chunks * kSums * w;
  hipLaunchKernelGGL(film_bwd_reduce_kernel, dim3(ceil_div(w, 64), kSums, b), dim3(256), 0, st,
                     (const float*)part, b, chunks, w, dsp1, dshift, perb);
  hipLaunchKernelGGL(film_bwd_reduce2_kernel, dim3(ceil_div(w, 64), 3), dim3(64), 0, st,
                     (const float*)perb, b, w, dgamma, dbeta, dbias);
  if (dbias_b != nullptr) {  // per-batch bias grad of the preceding Linear (its hb rows)
    const hipError_t e = hipMemcpyAsync(dbias_b, perb + 2 * (size_t)b * w,
                                        (size_t)b * w * sizeof(float), hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) {
      set_error("head_film_bwd: hipMemcpyAsync: %s", hipGetErrorString(e));
      return (int)e;
    }
  }
  return check_launch(FILM ? "head_film_bwd" : "head_silu_bwd");
}

}  // namespace
}  // namespace pcfm

using namespace pcfm;

extern "C" int pcfm_head_film_fwd(const void* h16, const float* hbias, const float* uprev,
                                  const void* gprev, const float* gamma, const float* beta,
                                  const void* sp1, const void* shift, int b, int n, int w,
                                  float eps, float* u, void* a, float* mean, float* rstd,
                                  void* stream) {
  PCFM_CHECK_ARG(film_ok(b, n, w), "head_film_fwd: bad shape b=%d n=%d w=%d", b, n, w);
  PCFM_CHECK_ARG(h16 != nullptr || (uprev != nullptr && gprev != nullptr),
                 "head_film_fwd: need h16 or (uprev, gprev)");
  return launch_fwd<true>(h16, uprev, gprev, gamma, beta, sp1, shift,
                          h16 != nullptr ? hbias : nullptr, b, n, w, eps, u, a, mean, rstd,
                          (hipStream_t)stream);
}

extern "C" int pcfm_head_silu_fwd(const float* uprev, const void* gprev, int b, int n, int w,
                                  void* a, void* stream) {
  PCFM_CHECK_ARG(film_ok(b, n, w), "head_silu_fwd: bad shape b=%d n=%d w=%d", b, n, w);
  return launch_fwd<false>(nullptr, uprev, gprev, nullptr, nullptr, nullptr, nullptr, nullptr, b,
                           n, w, 0.0f, nullptr, a, nullptr, nullptr, (hipStream_t)stream);
}

extern "C" size_t pcfm_head_bwd_workspace_bytes(int b, int n, int w) {
  if (!film_ok(b, n, w)) return 0;
  return ((size_t)b * ceil_div(n, kRowsPerBlock) * kSums + 3 * (size_t)b) * w * sizeof(float);
}

extern "C" int pcfm_head_film_bwd(const float* dh_next, const void* da16, const float* u,
                                  const void* h16, const float* hbias, const float* uprev,
                                  const void* gprev, const float* mean, const float* rstd,
                                  const float* gamma, const float* beta, const void* sp1,
                                  const void* shift, int b, int n, int w, float* dh, void* dh16,
                                  float* dsp1, float* dshift,
                                  float* dgamma, float* dbeta, float* dbias, float* dbias_b,
                                  void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(film_ok(b, n, w), "head_film_bwd: bad shape b=%d n=%d w=%d", b, n, w);
  PCFM_CHECK_ARG(h16 != nullptr || (uprev != nullptr && gprev != nullptr),
                 "head_film_bwd: need h16 or (uprev, gprev)");
  PCFM_CHECK_ARG(u != nullptr || shift != nullptr, "head_film_bwd: need u or shift");
  PCFM_CHECK_ARG(ws_bytes >= pcfm_head_bwd_workspace_bytes(b, n, w),
                 "head_film_bwd: workspace %zu < %zu bytes", ws_bytes,
                 pcfm_head_bwd_workspace_bytes(b, n, w));
  return launch_bwd<true>(dh_next, da16, u, h16, uprev, gprev, mean, rstd, gamma, beta, sp1, shift,
                          h16 != nullptr ? hbias : nullptr, b, n, w, dh, dh16, dsp1, dshift,
                          dgamma, dbeta, dbias, dbias_b, ws, (hipStream_t)stream);
}

extern "C" int pcfm_head_silu_bwd(const void* da16, const float* uprev, const void* gprev, int b,
                                  int n, int w, float* dh, void* dh16, float* dbias, void* ws,
                                  size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(film_ok(b, n, w), "head_silu_bwd: bad shape b=%d n=%d w=%d", b, n, w);
  PCFM_CHECK_ARG(ws_bytes >= pcfm_head_bwd_workspace_bytes(b, n, w),
                 "head_silu_bwd: workspace %zu < %zu bytes", ws_bytes,
                 pcfm_head_bwd_workspace_bytes(b, n, w));
  return launch_bwd<false>(nullptr, da16, nullptr, nullptr, uprev, gprev, nullptr, nullptr,
                           nullptr, nullptr, nullptr, nullptr, nullptr, b, n, w, dh, dh16, nullptr,
                           nullptr, nullptr, nullptr, dbias, nullptr, ws, (hipStream_t)stream);
}
