// Pointwise (1x1) convolution -- SharedMLP's Conv1d(C_in, C_out, 1)
// (third_party/pvcnn/modules/shared_mlp.py:15-27) and ContextNet's
// head_pre/head_out -- as bf16x3 GEMMs on the matrix cores (mfma_x3.hpp):
//   forward        y[b, m, p] = sum_k W[m, k] x[b, k, p] (+ bias[m])
//   backward-data  dx[b, k, p] = sum_m W[m, k] dy[b, m, p]   (transposed image)
//   backward-wt    dW[m, k] = sum_{b, p} dy[b, m, p] x[b, k, p]
// Tensors are (B, C, N) fp32 as the reference's Conv1d sees them.  Any C_in,
// C_out and N: the weight image is zero-padded to the tile grid and partial
// point / channel tiles are masked.
#include <algorithm>
#include <cstdlib>

#include "mfma_x3.hpp"

namespace pcfm {
namespace {

inline int pad_to(int x, int m) { return (x + m - 1) / m * m; }

// GEMM output stores are streamed (non-temporal): the outputs (80-330 MB) do
// not fit L2 and are next read by another kernel.  256 -> 256 at N = 20000:
// forward 112 -> 106 us, backward-data 134 -> 116 us (tools/pw_ab.py)
__device__ __forceinline__ void out_store(float* p, float v) {
#ifndef PCFM_PW_CACHED_STORE
  nt_st(v, p);
#else
  *p = v;
#endif
}
// rows of the weight image: above 256 a multiple of 256, so the 256-row tile
// (x read once per 256 output rows) applies -- ContextNet head_pre's backward-data
// (M = 640 -> 768: x read 3 times instead of 5 by 128-row tiles)
inline int pw_mpad(int m) { return m > 256 ? pad_to(m, 256) : pad_to(m, 128); }

// A channel-segmented (B, C, N) tensor: channels [off[i], off[i+1]) live in
// their own (B, off[i+1] - off[i], N) tensor p[i] -- ContextNet's head input
// is the channel concat of the stage outputs, read in place instead of copied.
// Segment boundaries are multiples of 32 (inputs) / 128 (outputs).
constexpr int kMaxParts = 4;
struct Parts {
  float* p[kMaxParts];
  int off[kMaxParts + 1];
  int n;
  __device__ __forceinline__ float* row(int b, int c, int N) const {
    int i = 0;
#pragma unroll
    for (int k = 1; k < kMaxParts; ++k) i += (k < n && c >= off[k]) ? 1 : 0;
    const int w = off[i + 1] - off[i];
    return p[i] + ((size_t)b * w + (c - off[i])) * N;
  }
};
inline Parts one_part(const float* x, int c) {
  Parts q{};
  q.p[0] = const_cast<float*>(x);
  q.off[0] = 0;
  q.off[1] = c;
  q.n = 1;
  return q;
}

// W [cout][cin] -> image [Mpad][Kpad] bf16 hi, lo; transpose: [cin][cout]
__global__ void __launch_bounds__(256)
    pw_wsplit_kernel(const float* __restrict__ w, int cout, int cin, int transpose, int Mpad,
                     int Kpad, uint16_t* __restrict__ wh, uint16_t* __restrict__ wl) {
  const size_t total = (size_t)Mpad * Kpad;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int m = (int)(i / Kpad), k = (int)(i - (size_t)m * Kpad);
  const int M = transpose ? cin : cout, K = transpose ? cout : cin;
  float v = 0.0f;
  if (m < M && k < K) v = transpose ? w[(size_t)k * cin + m] : w[(size_t)m * cin + k];
  uint32_t hi, lo;
  split_bf16(v, hi, lo);
  wh[i] = (uint16_t)hi;
  wl[i] = (uint16_t)lo;
}

// grid = (ceil(N / TN), Mpad / TM, B), 256 threads.
template <int TM, int TN>
__global__ void __launch_bounds__(256)
    pw_gemm_kernel(const Parts x, const uint16_t* __restrict__ wh,
                   const uint16_t* __restrict__ wl, const float* __restrict__ bias, int bias_bstride,
                   const Parts y, int K, int M, int N, int Kpad) {
  using T = Tile<TM, TN>;
  __shared__ __attribute__((aligned(16))) uint16_t lds[T::BUF];
  const int b = blockIdx.z, m0 = blockIdx.y * TM, p0 = blockIdx.x * TN;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1, r = lane & 31, h = lane >> 5;
  constexpr int CPT = kKT * TN / 256;  // channels per thread per K-step
  // TN >= 64: a wave's threads share one channel group (uniform -> SGPR row pointers)
  const int sp = t % TN, ch = __builtin_amdgcn_readfirstlane((t / TN) * CPT);
  const int pt = p0 + sp;
  const bool pok = pt < N;
  const int ptc = pok ? pt : N - 1;  // clamped: always a valid address
  const bool astage = 2 * TM >= 256 || t < 2 * TM;
  const int arow = t >> 1, ahalf = (t & 1) * 16;
  const int nsteps = Kpad / kKT;

  uint4 ra0 = {}, ra1 = {}, ra2 = {}, ra3 = {};
  float rb[CPT];
  uint32_t rmask = 0u;  // elements to zero (channel >= K or point >= N)
  auto load = [&](int s) {
    const int c0 = s * kKT;
    if (astage) {
      const size_t g = (size_t)(m0 + arow) * Kpad + c0 + ahalf;
      ra0 = *reinterpret_cast<const uint4*>(wh + g);
      ra1 = *reinterpret_cast<const uint4*>(wh + g + 8);
      ra2 = *reinterpret_cast<const uint4*>(wl + g);
      ra3 = *reinterpret_cast<const uint4*>(wl + g + 8);
    }
    rmask = 0u;
    // the CPT channels are consecutive and inside one part (parts are 32-aligned)
    const int cb = min(c0 + ch, K - 1);
    const float* __restrict__ xr = x.row(b, cb, N);
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
      const int c = c0 + ch + q;
      const bool ok = pok && c < K;
      rb[q] = xr[(size_t)(c < K ? c - cb : 0) * N + ptc];
      rmask |= ok ? 0u : (1u << q);
    }
  };
  auto store = [&](uint16_t* buf) {
    if (astage) {
      uint16_t* dh = buf + arow * kLDR + ahalf;
      uint16_t* dl = buf + T::A_ELEMS + arow * kLDR + ahalf;
      *reinterpret_cast<uint4*>(dh) = ra0;
      *reinterpret_cast<uint4*>(dh + 8) = ra1;
      *reinterpret_cast<uint4*>(dl) = ra2;
      *reinterpret_cast<uint4*>(dl + 8) = ra3;
    }
#pragma unroll
    for (int q = 0; q < CPT; ++q) rb[q] = (rmask >> q) & 1u ? 0.0f : rb[q];
    uint16_t* bh = buf + 2 * T::A_ELEMS + sp * kLDR + ch;
    store_split<CPT>(rb, bh, bh + T::B_ELEMS);
  };

  f32x16 acc[T::SI][T::SJ];
#pragma unroll
  for (int i = 0; i < T::SI; ++i)
#pragma unroll
    for (int j = 0; j < T::SJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  load(0);
  store(lds);
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    if (s + 1 < nsteps) load(s + 1);
    tile_mfma<TM, TN>(lds, wr, wc, r, h, acc);
    __syncthreads();
    if (s + 1 < nsteps) store(lds);
    __syncthreads();
  }
  const int bo = b * bias_bstride;  // per-cloud bias row (0: one shared bias)
#pragma unroll
  for (int i = 0; i < T::SI; ++i) {
    // a 32-row group lies inside one output part (parts are 128-aligned)
    const int mg = m0 + wr * (TM / 2) + i * 32;
    float* __restrict__ yr = y.row(b, min(mg, M - 1), N);
    float bv[16];
    load_bias16(bias != nullptr ? bias + bo : nullptr, mg, h, M, bv);
#pragma unroll
    for (int j = 0; j < T::SJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int dm = (e & 3) + 8 * (e >> 2) + 4 * h;
        const int m = mg + dm;
        const int p = p0 + wc * (TN / 2) + j * 32 + r;
        if (m < M && p < N) out_store(yr + (size_t)dm * N + p, acc[i][j][e] + bv[e]);
      }
  }
}

// Wide form for Mpad % 256 == 0: a 256 (m) x 128 (point) tile, 8 waves of
// 64 x 64 (4 x 2), 512 threads, 60 KiB LDS (two blocks per CU).  Every output
// channel of a point tile comes from one block, so x is read from HBM once
// (the 128-row tile above reads it Mpad / 128 times).
// stats != nullptr (a SharedMLP layer's BatchNorm follows): per output channel m
// and 64-point group g of batch element b, the group's mean and centred sum of
// squares of y go to stats[m * P + b * ngroups + g] (P = B * ngroups) -- the
// BatchNorm statistics pass over y is not needed (bn_fin_parts_kernel combines
// the groups, Chan's formula, in a fixed order).  Sums are taken about a shift
// (the group's first value of the row, so no cancellation) and reduced over the
// 32 lanes of a row segment by a transposing butterfly: at each xor stage a
// lane keeps one half of its values and sends the other, so the 32 sums of 16
// rows cost 31 lane swizzles instead of 5 per value (measured: the per-value
// shuffle tree, 320 ds_bpermute per wave, made the GEMM 0.28 ms/step slower
// than the separate statistics pass it replaced).
template <int MASK>
__device__ __forceinline__ float swz_xor(float v) {  // lane ^ MASK within 32 lanes
  return __builtin_bit_cast(
      float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), (MASK << 10) | 0x1f));
}
template <int K, int MASK>
__device__ __forceinline__ void xpose_reduce_stage(float* v, bool upper) {
#pragma unroll
  for (int k = 0; k < K / 2; ++k) {
    const float keep = upper ? v[k + K / 2] : v[k];
    const float send = upper ? v[k] : v[k + K / 2];
    v[k] = keep + swz_xor<MASK>(send);
  }
}

// Epilogue of a 256 (m) x 128 (point) tile held as 8 waves of 64 x 64
// (pw_gemm256_kernel): y = acc + bias, streamed stores, and with stats the
// per-(channel, 64-point group) BatchNorm statistics (see pw_gemm256_kernel).
// nb = batch elements (the stats row length is nb * groups).  sbias: the tile's
// 256 bias values (rows m0 + i, clamped to M - 1), staged in LDS by the kernel
// at its start -- read here without a global load's latency at the end.
__device__ __forceinline__ void pw256_epilogue(const f32x16 (&acc)[2][2], const Parts& y,
                                               const float* __restrict__ sbias, int b, int nb,
                                               int M, int N, int m0, int p0, int wr, int wc,
                                               int r, int h, float2* __restrict__ stats) {
  const int pw0 = p0 + wc * 64;  // this wave's 64 points
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int mg = m0 + wr * 64 + i * 32;
    float* __restrict__ yr = y.row(b, min(mg, M - 1), N);
    float bv[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) bv[e] = sbias[mg - m0 + (e & 3) + 8 * (e >> 2) + 4 * h];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int dm = (e & 3) + 8 * (e >> 2) + 4 * h;
        const int m = mg + dm;
        const int p = pw0 + j * 32 + r;
#ifdef PCFM_EXP_PW_NOSTORE
        if (acc[i][j][e] == 1.2345f)
#endif
        if (m < M && p < N) out_store(yr + (size_t)dm * N + p, acc[i][j][e] + bv[e]);
      }
    if (stats != nullptr && pw0 < N) {
      const int nv = min(64, N - pw0);
      const int ngroups = (N + 63) / 64, P = nb * ngroups;
      const bool ok0 = pw0 + r < N, ok1 = pw0 + 32 + r < N;
      float v[32], sr = 0.0f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float v0 = acc[i][0][e] + bv[e], v1 = acc[i][1][e] + bv[e];
        const float s0 = __builtin_bit_cast(
            float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v0), 0));
        const float s1 = __builtin_bit_cast(
            float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v0), 32));
        const float sh = h ? s1 : s0;  // row (e, h)'s value at point pw0
        sr = r == e ? sh : sr;
        const float d0 = ok0 ? v0 - sh : 0.0f, d1 = ok1 ? v1 - sh : 0.0f;
        v[e] = d0 + d1;
        v[16 + e] = __builtin_fmaf(d1, d1, d0 * d0);
      }
      xpose_reduce_stage<32, 16>(v, r & 16);
      xpose_reduce_stage<16, 8>(v, r & 8);
      xpose_reduce_stage<8, 4>(v, r & 4);
      xpose_reduce_stage<4, 2>(v, r & 2);
      xpose_reduce_stage<2, 1>(v, r & 1);
      // lane r: v[0] = sum of value r (r < 16: shifted sum of row e = r; else its squares)
      const float q = swz_xor<16>(v[0]);
      const int m = mg + (r & 3) + 8 * ((r >> 2) & 3) + 4 * h;
      if (r < 16 && m < M) {
        const float a = v[0], mu_s = a / (float)nv;
        stats[(size_t)m * P + b * ngroups + pw0 / 64] =
            make_float2(sr + mu_s, fmaxf(__builtin_fmaf(-a, mu_s, q), 0.0f));
      }
    }
  }
}

// (Measured, round 4: holding x two K-steps ahead in a second register slot
// did not change the time -- 0.090 vs 0.087 ms at 8 x 256 x 256 x 20000 -- so
// the kernel keeps one slot.)
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4)))
    pw_gemm256_kernel(const Parts x, const uint16_t* __restrict__ wh,
                      const uint16_t* __restrict__ wl, const float* __restrict__ bias,
                      int bias_bstride, const Parts y, int K, int M, int N, int Kpad,
                      float2* __restrict__ stats = nullptr) {
  constexpr int TM = 256, TN = 128;
  constexpr int A_ELEMS = TM * kLDR, B_ELEMS = TN * kLDR;
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * A_ELEMS + 2 * B_ELEMS];
  __shared__ float sbias[TM];
  const int b = blockIdx.z, m0 = blockIdx.y * TM, p0 = blockIdx.x * TN;
  const int t = threadIdx.x, lane = t & 63;
  // the tile's bias rows, visible after the first barrier below
  if (t < TM) sbias[t] = bias != nullptr ? bias[b * bias_bstride + min(m0 + t, M - 1)] : 0.0f;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1, r = lane & 31, h = lane >> 5;
  constexpr int CPT = kKT * TN / 512;  // 8 channels per thread per K-step
  const int sp = t % TN, ch = __builtin_amdgcn_readfirstlane((t / TN) * CPT);
  const int pt = p0 + sp;
  const bool pok = pt < N;
  const int ptc = pok ? pt : N - 1;
  const int arow = t >> 1, ahalf = (t & 1) * 16;
  const int nsteps = Kpad / kKT;

  uint4 ra0 = {}, ra1 = {}, ra2 = {}, ra3 = {};
  float rb[CPT];
  // the weight images through buffer descriptors too (one lane offset, the
  // K-step in soffset)
  const __amdgpu_buffer_rsrc_t rwh = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(wh), (short)0, 0x7FFFFFF0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rwl = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(wl), (short)0, 0x7FFFFFF0, 0x00020000);
  const int aoff = ((m0 + arow) * Kpad + ahalf) * 2;
  auto load_a = [&](int s) {
#ifdef PCFM_EXP_PW_NOW
    if (s > 0) return;
#endif
    const int so = s * kKT * 2;
    ra0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rwh, aoff, so, 0));
    ra1 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rwh, aoff, so + 16, 0));
    ra2 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rwl, aoff, so, 0));
    ra3 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rwl, aoff, so + 16, 0));
  };
  // x through a buffer descriptor on the (wave-uniform) row of channel cb:
  // one 32-bit lane offset for all CPT loads, the channel step in soffset
  // (instead of a 64-bit address register pair per load)
  const int voff = ptc * 4;
  auto load_b = [&](int s, float (&v)[CPT]) {
    const int c0 = s * kKT;
    const int cb = __builtin_amdgcn_readfirstlane(min(c0 + ch, K - 1));
    const float* xr = x.row(b, cb, N);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(xr), (short)0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
      const int c = c0 + ch + q;
#ifdef PCFM_EXP_PW_NOX
      v[q] = (float)(c + voff);
      (void)rs;
#else
      v[q] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, (c < K ? c - cb : 0) * N * 4, 0));
#endif
    }
  };
  // the padding (points >= N, channels >= K) is zeroed at the store
  auto store = [&](int s, float (&v)[CPT]) {
    uint16_t* dh = lds + arow * kLDR + ahalf;
    uint16_t* dl = lds + A_ELEMS + arow * kLDR + ahalf;
    *reinterpret_cast<uint4*>(dh) = ra0;
    *reinterpret_cast<uint4*>(dh + 8) = ra1;
    *reinterpret_cast<uint4*>(dl) = ra2;
    *reinterpret_cast<uint4*>(dl + 8) = ra3;
#pragma unroll
    for (int q = 0; q < CPT; ++q) v[q] = pok && s * kKT + ch + q < K ? v[q] : 0.0f;
    uint16_t* bh = lds + 2 * A_ELEMS + sp * kLDR + ch;
    store_split<CPT>(v, bh, bh + B_ELEMS);
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  auto frag = [&](int o) {
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + o));
  };
  auto mfma_step = [&]() {
#pragma unroll
    for (int kk = 0; kk < kKT / 16; ++kk) {
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int o = (wr * 64 + i * 32 + r) * kLDR + kk * 16 + 8 * h;
        ah[i] = frag(o);
        al[i] = frag(A_ELEMS + o);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int o = 2 * A_ELEMS + (wc * 64 + j * 32 + r) * kLDR + kk * 16 + 8 * h;
        bh[j] = frag(o);
        bl[j] = frag(B_ELEMS + o);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
  };

  load_a(0);
  load_b(0, rb);
  store(0, rb);
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    if (s + 1 < nsteps) {
      load_a(s + 1);
      load_b(s + 1, rb);
    }
    // keep the loads in front of the MFMA work (left to itself the scheduler
    // sinks the weight loads to the end of the step)
    __builtin_amdgcn_sched_barrier(0);
#ifndef PCFM_EXP_PW_NOMFMA
    mfma_step();
#else
    acc[0][0][0] += (float)lds[t];
#endif
    __syncthreads();
    if (s + 1 < nsteps) store(s + 1, rb);
    __syncthreads();
  }
  pw256_epilogue(acc, y, sbias, b, (int)gridDim.z,
                 M, N, m0, p0, wr, wc, r, h, stats);
}

// Streaming form for M <= 128, K <= 256, both multiples of 32 (SharedMLP 128 -> 128 layers and
// their backward-data, stage-2 proj backward-data): a skinny GEMM that is
// HBM-bound (x in, y out once), so no point tile is staged through LDS.  The
// whole weight image (hi + lo, <= 132 KiB) is loaded into LDS once per
// persistent block; then every wave streams its own 32-point tiles with no
// barrier: the B operand comes straight from global memory into registers
// (lane l: point p0 + (l & 31), channels 16 kk + 8 (l >> 5) + 0..7 -- per load
// instruction 32 consecutive points of one channel row, 128 B) and is split to
// bf16 hi / lo in registers; the next 32-channel chunk's loads (and across tile
// boundaries the next tile's first chunk) are in flight while the current
// chunk's 24 MFMAs run.  LDS rows of Kpad + 8 bf16 keep the ds_read_b128
// fragment reads conflict-free.  grid = min(tiles / 8, CUs x blocks per CU),
// 512 threads.
constexpr int kSW = 8;  // waves per streaming block
#ifndef PCFM_PW_STREAM_PF
#define PCFM_PW_STREAM_PF 1  // B-operand chunks prefetched (1 or 2)
#endif
__device__ __forceinline__ bf16x8 split8(const float (&v)[8], bf16x8& lo) {
  bf16x8 hi;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = (__bf16)v[j];
    lo[j] = (__bf16)(v[j] - (float)hi[j]);
  }
  return hi;
}

__device__ __forceinline__ const float* uniform_ptr(const float* p) {
  const unsigned long long u = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return (const float*)(((unsigned long long)hi << 32) | lo);
}

// the 16 B-operand values of one 32-channel chunk for lane (n, h): channels
// c0 + 16 kk + 8 h + j (kk < 2, j < 8) of point p (K % 32 == 0: whole chunks);
// one uniform row pointer + one 32-bit lane offset, so the 16 loads differ by
// uniform multiples of N.  Points >= N read row N - 1 and are zeroed.
__device__ __forceinline__ void pw_stream_load(const Parts& x, int b, int c0, int N, int p, int h,
                                               float (&v)[16]) {
  const bool pok = p < N;
  // 32 channels in one part (parts are 32-aligned); the row pointer is wave-uniform
  const float* __restrict__ xr = uniform_ptr(x.row(b, c0, N));
  const int lo = 8 * h * N + (pok ? p : N - 1);  // pw_ok: C * N < 2^31
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float val = xr[lo + (16 * kk + j) * N];
      v[8 * kk + j] = pok ? val : 0.0f;
    }
}

// stats != nullptr: per output channel m and 32-point group g of batch element
// b (one wave's tile), the group's mean and centred sum of squares go to
// stats[m * P + b * ceil(N / 32) + g] -- the 256-row tile's epilogue statistics
// (pw256_epilogue) at 32-point groups.
template <int NCH, bool ST = false>  // Kpad / 32; ST: the statistics epilogue
__global__ void __launch_bounds__(kSW * 64)
    pw_stream128_kernel(const Parts x, const uint16_t* __restrict__ wh,
                        const uint16_t* __restrict__ wl, const float* __restrict__ bias,
                        int bias_bstride, const Parts y, int K, int M, int N, int B,
                        float2* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) uint16_t sa[];  // [2][128][Kpad + 8]
  constexpr int Kpad = 32 * NCH, ldr = Kpad + 8, cpr = Kpad / 8;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  // blockIdx.y: the block's 128-row slice of the output channels (M > 128:
  // every slice streams all point tiles; slices of a tile share its x reads
  // in L2 -- blocks (x, y) and (x, y') sit on one XCD when gridDim.x % 8 == 0)
  const int m0 = (int)blockIdx.y * 128;
  // one bias shared by the batch: the slice's 128 rows staged in LDS with the
  // weights, so a tile's epilogue does not wait on global loads
  __shared__ float sbias[128];
  const bool lbias = bias != nullptr && bias_bstride == 0;
  if (lbias && t < 128) sbias[t] = bias[min(m0 + t, M - 1)];
  for (int e = t; e < 2 * 128 * cpr; e += kSW * 64) {  // weight image -> LDS, 16-B pieces
    const int img = e / (128 * cpr), rem = e - img * 128 * cpr;
    const int row = rem / cpr, pc = rem - row * cpr;
    const uint16_t* src = (img ? wl : wh) + (size_t)(m0 + row) * Kpad + pc * 8;
    *reinterpret_cast<uint4*>(sa + img * 128 * ldr + row * ldr + pc * 8) =
        *reinterpret_cast<const uint4*>(src);
  }
  __syncthreads();

  const int n = lane & 31, h = lane >> 5;
  const int ntn = (N + 31) / 32, tiles = B * ntn;
  const int wstride = (int)gridDim.x * kSW;
  int tl = __builtin_amdgcn_readfirstlane((int)blockIdx.x * kSW + w);
  if (tl >= tiles) return;  // wave-uniform; no barrier below
  const uint16_t* sah = sa;
  const uint16_t* sal = sa + 128 * ldr;
#if PCFM_PW_STREAM_PF >= 2
  // B-operand chunks two ahead in registers: (tile, chunk) positions walk the
  // wave's tiles chunk by chunk; while chunk s computes, s+1 and s+2 are in
  // flight (twice the bytes in flight of the one-ahead form)
  auto adv = [&](int& t, int& c) {
    if (++c == NCH) {
      c = 0;
      t += wstride;
    }
  };
  auto load_at = [&](int t, int c, float (&v)[16]) {
    const int bb = __builtin_amdgcn_readfirstlane(t / ntn);
    pw_stream_load(x, bb, 32 * c, N, (t - bb * ntn) * 32 + n, h, v);
  };
  int t1 = tl, c1 = 0;
  adv(t1, c1);
  int t2 = t1, c2 = c1;
  adv(t2, c2);
  float nx[16], nx1[16];
  load_at(tl, 0, nx);
  if (t1 < tiles) load_at(t1, c1, nx1);
  int ck = 0;
  f32x16 acc[4];
  while (true) {
    const int b = __builtin_amdgcn_readfirstlane(tl / ntn);
    const int p = (tl - b * ntn) * 32 + n;
    float cur[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      cur[q] = nx[q];
      nx[q] = nx1[q];
    }
    if (t2 < tiles) load_at(t2, c2, nx1);
    if (ck == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.0f;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 bh, bl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bh[j] = (__bf16)cur[8 * kk + j];
        bl[j] = (__bf16)(cur[8 * kk + j] - (float)bh[j]);
      }
      const int ko = ck * 32 + kk * 16 + 8 * h;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = (32 * i + n) * ldr + ko;
        const bf16x8 ah = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sah + o));
        const bf16x8 al = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sal + o));
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[i], 0, 0, 0);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[i], 0, 0, 0);
      }
    }
    if (ck == NCH - 1) {
      const int bo = b * bias_bstride;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mg = m0 + 32 * i;
        if (mg < M) {
          float* __restrict__ yr = const_cast<float*>(uniform_ptr(y.row(b, mg, N)));
          float* __restrict__ yl = yr + 4 * h * N + p;
          float bv[16];
          const float* bl = bias != nullptr ? uniform_ptr(bias + bo + mg) + 4 * h : nullptr;
#pragma unroll
          for (int e = 0; e < 16; ++e) bv[e] = bl != nullptr ? bl[(e & 3) + 8 * (e >> 2)] : 0.0f;
          if (p < N) {
#pragma unroll
            for (int e = 0; e < 16; ++e)
              out_store(yl + ((e & 3) + 8 * (e >> 2)) * N, acc[i][e] + bv[e]);
          }
        }
      }
    }
    adv(tl, ck);
    adv(t1, c1);
    adv(t2, c2);
    if (tl >= tiles) break;
  }
}
#else
  float nx[16];
  {
    const int b = tl / ntn;
    pw_stream_load(x, b, 0, N, (tl - b * ntn) * 32 + n, h, nx);
  }
  while (true) {
    const int b = __builtin_amdgcn_readfirstlane(tl / ntn);
    const int p = (tl - b * ntn) * 32 + n;
    const int ntl = tl + wstride;  // the next tile's chunk 0 is issued during chunk NCH-1
    const int nb = __builtin_amdgcn_readfirstlane(ntl / ntn);
    const int np = (ntl - nb * ntn) * 32 + n;
    f32x16 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.0f;
#pragma unroll 1
    for (int ck = 0; ck < NCH; ++ck) {
      float cur[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) cur[q] = nx[q];
      if (ck + 1 < NCH) {
        pw_stream_load(x, b, 32 * (ck + 1), N, p, h, nx);
      } else if (ntl < tiles) {
        pw_stream_load(x, nb, 0, N, np, h, nx);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 bh, bl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          bh[j] = (__bf16)cur[8 * kk + j];
          bl[j] = (__bf16)(cur[8 * kk + j] - (float)bh[j]);
        }
        const int ko = ck * 32 + kk * 16 + 8 * h;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int o = (32 * i + n) * ldr + ko;
          const bf16x8 ah = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sah + o));
          const bf16x8 al = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sal + o));
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[i], 0, 0, 0);
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[i], 0, 0, 0);
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[i], 0, 0, 0);
        }
      }
    }
    // epilogue: rows 32 i + (e & 3) + 8 (e >> 2) + 4 h, point p
    const int bo = b * bias_bstride;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int mg = m0 + 32 * i;
      if (mg < M) {
        // a 32-row group lies in one output part
        float* __restrict__ yr = const_cast<float*>(uniform_ptr(y.row(b, mg, N)));
        float* __restrict__ yl = yr + 4 * h * N + p;  // + uniform row offsets below
        // M % 32 == 0: whole row groups.  One lane pointer + immediate offsets (a
        // per-element index is loop-invariant: the compiler would hoist 64
        // addresses out of the tile loop)
        float bv[16];
        const float* bl = bias != nullptr ? uniform_ptr(bias + bo + mg) + 4 * h : nullptr;
        if (lbias) {  // block-uniform
#pragma unroll
          for (int e = 0; e < 16; ++e) bv[e] = sbias[32 * i + (e & 3) + 8 * (e >> 2) + 4 * h];
        } else {
#pragma unroll
          for (int e = 0; e < 16; ++e) bv[e] = bl != nullptr ? bl[(e & 3) + 8 * (e >> 2)] : 0.0f;
        }
        if (p < N) {
#pragma unroll
          for (int e = 0; e < 16; ++e) out_store(yl + ((e & 3) + 8 * (e >> 2)) * N, acc[i][e] + bv[e]);
        }
        if (ST) {
          const int p0 = p - n, nv = min(32, N - p0);
          const int ngroups = (N + 31) / 32, P = B * ngroups;
          const bool ok = p < N;
          float v[32], sr = 0.0f;
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const float v0 = acc[i][e] + bv[e];
            const float s0 = __builtin_bit_cast(
                float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v0), 0));
            const float s1 = __builtin_bit_cast(
                float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v0), 32));
            const float sh = h ? s1 : s0;  // row (e, h)'s value at point p0
            sr = n == e ? sh : sr;
            const float d0 = ok ? v0 - sh : 0.0f;
            v[e] = d0;
            v[16 + e] = d0 * d0;
          }
          xpose_reduce_stage<32, 16>(v, n & 16);
          xpose_reduce_stage<16, 8>(v, n & 8);
          xpose_reduce_stage<8, 4>(v, n & 4);
          xpose_reduce_stage<4, 2>(v, n & 2);
          xpose_reduce_stage<2, 1>(v, n & 1);
          const float q = swz_xor<16>(v[0]);
          const int m = mg + (n & 3) + 8 * ((n >> 2) & 3) + 4 * h;
          if (n < 16 && m < M) {
            const float a = v[0], mu_s = a / (float)nv;
            stats[(size_t)m * P + b * ngroups + p0 / 32] =
                make_float2(sr + mu_s, fmaxf(__builtin_fmaf(-a, mu_s, q), 0.0f));
          }
        }
      }
    }
    tl = ntl;
    if (tl >= tiles) break;
  }
}
#endif

// dW partials: grid = (ceil(Cout/128) * ceil(Cin/128), S); K-steps of 32
// points (a step never crosses a batch element).  part [S][Cout][Cin].
#ifdef PCFM_PW_WG_WAVES
#define PW_WG_WAVES __attribute__((amdgpu_waves_per_eu(PCFM_PW_WG_WAVES, PCFM_PW_WG_WAVES)))
#else
#define PW_WG_WAVES
#endif
__global__ void __launch_bounds__(256) PW_WG_WAVES
    pw_wgrad_kernel(const Parts x, const float* __restrict__ dy, int B, int cin,
                    int cout, int N, int S, float* __restrict__ part) {
  using T = Tile<128, 128>;
  __shared__ __attribute__((aligned(16))) uint16_t lds[T::BUF];
  const int nco = (cout + 127) / 128;
  const int co0 = (blockIdx.x % nco) * 128, ci0 = (blockIdx.x / nco) * 128;
  const int sp = blockIdx.y;
  const int steps_per_b = (N + kKT - 1) / kKT;
  const long long nsteps = (long long)B * steps_per_b;
  const long long k0 = nsteps * sp / S, k1 = nsteps * (sp + 1) / S;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1, r = lane & 31, h = lane >> 5;
  const int srow = t >> 1, shalf = (t & 1) * 16;
  const int co = co0 + srow, ci = ci0 + srow;
  const bool cook = co < cout, ciok = ci < cin;
  const int coc = cook ? co : cout - 1, cic = ciok ? ci : cin - 1;
  const bool vec = (N & 3) == 0;  // rows 16-B aligned (the runs start at multiples of 16)
  // this thread's x row of batch 0 and the batch stride of its part
  const float* __restrict__ xrow = x.row(0, cic, N);
  const size_t xbstride = (size_t)(x.row(1, cic, N) - xrow);

  float ra[16], rb[16];
  uint32_t amask = 0u, bmask = 0u;
  auto load = [&](long long ks) {
    const int b = (int)(ks / steps_per_b);
    const int p0 = (int)(ks - (long long)b * steps_per_b) * kKT + shalf;
    const float* as = dy + ((size_t)b * cout + coc) * N;
    const float* bs = xrow + (size_t)b * xbstride;
    amask = cook ? 0u : 0xFFFFu;
    bmask = ciok ? 0u : 0xFFFFu;
    if (vec && p0 + 16 <= N) {  // whole 16-point run: four 16-B loads per operand
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 fa = *reinterpret_cast<const float4*>(as + p0 + 4 * q);
        const float4 fb = *reinterpret_cast<const float4*>(bs + p0 + 4 * q);
        ra[4 * q] = fa.x;
        ra[4 * q + 1] = fa.y;
        ra[4 * q + 2] = fa.z;
        ra[4 * q + 3] = fa.w;
        rb[4 * q] = fb.x;
        rb[4 * q + 1] = fb.y;
        rb[4 * q + 2] = fb.z;
        rb[4 * q + 3] = fb.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int p = p0 + q;
        const int pc = p < N ? p : N - 1;
        ra[q] = as[pc];
        rb[q] = bs[pc];
        const uint32_t bit = p < N ? 0u : (1u << q);
        amask |= bit;
        bmask |= bit;
      }
    }
  };
  auto store = [&](uint16_t* buf) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      ra[q] = (amask >> q) & 1u ? 0.0f : ra[q];
      rb[q] = (bmask >> q) & 1u ? 0.0f : rb[q];
    }
    uint16_t* ah = buf + srow * kLDR + shalf;
    store_split<16>(ra, ah, ah + T::A_ELEMS);
    uint16_t* bh = buf + 2 * T::A_ELEMS + srow * kLDR + shalf;
    store_split<16>(rb, bh, bh + T::B_ELEMS);
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
    store(lds);
  }
  __syncthreads();
  for (long long ks = k0; ks < k1; ++ks) {
    if (ks + 1 < k1) load(ks + 1);
    tile_mfma<128, 128>(lds, wr, wc, r, h, acc);
    __syncthreads();
    if (ks + 1 < k1) store(lds);
    __syncthreads();
  }
  float* pb = part + (size_t)sp * cout * cin;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int o = co0 + wr * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int c = ci0 + wc * 64 + j * 32 + r;
        if (o < cout && c < cin) pb[(size_t)o * cin + c] = acc[i][j][e];
      }
}

// Wide form for cout, cin multiples of 256 (one 256 x 256 tile): 512 threads,
// 8 waves of 64 (co) x 128 (ci), so dY and x rows are each read once per
// K-range instead of cin/128 resp. cout/128 times; 80 KiB LDS, one block per CU.
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
    pw_wgrad256_kernel(const Parts x, const float* __restrict__ dy, int B, int cin, int cout,
                       int N, int S, float* __restrict__ part) {
  constexpr int TM = 256, TN = 256;
  constexpr int A_ELEMS = TM * kLDR, B_ELEMS = TN * kLDR;
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * A_ELEMS + 2 * B_ELEMS];
  const int nco = cout / TM;
  const int co0 = (blockIdx.x % nco) * TM, ci0 = (blockIdx.x / nco) * TN;
  const int sp = blockIdx.y;
  const int steps_per_b = (N + kKT - 1) / kKT;
  const long long nsteps = (long long)B * steps_per_b;
  const long long k0 = nsteps * sp / S, k1 = nsteps * (sp + 1) / S;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1, r = lane & 31, h = lane >> 5;  // wr 0..3 (co), wc 0..1 (ci)
  const int srow = t >> 1, shalf = (t & 1) * 16;                     // row 0..255, 16-point half
  const int co = co0 + srow, ci = ci0 + srow;
  // a ragged last input-channel tile (cin % 256 != 0): rows past cin read the
  // last row and are zeroed
  const bool ciok = ci < cin;
  const int cic = ciok ? ci : cin - 1;
  const bool vec = (N & 3) == 0;
  const float* __restrict__ xrow = x.row(0, cic, N);
  const size_t xbstride = (size_t)(x.row(1, cic, N) - xrow);

  float ra[16], rb[16];
  uint32_t pmask = 0u;
  auto load = [&](long long ks) {
    const int b = (int)(ks / steps_per_b);
    const int p0 = (int)(ks - (long long)b * steps_per_b) * kKT + shalf;
    const float* as = dy + ((size_t)b * cout + co) * N;
    const float* bs = xrow + (size_t)b * xbstride;
    pmask = 0u;
    if (vec && p0 + 16 <= N) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 fa = *reinterpret_cast<const float4*>(as + p0 + 4 * q);
        const float4 fb = *reinterpret_cast<const float4*>(bs + p0 + 4 * q);
        ra[4 * q] = fa.x;
        ra[4 * q + 1] = fa.y;
        ra[4 * q + 2] = fa.z;
        ra[4 * q + 3] = fa.w;
        rb[4 * q] = fb.x;
        rb[4 * q + 1] = fb.y;
        rb[4 * q + 2] = fb.z;
        rb[4 * q + 3] = fb.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int p = p0 + q;
        const int pc = p < N ? p : N - 1;
        ra[q] = as[pc];
        rb[q] = bs[pc];
        pmask |= p < N ? 0u : (1u << q);
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      ra[q] = (pmask >> q) & 1u ? 0.0f : ra[q];
      rb[q] = ((pmask >> q) & 1u) || !ciok ? 0.0f : rb[q];
    }
    uint16_t* ah = lds + srow * kLDR + shalf;
    store_split<16>(ra, ah, ah + A_ELEMS);
    uint16_t* bh = lds + 2 * A_ELEMS + srow * kLDR + shalf;
    store_split<16>(rb, bh, bh + B_ELEMS);
  };

  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  if (k0 < k1) {
    load(k0);
    store();
  }
  __syncthreads();
  for (long long ks = k0; ks < k1; ++ks) {
    if (ks + 1 < k1) load(ks + 1);
#pragma unroll
    for (int kk = 0; kk < kKT / 16; ++kk) {
      bf16x8 ah[2], al[2], bh[4], bl[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int o = (wr * 64 + i * 32 + r) * kLDR + kk * 16 + 8 * h;
        ah[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + o));
        al[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + A_ELEMS + o));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int o = 2 * A_ELEMS + (wc * 128 + j * 32 + r) * kLDR + kk * 16 + 8 * h;
        bh[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + o));
        bl[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(lds + B_ELEMS + o));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
    __syncthreads();
    if (ks + 1 < k1) store();
    __syncthreads();
  }
  float* pb = part + (size_t)sp * cout * cin;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int o = co0 + wr * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int c = ci0 + wc * 128 + j * 32 + r;
        if (c < cin) pb[(size_t)o * cin + c] = acc[i][j][e];
      }
}

__global__ void __launch_bounds__(256)
    pw_wgrad_reduce_kernel(const float* __restrict__ part, size_t total, int S,
                           float* __restrict__ dw) {
  // 64 outputs per block; 4 thread groups take every 4th split, combined in
  // group order (deterministic), so a thread chains S / 4 dependent adds
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
  if (grp == 0 && i < total) dw[i] = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
}

bool pw_wgrad_wide(int cin, int cout) {
#ifdef PCFM_PW_NO256
  return false;
#else
  // (a ragged last input-channel tile is supported and masked, but measured
  // slower than the 128 x 128 tiles for ContextNet head_pre, cin = 640: 378 vs
  // 290 us -- one block per CU over a half-empty third tile)
  return cin % 256 == 0 && cout % 256 == 0;
#endif
}

int pw_wgrad_splits(int B, int cin, int cout, int N) {
  if (pw_wgrad_wide(cin, cout)) {  // one 512-thread block per CU
    const long long tiles = (long long)(cout / 256) * ((cin + 255) / 256);
    const long long steps = (long long)B * ((N + kKT - 1) / kKT);
    long long s = std::max(1LL, ((long long)kCUs + tiles - 1) / tiles);
    s = std::min(s, std::max(1LL, steps / 16));
    return (int)std::min(s, 256LL);
  }
#ifndef PCFM_PW_WG_BPC
#define PCFM_PW_WG_BPC 2  // target blocks per CU
#endif
#ifndef PCFM_PW_WG_MINSTEPS
#define PCFM_PW_WG_MINSTEPS 8  // K-steps per split at least
#endif
#ifndef PCFM_PW_WG_CAP
#define PCFM_PW_WG_CAP 512  // splits at most (128: 72 -> 49 us at C128, tools/pw_ab.py)
#endif
  const long long tiles = (long long)((cout + 127) / 128) * ((cin + 127) / 128);
  const long long steps = (long long)B * ((N + kKT - 1) / kKT);
  long long s = std::max(1LL, ((long long)PCFM_PW_WG_BPC * kCUs + tiles - 1) / tiles);
  s = std::min(s, std::max(1LL, steps / PCFM_PW_WG_MINSTEPS));
  return (int)std::min(s, (long long)PCFM_PW_WG_CAP);
}

bool pw_ok(int b, int cin, int cout, int n) {
  return b >= 0 && cin > 0 && cout > 0 && n >= 0 && (long long)cin * n < (1LL << 31) &&
         (long long)cout * n < (1LL << 31);
}

}  // namespace
}  // namespace pcfm

using namespace pcfm;

extern "C" size_t pcfm_pointwise_weight_bytes(int cout, int cin) {
  if (cout <= 0 || cin <= 0) return 0;
  const size_t a = (size_t)pw_mpad(cout) * pad_to(cin, kKT);
  const size_t b = (size_t)pw_mpad(cin) * pad_to(cout, kKT);
  return 2 * std::max(a, b) * sizeof(uint16_t);
}

extern "C" int pcfm_pointwise_prep_weight(const float* w, int cout, int cin, int transpose,
                                          void* wsplit, void* stream) {
  PCFM_CHECK_ARG(cout > 0 && cin > 0, "pointwise_prep_weight: bad size %d x %d", cout, cin);
  const int M = transpose ? cin : cout, K = transpose ? cout : cin;
  const int Mpad = pw_mpad(M), Kpad = pad_to(K, kKT);
  const size_t total = (size_t)Mpad * Kpad;
  uint16_t* wh = (uint16_t*)wsplit;
  hipLaunchKernelGGL(pw_wsplit_kernel, dim3(ceil_div((long long)total, 256)), dim3(256), 0,
                     (hipStream_t)stream, w, cout, cin, transpose ? 1 : 0, Mpad, Kpad, wh,
                     wh + total);
  return check_launch("pointwise_prep_weight");
}

// The forward GEMM's kernel for a shape: ONE decision, used by the launcher
// and by pcfm_pointwise_bnstats_groups(), so a caller is never told that a
// shape writes BatchNorm statistics when the kernel that runs does not.
// (Measured and removed in round 6, with their A/B final: the 128-row streaming
// kernel in 128-row slices for M > 128 -- correct, slower: 256->256 forward 98.9
// vs 88.9 us, profiles/r05_ab_pw_stream_m.jsonl -- and the persistent LDS-DMA
// 256-row form -- bit-identical, 106.6 vs 94.0 us, profiles/r05_ab_pw_glds256.jsonl.)
enum class PwPath { Stream128, Tile256, Tile128, Tile64 };

static PwPath pw_path(int b, int cin, int cout, int n) {
  const int Mpad = pw_mpad(cout), Kpad = pad_to(cin, kKT);
  const long long big = (long long)ceil_div(n, 128) * (Mpad / 128) * b;
#ifndef PCFM_PW_NOSTREAM
  if (Mpad == 128 && Kpad <= 256 && cin % 32 == 0 && cout % 32 == 0) return PwPath::Stream128;
#endif
#ifndef PCFM_PW_NO256
  if (Mpad % 256 == 0 && big / 2 >= 2 * kCUs) return PwPath::Tile256;
#endif
  return big >= 2 * kCUs ? PwPath::Tile128 : PwPath::Tile64;
}

// The 256-row tiles (64-point groups) and the 128-row streaming form (32-point
// groups) have the statistics epilogue.
static bool pw_path_has_stats(PwPath p) {
  if (p == PwPath::Stream128) {  // PCFM_PW_STREAM_STATS=0: measurement switch
    const char* e = std::getenv("PCFM_PW_STREAM_STATS");
    return PCFM_PW_STREAM_PF < 2 && (e == nullptr || e[0] != '0');
  }
  return p == PwPath::Tile256;
}
static int pw_stats_group(PwPath p) { return p == PwPath::Stream128 ? 32 : 64; }

static int pw_gemm_launch(const Parts& x, const void* wsplit, const float* bias, int bias_bstride,
                          int b, int cin, int cout, int n, const Parts& y, hipStream_t st,
                          float2* stats = nullptr) {
  const int Mpad = pw_mpad(cout), Kpad = pad_to(cin, kKT);
  const size_t total = (size_t)Mpad * Kpad;
  const uint16_t* wh = (const uint16_t*)wsplit;
  const PwPath path = pw_path(b, cin, cout, n);
  // a statistics request the chosen kernel cannot serve fails loudly (it used
  // to be dropped, leaving the caller's stats buffer unwritten)
  PCFM_CHECK_ARG(stats == nullptr || pw_path_has_stats(path),
                 "pointwise_gemm: BatchNorm statistics requested for a shape whose kernel has "
                 "no statistics epilogue (b=%d cin=%d cout=%d n=%d)", b, cin, cout, n);
  if (path == PwPath::Stream128) {
    const uint16_t* wl_img = wh + total;
    const long long tiles = (long long)b * ceil_div(n, 32);
    const size_t lds = (size_t)2 * 128 * (Kpad + 8) * sizeof(uint16_t);
    const int per_cu = lds <= 80 * 1024 ? 2 : 1;
    const int slices = Mpad / 128;
    // the slices share the chip: grid.x a multiple of 8 (XCD pairing, see the kernel)
    const long long cap = std::max(8LL, ((long long)kCUs * per_cu / slices) & ~7LL);
    const int grid = (int)std::max(1LL, std::min((tiles + kSW - 1) / kSW, cap));
    const void* kfn = nullptr;
    switch (Kpad / 32) {
#define PW_STREAM_CASE(NC)                                                                 \
  case NC:                                                                                 \
    kfn = stats != nullptr ? (const void*)pw_stream128_kernel<NC, true>                    \
                           : (const void*)pw_stream128_kernel<NC, false>;                  \
    break;
      PW_STREAM_CASE(1) PW_STREAM_CASE(2) PW_STREAM_CASE(3) PW_STREAM_CASE(4)
      PW_STREAM_CASE(5) PW_STREAM_CASE(6) PW_STREAM_CASE(7) PW_STREAM_CASE(8)
#undef PW_STREAM_CASE
    }
    const int e = allow_big_lds(kfn);
    if (e) return e;
    void* args[] = {(void*)&x,    (void*)&wh,  (void*)&wl_img, (void*)&bias,
                    (void*)&bias_bstride, (void*)&y, (void*)&cin, (void*)&cout,
                    (void*)&n,    (void*)&b,   (void*)&stats};
    const hipError_t le = hipLaunchKernel(kfn, dim3(grid, slices), dim3(kSW * 64), args, lds, st);
    if (le != hipSuccess) {
      set_error("pointwise_gemm: launch failed");
      return (int)le;
    }
    return check_launch("pointwise_gemm");
  }
  if (path == PwPath::Tile256) {
    const dim3 g256(ceil_div(n, 128), Mpad / 256, b);
    hipLaunchKernelGGL(pw_gemm256_kernel, g256, dim3(512), 0, st, x, wh, wh + total, bias,
                       bias_bstride, y, cin, cout, n, Kpad, stats);
    return check_launch("pointwise_gemm");
  }
  if (path == PwPath::Tile128) {
    hipLaunchKernelGGL((pw_gemm_kernel<128, 128>), dim3(ceil_div(n, 128), Mpad / 128, b),
                       dim3(256), 0, st, x, wh, wh + total, bias, bias_bstride, y, cin, cout, n,
                       Kpad);
  } else {
    hipLaunchKernelGGL((pw_gemm_kernel<64, 64>), dim3(ceil_div(n, 64), Mpad / 64, b), dim3(256),
                       0, st, x, wh, wh + total, bias, bias_bstride, y, cin, cout, n, Kpad);
  }
  return check_launch("pointwise_gemm");
}

// host arrays -> Parts; every width a multiple of `align` (the last may be ragged)
static bool make_parts(int np, float* const* ptr, const int* width, int align, Parts& q,
                       int& total) {
  if (np < 1 || np > kMaxParts || ptr == nullptr || width == nullptr) return false;
  q = Parts{};
  q.n = np;
  total = 0;
  for (int i = 0; i < np; ++i) {
    if (width[i] <= 0 || ptr[i] == nullptr) return false;
    if (i + 1 < np && width[i] % align != 0) return false;
    q.p[i] = ptr[i];
    q.off[i] = total;
    total += width[i];
  }
  q.off[np] = total;
  for (int i = np + 1; i <= kMaxParts; ++i) q.off[i] = total;
  return true;
}

extern "C" int pcfm_pointwise_gemm(const float* x, const void* wsplit, const float* bias, int b,
                                   int cin, int cout, int n, float* y, void* stream) {
  PCFM_CHECK_ARG(pw_ok(b, cin, cout, n), "pointwise_gemm: bad shape b=%d cin=%d cout=%d n=%d", b,
                 cin, cout, n);
  if (b == 0 || n == 0) return PCFM_OK;
  return pw_gemm_launch(one_part(x, cin), wsplit, bias, 0, b, cin, cout, n, one_part(y, cout),
                        (hipStream_t)stream);
}

// y = W x + bias with the BatchNorm statistics of y per (channel, 64-point
// group): stats float2 [cout][b * ceil(n / 64)] (mean, centred sum of squares);
// pcfm_pointwise_bnstats_groups() > 0 for the shapes that take this path.
extern "C" int pcfm_pointwise_bnstats_groups(int b, int cin, int cout, int n) {
  if (!pw_ok(b, cin, cout, n) || b <= 0 || n <= 0) return 0;
  const PwPath p = pw_path(b, cin, cout, n);
  if (!pw_path_has_stats(p)) return 0;
  return b * ceil_div(n, pw_stats_group(p));
}

extern "C" int pcfm_pointwise_gemm_bnstats(const float* x, const void* wsplit, const float* bias,
                                           int b, int cin, int cout, int n, float* y,
                                           float* stats, void* stream) {
  PCFM_CHECK_ARG(pcfm_pointwise_bnstats_groups(b, cin, cout, n) > 0 && stats != nullptr,
                 "pointwise_gemm_bnstats: unsupported shape b=%d cin=%d cout=%d n=%d", b, cin,
                 cout, n);
  return pw_gemm_launch(one_part(x, cin), wsplit, bias, 0, b, cin, cout, n, one_part(y, cout),
                        (hipStream_t)stream, reinterpret_cast<float2*>(stats));
}

extern "C" int pcfm_pointwise_gemm_parts(int nx, const float* const* x, const int* xw,
                                         const void* wsplit, const float* bias, int bias_per_batch,
                                         int b, int n, int ny, float* const* y, const int* yw,
                                         void* stream) {
  Parts px, py;
  int cin = 0, cout = 0;
  PCFM_CHECK_ARG(make_parts(nx, const_cast<float* const*>(x), xw, kKT, px, cin),
                 "pointwise_gemm_parts: bad input parts (1..%d, widths %% %d)", kMaxParts, kKT);
  PCFM_CHECK_ARG(make_parts(ny, y, yw, 128, py, cout),
                 "pointwise_gemm_parts: bad output parts (1..%d, widths %% 128)", kMaxParts);
  PCFM_CHECK_ARG(pw_ok(b, cin, cout, n), "pointwise_gemm_parts: bad shape b=%d cin=%d cout=%d n=%d",
                 b, cin, cout, n);
  if (b == 0 || n == 0) return PCFM_OK;
  return pw_gemm_launch(px, wsplit, bias, bias_per_batch ? cout : 0, b, cin, cout, n, py,
                        (hipStream_t)stream);
}

static int pw_wgrad_launch(const Parts& x, const float* grad_y, int b, int cin, int cout, int n,
                           float* grad_w, void* ws, hipStream_t st) {
  const size_t total = (size_t)cout * cin;
  const int S = pw_wgrad_splits(b, cin, cout, n);
  if (pw_wgrad_wide(cin, cout)) {
    hipLaunchKernelGGL(pw_wgrad256_kernel, dim3((cout / 256) * ((cin + 255) / 256), S), dim3(512), 0, st,
                       x, grad_y, b, cin, cout, n, S, (float*)ws);
  } else {
    const int tiles = ((cout + 127) / 128) * ((cin + 127) / 128);
    hipLaunchKernelGGL(pw_wgrad_kernel, dim3(tiles, S), dim3(256), 0, st, x, grad_y, b, cin,
                       cout, n, S, (float*)ws);
  }
  hipLaunchKernelGGL(pw_wgrad_reduce_kernel, dim3(ceil_div((long long)total, 64)), dim3(256), 0,
                     st, (const float*)ws, total, S, grad_w);
  return check_launch("pointwise_wgrad");
}

extern "C" size_t pcfm_pointwise_wgrad_workspace_bytes(int b, int cin, int cout, int n) {
  if (!pw_ok(b, cin, cout, n) || b == 0 || n == 0) return 0;
  return (size_t)pw_wgrad_splits(b, cin, cout, n) * cout * cin * sizeof(float);
}

extern "C" int pcfm_pointwise_wgrad(const float* x, const float* grad_y, int b, int cin, int cout,
                                    int n, float* grad_w, void* ws, size_t ws_bytes,
                                    void* stream) {
  PCFM_CHECK_ARG(pw_ok(b, cin, cout, n), "pointwise_wgrad: bad shape b=%d cin=%d cout=%d n=%d",
                 b, cin, cout, n);
  hipStream_t st = (hipStream_t)stream;
  const size_t total = (size_t)cout * cin;
  if (b == 0 || n == 0) {
    const hipError_t e = hipMemsetAsync(grad_w, 0, total * sizeof(float), st);
    if (e != hipSuccess) {
      set_error("pointwise_wgrad: hipMemsetAsync: %s", hipGetErrorString(e));
      return (int)e;
    }
    return PCFM_OK;
  }
  const size_t need = pcfm_pointwise_wgrad_workspace_bytes(b, cin, cout, n);
  PCFM_CHECK_ARG(ws_bytes >= need, "pointwise_wgrad: workspace %zu < %zu bytes", ws_bytes, need);
  return pw_wgrad_launch(one_part(x, cin), grad_y, b, cin, cout, n, grad_w, ws, st);
}

extern "C" int pcfm_pointwise_wgrad_parts(int nx, const float* const* x, const int* xw,
                                          const float* grad_y, int b, int cout, int n,
                                          float* grad_w, void* ws, size_t ws_bytes, void* stream) {
  Parts px;
  int cin = 0;
  PCFM_CHECK_ARG(make_parts(nx, const_cast<float* const*>(x), xw, 1, px, cin),
                 "pointwise_wgrad_parts: bad input parts (1..%d)", kMaxParts);
  PCFM_CHECK_ARG(pw_ok(b, cin, cout, n) && b > 0 && n > 0,
                 "pointwise_wgrad_parts: bad shape b=%d cin=%d cout=%d n=%d", b, cin, cout, n);
  const size_t need = pcfm_pointwise_wgrad_workspace_bytes(b, cin, cout, n);
  PCFM_CHECK_ARG(ws_bytes >= need, "pointwise_wgrad_parts: workspace %zu < %zu bytes", ws_bytes,
                 need);
  return pw_wgrad_launch(px, grad_y, b, cin, cout, n, grad_w, ws, (hipStream_t)stream);
}
