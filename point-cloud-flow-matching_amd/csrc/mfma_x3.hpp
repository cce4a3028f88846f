// bf16x3 matrix-core machinery shared by the voxel convolution (conv3d.hip)
// and the pointwise (1x1) convolution (pointwise.hip).
//
// Every fp32 operand x is split into hi = bf16(x) and lo = bf16(x - hi);
// a*b ~= ah*bh + ah*bl + al*bh with fp32 accumulation in the MFMA (the al*bl
// term, ~2^-16 relative, is dropped).  A 256-thread block (2 x 2 waves)
// accumulates a TM x TN fp32 tile from LDS images of bf16 hi/lo rows, K-steps
// of 32, via v_mfma_f32_32x32x16_bf16 (cdna_hip_programming.md section 3 maps).
#pragma once

#include "pcfm_common.hpp"

namespace pcfm {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// round-to-nearest-even fp32 -> bf16 bits (finite inputs)
__device__ __forceinline__ uint32_t bf16_bits(float x) {
  uint32_t u = __float_as_uint(x);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return u >> 16;
}
__device__ __forceinline__ void split_bf16(float x, uint32_t& hi, uint32_t& lo) {
  hi = bf16_bits(x);
  lo = bf16_bits(x - __uint_as_float(hi << 16));
}

constexpr int kMT = 128;  // rows of D (output channels) per block
constexpr int kNT = 128;  // voxels per block
constexpr int kKT = 32;   // reduction channels per K-step
constexpr int kLDR = 40;  // LDS row stride in bf16 (80 B: conflict-free ds_read_b128 rows)

// ---------------------------------------------------------------------------
// Shared block machinery: a 256-thread block (2 x 2 waves) computes a TM x TN
// fp32 tile D += A[TM][k] * B[TN][k]^T over K-steps of 32, from LDS images of
// bf16 hi/lo rows (kLDR-strided).  Register-prefetched: the global loads of
// step s+1 are issued before step s's MFMAs and split + written to LDS after
// them, so the load latency hides behind 24 (TM = TN = 128) MFMAs per wave.
// One LDS buffer (two barriers per step) keeps 40 KB per block, i.e. several
// blocks per CU -- measured faster than two buffers at one block per CU.
// ---------------------------------------------------------------------------
#ifndef PCFM_CONV_NBUF
#define PCFM_CONV_NBUF 1
#endif
constexpr int kNBuf = PCFM_CONV_NBUF;  // LDS buffers: 1 = more blocks per CU, 2 = one barrier

template <int TM, int TN>
struct Tile {
  static constexpr int SI = TM / 64, SJ = TN / 64;  // 32x32 MFMA tiles per wave
  static constexpr int A_ELEMS = TM * kLDR, B_ELEMS = TN * kLDR;
  // one buffer: Ah | Al | Bh | Bl
  static constexpr int BUF = 2 * A_ELEMS + 2 * B_ELEMS;
};

template <int TM, int TN>
__device__ __forceinline__ void tile_mfma(const uint16_t* buf, int wr, int wc, int r, int h,
                                          f32x16 (&acc)[TM / 64][TN / 64]) {
  using T = Tile<TM, TN>;
  const uint16_t* sAh = buf;
  const uint16_t* sAl = buf + T::A_ELEMS;
  const uint16_t* sBh = buf + 2 * T::A_ELEMS;
  const uint16_t* sBl = sBh + T::B_ELEMS;
#pragma unroll
  for (int kk = 0; kk < kKT / 16; ++kk) {
    bf16x8 ah[T::SI], al[T::SI], bh[T::SJ], bl[T::SJ];
#pragma unroll
    for (int i = 0; i < T::SI; ++i) {
      const int o = (wr * (TM / 2) + i * 32 + r) * kLDR + kk * 16 + 8 * h;
      ah[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sAh + o));
      al[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sAl + o));
    }
#pragma unroll
    for (int j = 0; j < T::SJ; ++j) {
      const int o = (wc * (TN / 2) + j * 32 + r) * kLDR + kk * 16 + 8 * h;
      bh[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sBh + o));
      bl[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sBl + o));
    }
#pragma unroll
    for (int i = 0; i < T::SI; ++i)
#pragma unroll
      for (int j = 0; j < T::SJ; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
      }
  }
}

// split N consecutive fp32 (same LDS row) into the hi and lo images.  The
// (__bf16) casts round to nearest even and lower to gfx950's packed
// v_cvt_pk_bf16_f32 (one instruction per pair), hi is widened back exactly.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
template <int N>
__device__ __forceinline__ void store_split(const float (&v)[N], uint16_t* dh, uint16_t* dl) {
  uint32_t* h32 = reinterpret_cast<uint32_t*>(dh);
  uint32_t* l32 = reinterpret_cast<uint32_t*>(dl);
#pragma unroll
  for (int q = 0; q < N / 2; ++q) {
    bf16x2 hi;
    hi.x = (__bf16)v[2 * q];
    hi.y = (__bf16)v[2 * q + 1];
    bf16x2 lo;
    lo.x = (__bf16)(v[2 * q] - (float)hi.x);
    lo.y = (__bf16)(v[2 * q + 1] - (float)hi.y);
    h32[q] = __builtin_bit_cast(uint32_t, hi);
    l32[q] = __builtin_bit_cast(uint32_t, lo);
  }
}


// Staging registers as one vector value per operand image (an array of uint4
// captured by the load/store lambdas is placed in scratch by hipcc).
template <int Q>
using StageVec = unsigned int __attribute__((ext_vector_type(4 * Q)));
template <int Q>
__device__ __forceinline__ void sv_put(StageVec<Q>& v, int q, uint4 x) {
  v[4 * q] = x.x;
  v[4 * q + 1] = x.y;
  v[4 * q + 2] = x.z;
  v[4 * q + 3] = x.w;
}
template <int Q>
__device__ __forceinline__ uint4 sv_get(const StageVec<Q>& v, int q) {
  return uint4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
}

// ---------------------------------------------------------------------------
// Transposed-read images (cdna_hip_programming.md T10): a [rows][128] bf16
// tile stored as it lies in memory (256-B rows, 16-B chunks XOR-swizzled) and
// read with ds_read_b64_tr_b16, which delivers 4 consecutive ROWS of one
// column per lane -- the MFMA operand for a reduction over the row index.
// ---------------------------------------------------------------------------
typedef short v4s_tr __attribute__((ext_vector_type(4)));

// byte offset of 16-B chunk `ch` (0..15) of row `row` (the T10 (b) swizzle)
__device__ __forceinline__ int swz256(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ v4s_tr tr_read16(const uint8_t* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s_tr*)(base + off));
}

// 32x32x16 operand (8 consecutive rows kk*16 + 8*(lane/32) .. +8 of column
// col0 + lane%32) from a swizzled [rows][128] image
__device__ __forceinline__ bf16x8 tr_operand(const uint8_t* img, int kk, int col0, int lane) {
  const int g = lane >> 4, i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;
  const int row = kk * 16 + 8 * (g >> 1) + q4;
  const int col = col0 + (g & 1) * 16 + 4 * p4;
  const v4s_tr x0 = tr_read16(img, swz256(row, col >> 3) + 8 * (p4 & 1));
  const v4s_tr x1 = tr_read16(img, swz256(row + 4, col >> 3) + 8 * (p4 & 1));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
}

// ---------------------------------------------------------------------------
// Epilogue bias of one 32x32 accumulator: element e of lane half h is row
// mg + (e & 3) + 8 (e >> 2) + 4 h.  All 16 values are loaded before the
// tile's first store: vmcnt counts stores too, so a bias load placed after
// a store waits for that store's acknowledgement -- 16-64 serialised round
// trips per wave in the fused-add form.  Rows >= M read row M - 1 (unused).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_bias16(const float* __restrict__ bias, int mg, int h, int M,
                                            float (&bv)[16]) {
#pragma unroll
  for (int e = 0; e < 16; ++e)
    bv[e] = bias != nullptr ? bias[min(mg + (e & 3) + 8 * (e >> 2) + 4 * h, M - 1)] : 0.0f;
}

}  // namespace
}  // namespace pcfm
