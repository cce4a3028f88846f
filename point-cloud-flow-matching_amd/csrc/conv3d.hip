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

#include "mfma_x3.hpp"

namespace pcfm {
namespace {

// W [Cout][Cin][27] fp32 -> W' [27][M][K] bf16 hi, lo (see header)
__global__ void __launch_bounds__(256)
    conv3_wsplit_kernel(const float* __restrict__ w, int cout, int cin, int transpose,
                        uint16_t* __restrict__ wh, uint16_t* __restrict__ wl) {
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
  wh[i] = (uint16_t)hi;
  wl[i] = (uint16_t)lo;
}

// ---------------------------------------------------------------------------
// Forward / backward-data implicit GEMM.
// grid = (V / TN, M / TM, B); K-steps s = tap * (K / 32) + channel chunk.
// A = pre-split weights W'[tap][m][k] (bf16 hi, lo), B = input voxels split
// on the fly.  TM = TN = 128 normally, 64 for the small r = 8 grids.
// ---------------------------------------------------------------------------
template <int TM, int TN>
__global__ void __launch_bounds__(256)
    conv3_igemm_kernel(const float* __restrict__ x, const uint16_t* __restrict__ wh,
                       const uint16_t* __restrict__ wl, const float* __restrict__ bias,
                       float* __restrict__ y, int K, int M, int R) {
  using T = Tile<TM, TN>;
  __shared__ __attribute__((aligned(16))) uint16_t lds[kNBuf * T::BUF];
  const int V = R * R * R, R2 = R * R;
  const int b = blockIdx.z, m0 = blockIdx.y * TM, v0 = blockIdx.x * TN;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1, r = lane & 31, h = lane >> 5;
  const float* __restrict__ xb = x + (size_t)b * K * V;

  // B staging: thread t owns voxel v0 + (t % TN) and CPT of the 32 channels
  constexpr int CPT = kKT * TN / 256;  // 16 (TN = 128) or 8 (TN = 64)
  const int sv = t % TN, ch = (t / TN) * CPT;
  const int vs = v0 + sv;
  const int xs = vs / R2, ys = (vs / R) % R, zs = vs % R;
  // A staging: threads < 2*TM own 16 bf16 (32 B) of weight row t >> 1
  const bool astage = 2 * TM >= 256 || t < 2 * TM;
  const int arow = t >> 1, ahalf = (t & 1) * 16;
  const int nck = K / kKT, nsteps = 27 * nck;

  uint4 ra0 = {}, ra1 = {}, ra2 = {}, ra3 = {};  // named: an array here went to scratch
  float rb[CPT];
  bool rb_ok = true;
  auto load = [&](int s) {
    const int tap = s / nck, c0 = (s - tap * nck) * kKT;
    if (astage) {
      const size_t g = ((size_t)tap * M + m0 + arow) * K + c0 + ahalf;
      ra0 = *reinterpret_cast<const uint4*>(wh + g);
      ra1 = *reinterpret_cast<const uint4*>(wh + g + 8);
      ra2 = *reinterpret_cast<const uint4*>(wl + g);
      ra3 = *reinterpret_cast<const uint4*>(wl + g + 8);
    }
    const int dx = tap / 9 - 1, dy = (tap / 3) % 3 - 1, dz = tap % 3 - 1;
    const bool inb = (unsigned)(xs + dx) < (unsigned)R && (unsigned)(ys + dy) < (unsigned)R &&
                     (unsigned)(zs + dz) < (unsigned)R;
    // branch-free: out-of-grid lanes load their own voxel and are zeroed in
    // store() -- after the MFMAs, so no wait lands in front of them
    const float* src = xb + (size_t)(c0 + ch) * V + (inb ? vs + dx * R2 + dy * R + dz : vs);
#pragma unroll
    for (int q = 0; q < CPT; ++q) rb[q] = src[(size_t)q * V];
    rb_ok = inb;
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
    uint16_t* bh = buf + 2 * T::A_ELEMS + sv * kLDR + ch;
#pragma unroll
    for (int q = 0; q < CPT; ++q) rb[q] = rb_ok ? rb[q] : 0.0f;
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
    uint16_t* cur = lds + (kNBuf == 2 ? (s & 1) * T::BUF : 0);
    if (s + 1 < nsteps) load(s + 1);  // next step's loads fly during the MFMAs
    tile_mfma<TM, TN>(cur, wr, wc, r, h, acc);
    if constexpr (kNBuf == 1) __syncthreads();
    if (s + 1 < nsteps) store(lds + (kNBuf == 2 ? ((s + 1) & 1) * T::BUF : 0));
    __syncthreads();
  }
  // epilogue: D[m][v], column v = lane & 31 -> 128-B coalesced rows of NCDHW
  float* __restrict__ yb = y + (size_t)b * M * V;
#pragma unroll
  for (int i = 0; i < T::SI; ++i)
#pragma unroll
    for (int j = 0; j < T::SJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + wr * (TM / 2) + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int v = v0 + wc * (TN / 2) + j * 32 + r;
        yb[(size_t)m * V + v] = acc[i][j][e] + (bias != nullptr ? bias[m] : 0.0f);
      }
}

// ---------------------------------------------------------------------------
// Weight gradient: dW[co, ci, tap] = sum_{b, v} dY[b, co, v] * X[b, ci, v + off(tap)]
// One GEMM per tap with K = B*V voxels: A = dY tile [co][voxel], B = shifted X
// tile [ci][voxel] -- both are voxel-contiguous rows of the NCDHW tensors, so
// the A/B fragments (8 consecutive k per lane) come straight from LDS rows.
// 27 * (Cout/128) * (Cin/128) tiles x S voxel splits (1-D grid); each
// block writes an fp32 partial [s][tap][co][ci]; conv3_wgrad_reduce_kernel
// sums the S partials in split order into dW [co][ci][27].
// ---------------------------------------------------------------------------
constexpr int kWK = 32;  // voxels per K-step

__global__ void __launch_bounds__(256)
    conv3_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy, int B, int cin,
                       int cout, int R, int S, float* __restrict__ part) {
  using T = Tile<128, 128>;
  __shared__ __attribute__((aligned(16))) uint16_t lds[kNBuf * T::BUF];
  const int V = R * R * R, R2 = R * R;
  const int nco = cout / kMT;
  // 1-D grid of items ((ci tile * nco + co tile) * S + split) * 27 + tap, dealt
  // to XCDs in contiguous runs (bijective remap, cdna_hip_programming.md T1):
  // the 27 taps of one (tile, voxel range) share the dY rows and overlapping X
  // rows, so they should meet in one XCD's L2 instead of all re-reading HBM.
  int id = (int)blockIdx.x;
#ifndef PCFM_WGRAD_NOSWZ
  {
    const int nwg = (int)gridDim.x, q = nwg / 8, rr = nwg % 8, xcd = id % 8;
    id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + id / 8;
  }
#endif
  const int tap = id % 27;
  id /= 27;
  const int sp = id % S;
  id /= S;
  const int co0 = (id % nco) * kMT;
  const int ci0 = (id / nco) * kMT;
  const int steps_per_b = V / kWK;
  const long long nsteps = (long long)B * steps_per_b;
  const long long k0 = nsteps * sp / S, k1 = nsteps * (sp + 1) / S;
  const int dx = tap / 9 - 1, dy_ = (tap / 3) % 3 - 1, dz = tap % 3 - 1;
  const int off = dx * R2 + dy_ * R + dz;

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = w >> 1, wc = w & 1, r = lane & 31, h = lane >> 5;
  const int srow = t >> 1, shalf = (t & 1) * 16;  // staging: row, 16 voxels

  float ra[16], rb[16];
  uint32_t rmask = 0u;  // out-of-grid voxels of rb, zeroed in store()
  auto load = [&](long long ks) {
    const int b = (int)(ks / steps_per_b);
    const int v0 = (int)(ks - (long long)b * steps_per_b) * kWK + shalf;
    const float4* asrc =
        reinterpret_cast<const float4*>(dy + ((size_t)b * cout + co0 + srow) * V + v0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 f = asrc[q];
      ra[4 * q] = f.x;
      ra[4 * q + 1] = f.y;
      ra[4 * q + 2] = f.z;
      ra[4 * q + 3] = f.w;
    }
    // B: X[b, ci0 + srow, v + off] for v = v0 .. v0+15, as two 8-voxel halves
    // (R % 8 == 0, so a half never crosses a z-row).  Each half loads 8
    // aligned floats at its row's base (off - dz is a multiple of 8) plus one
    // neighbour for dz = -1 / +1 and shifts; out-of-grid voxels are recorded
    // in rmask and zeroed in store().
    const float* bsrc = x + ((size_t)b * cin + ci0 + srow) * V;
    rmask = 0u;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int vh = v0 + 8 * hh;
      const int xq = vh / R2, yq = (vh / R) % R, zq = vh % R;
      const bool rowok = (unsigned)(xq + dx) < (unsigned)R && (unsigned)(yq + dy_) < (unsigned)R;
      const int base = rowok ? vh + off - dz : vh;  // always inside this (b, ci) row
      const float4 f0 = *reinterpret_cast<const float4*>(bsrc + base);
      const float4 f1 = *reinterpret_cast<const float4*>(bsrc + base + 4);
      const float e = bsrc[dz < 0 ? max(base - 1, 0) : min(base + 8, V - 1)];
      const float g[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j)
        rb[8 * hh + j] = dz == 0 ? g[j] : dz < 0 ? (j == 0 ? e : g[j - 1]) : (j == 7 ? e : g[j + 1]);
      uint32_t m = rowok ? 0u : 0xFFu;
      if (dz < 0 && zq == 0) m |= 1u;
      if (dz > 0 && zq + 7 == R - 1) m |= 0x80u;
      rmask |= m << (8 * hh);
    }
  };
  auto store = [&](uint16_t* buf) {
    uint16_t* ah = buf + srow * kLDR + shalf;
    store_split<16>(ra, ah, ah + T::A_ELEMS);
    uint16_t* bh = buf + 2 * T::A_ELEMS + srow * kLDR + shalf;
#pragma unroll
    for (int q = 0; q < 16; ++q) rb[q] = (rmask >> q) & 1u ? 0.0f : rb[q];
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
    uint16_t* cur = lds + (kNBuf == 2 ? ((ks - k0) & 1) * T::BUF : 0);
#ifndef PCFM_EXP_NOLOAD
    if (ks + 1 < k1) load(ks + 1);
#endif
#ifndef PCFM_EXP_NOMFMA
    tile_mfma<128, 128>(cur, wr, wc, r, h, acc);
#endif
    if constexpr (kNBuf == 1) __syncthreads();
#ifndef PCFM_EXP_NOLOAD
    if (ks + 1 < k1) store(lds + (kNBuf == 2 ? ((ks + 1 - k0) & 1) * T::BUF : 0));
#endif
    __syncthreads();
  }
  // partial[s][tap][co][ci]: column ci = lane & 31 -> coalesced rows
  float* pb = part + ((size_t)sp * 27 + tap) * cout * cin;
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

// dw[co][ci][tap] = sum_s part[s][tap][co][ci], in split order
__global__ void __launch_bounds__(256)
    conv3_wgrad_reduce_kernel(const float* __restrict__ part, int cout, int cin, int S,
                              float* __restrict__ dw) {
  const size_t total = (size_t)27 * cout * cin;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // dw index
  if (i >= total) return;
  const int tap = (int)(i % 27);
  const size_t cc = i / 27;  // co * cin + ci
  const float* p = part + (size_t)tap * cout * cin + cc;
  const size_t ps = total;
  float sum = 0.0f;
  int q = 0;
  for (; q + 4 <= S; q += 4) {
    const float a0 = p[(size_t)q * ps], a1 = p[(size_t)(q + 1) * ps];
    const float a2 = p[(size_t)(q + 2) * ps], a3 = p[(size_t)(q + 3) * ps];
    sum = sum + a0;
    sum = sum + a1;
    sum = sum + a2;
    sum = sum + a3;
  }
  for (; q < S; ++q) sum = sum + p[(size_t)q * ps];
  dw[i] = sum;
}

#ifndef PCFM_WGRAD_OCC
#define PCFM_WGRAD_OCC 4
#endif
int conv3_wgrad_splits(int B, int cin, int cout, int R) {
  const long long tiles = 27LL * (cout / kMT) * (cin / kMT);
  const long long steps = (long long)B * R * R * R / kWK;
  // blocks per CU the split aims for (one block's staging overlaps another's MFMAs)
  long long s = std::max(1LL, ((long long)PCFM_WGRAD_OCC * kCUs + tiles - 1) / tiles);
  s = std::min(s, std::max(1LL, steps / 16));  // keep >= 16 K-steps per block
  return (int)std::min(s, 64LL);
}

bool conv3_shape_ok(int b, int cin, int cout, int r) {
  if (b < 0 || cin <= 0 || cout <= 0 || r <= 0 || r > 1024) return false;
  const long long v = (long long)r * r * r;
  return cin % kKT == 0 && cout % kMT == 0 && v % kNT == 0 && v < (1LL << 31);
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
  PCFM_CHECK_ARG(cout > 0 && cin > 0, "conv3d_prep_weight: bad size cout=%d cin=%d", cout, cin);
  const size_t total = (size_t)27 * cout * cin;
  uint16_t* wh = (uint16_t*)wsplit;
  hipLaunchKernelGGL(conv3_wsplit_kernel, dim3(ceil_div((long long)total, 256)), dim3(256), 0,
                     (hipStream_t)stream, w, cout, cin, transpose ? 1 : 0, wh, wh + total);
  return check_launch("conv3d_prep_weight");
}

extern "C" int pcfm_conv3d_supported(int b, int cin, int cout, int r) {
  return conv3_shape_ok(b, cin, cout, r) ? 1 : 0;
}

extern "C" int pcfm_conv3d_igemm(const float* x, const void* wsplit, const float* bias, int b,
                                 int cin, int cout, int r, float* y, void* stream) {
  PCFM_CHECK_ARG(conv3_shape_ok(b, cin, cout, r),
                 "conv3d_igemm: unsupported shape b=%d cin=%d cout=%d r=%d (need cin %% %d, "
                 "cout %% %d, r^3 %% %d == 0)",
                 b, cin, cout, r, kKT, kMT, kNT);
  if (b == 0) return PCFM_OK;
  const int V = r * r * r;
  const size_t total = (size_t)27 * cout * cin;
  const uint16_t* wh = (const uint16_t*)wsplit;
  hipStream_t st = (hipStream_t)stream;
  const long long big_blocks = (long long)(V / 128) * (cout / 128) * b;
  if (big_blocks >= 2 * kCUs) {
    hipLaunchKernelGGL((conv3_igemm_kernel<128, 128>), dim3(V / 128, cout / 128, b), dim3(256), 0,
                       st, x, wh, wh + total, bias, y, cin, cout, r);
  } else {
    hipLaunchKernelGGL((conv3_igemm_kernel<64, 64>), dim3(V / 64, cout / 64, b), dim3(256), 0, st,
                       x, wh, wh + total, bias, y, cin, cout, r);
  }
  return check_launch("conv3d_igemm");
}

extern "C" size_t pcfm_conv3d_wgrad_workspace_bytes(int b, int cin, int cout, int r) {
  if (b <= 0 || !conv3_shape_ok(b, cin, cout, r) || cin % kMT != 0) return 0;
  return (size_t)conv3_wgrad_splits(b, cin, cout, r) * 27 * cout * cin * sizeof(float);
}

extern "C" int pcfm_conv3d_wgrad(const float* x, const float* grad_y, int b, int cin, int cout,
                                 int r, float* grad_w, void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(b > 0 && conv3_shape_ok(b, cin, cout, r) && cin % kMT == 0,
                 "conv3d_wgrad: unsupported shape b=%d cin=%d cout=%d r=%d", b, cin, cout, r);
  const size_t need = pcfm_conv3d_wgrad_workspace_bytes(b, cin, cout, r);
  PCFM_CHECK_ARG(ws_bytes >= need, "conv3d_wgrad: workspace %zu < %zu bytes", ws_bytes, need);
  const int S = conv3_wgrad_splits(b, cin, cout, r);
  hipStream_t st = (hipStream_t)stream;
  const int tiles = 27 * (cout / kMT) * (cin / kMT);
  hipLaunchKernelGGL(conv3_wgrad_kernel, dim3(tiles * S), dim3(256), 0, st, x, grad_y, b, cin,
                     cout, r, S, (float*)ws);
  const size_t total = (size_t)27 * cout * cin;
  hipLaunchKernelGGL(conv3_wgrad_reduce_kernel, dim3(ceil_div((long long)total, 256)), dim3(256),
                     0, st, (const float*)ws, cout, cin, S, grad_w);
  return check_launch("conv3d_wgrad");
}
