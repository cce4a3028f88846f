// Chamfer-3D nearest neighbours, forward and backward (include/pcfm.h).
//
// Reference: third_party/ChamferDistancePytorch/chamfer3D/chamfer3D.cu:12-195.
// The reference runs a <<<(32,16),512>>> grid per direction in which only
// B*16 blocks work, with 512-point LDS tiles read by every thread.  Here:
//   * both directions are one launch (grid.z = 2*B);
//   * each lane owns Q = 8 query points in registers, paired into packed-fp32
//     operands; the candidate loop is wave-uniform, so candidates arrive
//     through scalar loads and every VALU op reads them straight from SGPRs
//     (no LDS, no per-lane address math);
//   * when B*N queries alone cannot fill 256 CUs the candidate range is split
//     and the per-split winners merge through a 64-bit atomicMin on
//     (float bits of d) << 32 | index.  d >= 0, so the packed order is exactly
//     "smaller distance, then lower index" -- the reference's tie rule (strict
//     `<` inside a tile, chamfer3D.cu:36-68, strict `>` across tiles, :126) --
//     and the result does not depend on arrival order.
#include "pcfm_common.hpp"

#include <algorithm>

namespace pcfm {
namespace {

constexpr int kQ = 8;          // queries per lane (4 packed pairs)
constexpr int kThreads = 256;  // 4 waves
constexpr int kPerBlock = kQ * kThreads;

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned long long pack_key(float d, int idx) {
  return ((unsigned long long)__float_as_uint(d) << 32) | (unsigned)idx;
}

// grid = (query blocks, splits, 2*b).  Two queries share each packed-fp32
// instruction (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32): the distance costs
// 6 packed ops per 2 pairs, the same per-component fma chain as sqdist3 (so
// the same bits as the oracle), leaving the compare / select per pair.
__global__ void __launch_bounds__(kThreads)
    nn_kernel(const float* __restrict__ xyz1, const float* __restrict__ xyz2, int b, int n, int m,
              int splits, float* __restrict__ dist1, int* __restrict__ idx1,
              float* __restrict__ dist2, int* __restrict__ idx2,
              unsigned long long* __restrict__ key1, unsigned long long* __restrict__ key2) {
  const int dir = blockIdx.z >= (unsigned)b;
  const int bb = blockIdx.z - dir * b;
  const float* __restrict__ qp = dir ? xyz2 : xyz1;
  const float* __restrict__ cp = dir ? xyz1 : xyz2;
  const int nq = dir ? m : n;
  const int nc = dir ? n : m;
  const int qbase = blockIdx.x * kPerBlock;
  if (qbase >= nq) return;
  const int s = blockIdx.y;
  const int k0 = (int)(((long long)nc * s) / splits);
  const int k1 = (int)(((long long)nc * (s + 1)) / splits);

  constexpr int kP = kQ / 2;
  f2 qx[kP], qy[kP], qz[kP];
  float best[kQ];
  int bi[kQ];
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    const int j = qbase + q * kThreads + threadIdx.x;
    const int jj = j < nq ? j : nq - 1;
    const float* p = qp + ((size_t)bb * nq + jj) * 3;
    qx[q >> 1][q & 1] = p[0];
    qy[q >> 1][q & 1] = p[1];
    qz[q >> 1][q & 1] = p[2];
    best[q] = __builtin_inff();
    bi[q] = k0;
  }
  const float* __restrict__ cb = cp + (size_t)bb * nc * 3;
  // one candidate: the same fma chain as sqdist3 on two queries at once
  auto visit = [&](float x, float y, float z, int k) {
    const f2 cx = x, cy = y, cz = z;
#pragma unroll
    for (int p = 0; p < kP; ++p) {
      // dx = candidate - query (chamfer3D.cu:32-35); fma(dz, dz, fma(dx, dx, dy * dy))
      const f2 dx = cx - qx[p], dy = cy - qy[p], dz = cz - qz[p];
      const f2 d = __builtin_elementwise_fma(dz, dz, __builtin_elementwise_fma(dx, dx, dy * dy));
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (d[h] < best[2 * p + h]) {
          best[2 * p + h] = d[h];
          bi[2 * p + h] = k;
        }
      }
    }
  };
  // groups of kG candidates through wide scalar loads (uniform address), the
  // next group's loads issued before the current group's arithmetic
  constexpr int kG = 8;
  const int kg1 = k0 + (k1 - k0) / kG * kG;
  int k = __builtin_amdgcn_readfirstlane(k0);
  if (k < kg1) {
    float c[3 * kG], nx[3 * kG];
#pragma unroll
    for (int e = 0; e < 3 * kG; ++e) c[e] = cb[3 * k + e];
    for (; k < kg1; k += kG) {
      const int kn = k + kG < kg1 ? k + kG : k;
#pragma unroll
      for (int e = 0; e < 3 * kG; ++e) nx[e] = cb[3 * kn + e];
#pragma unroll
      for (int g = 0; g < kG; ++g) visit(c[3 * g], c[3 * g + 1], c[3 * g + 2], k + g);
#pragma unroll
      for (int e = 0; e < 3 * kG; ++e) c[e] = nx[e];
    }
  }
  for (; k < k1; ++k) visit(cb[3 * k], cb[3 * k + 1], cb[3 * k + 2], k);
  float* __restrict__ dist = dir ? dist2 : dist1;
  int* __restrict__ idx = dir ? idx2 : idx1;
  unsigned long long* __restrict__ key = dir ? key2 : key1;
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    const int j = qbase + q * kThreads + threadIdx.x;
    if (j >= nq) continue;
    const size_t o = (size_t)bb * nq + j;
    if (splits == 1) {
      dist[o] = best[q];
      idx[o] = bi[q];
    } else {
      atomicMin(key + o, pack_key(best[q], bi[q]));
    }
  }
}

__global__ void key_init_kernel(unsigned long long* __restrict__ key, size_t total) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < total) key[i] = ~0ULL;
}

__global__ void key_unpack_kernel(const unsigned long long* __restrict__ key, size_t total,
                                  float* __restrict__ dist, int* __restrict__ idx) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < total) {
    const unsigned long long k = key[i];
    dist[i] = __uint_as_float((unsigned)(k >> 32));
    idx[i] = (int)(unsigned)(k & 0xffffffffu);
  }
}

// Backward: g = 2*grad_dist; own point += g*(a - b_nn), neighbour -= the same
// term (chamfer3D.cu:155-174).  Both directions in one launch, so both sides
// use float atomics, as the reference does.
__global__ void __launch_bounds__(256)
    nn_grad_kernel(const float* __restrict__ xyz1, const float* __restrict__ xyz2, int b, int n,
                   int m, const float* __restrict__ gd1, const float* __restrict__ gd2,
                   const int* __restrict__ idx1, const int* __restrict__ idx2,
                   float* __restrict__ g1, float* __restrict__ g2) {
  const int dir = blockIdx.y >= (unsigned)b;
  const int bb = blockIdx.y - dir * b;
  const int nq = dir ? m : n;
  const int nc = dir ? n : m;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nq) return;
  const float* __restrict__ qp = dir ? xyz2 : xyz1;
  const float* __restrict__ cp = dir ? xyz1 : xyz2;
  const float* __restrict__ gd = dir ? gd2 : gd1;
  const int* __restrict__ ix = dir ? idx2 : idx1;
  float* gq = dir ? g2 : g1;
  float* gc = dir ? g1 : g2;
  const size_t o = (size_t)bb * nq + j;
  const int j2 = ix[o];
  if ((unsigned)j2 >= (unsigned)nc) return;
  const float* a = qp + o * 3;
  const float* c = cp + ((size_t)bb * nc + j2) * 3;
  const float g = gd[o] * 2.0f;
  const float tx = g * (a[0] - c[0]);
  const float ty = g * (a[1] - c[1]);
  const float tz = g * (a[2] - c[2]);
  float* ga = gq + o * 3;
  float* gb = gc + ((size_t)bb * nc + j2) * 3;
  atomicAdd(ga + 0, tx);
  atomicAdd(ga + 1, ty);
  atomicAdd(ga + 2, tz);
  atomicAdd(gb + 0, -tx);
  atomicAdd(gb + 1, -ty);
  atomicAdd(gb + 2, -tz);
}

// Candidate splits so that the launch has >= ~4 waves per SIMD.
int choose_splits(int b, int n, int m) {
  const long long qblocks = (long long)b * (ceil_div(n, kPerBlock) + ceil_div(m, kPerBlock));
  const long long want_blocks = 4LL * kCUs * 4;  // 4 blocks of 4 waves per CU, x4 slack
  int s = (int)std::max(1LL, (want_blocks + qblocks - 1) / std::max(1LL, qblocks));
  const int cmin = std::max(1, std::min(n, m));
  s = std::min(s, std::max(1, cmin / 256));  // >= 256 candidates per split
  return std::min(s, 64);
}

}  // namespace
}  // namespace pcfm

using namespace pcfm;

extern "C" size_t pcfm_chamfer_workspace_bytes(int b, int n, int m) {
  if (b <= 0 || n < 0 || m < 0) return 0;
  if (choose_splits(b, n, m) == 1) return 0;
  return (size_t)b * ((size_t)n + m) * sizeof(unsigned long long);
}

extern "C" int pcfm_chamfer_fwd(const float* xyz1, const float* xyz2, int b, int n, int m,
                                float* dist1, float* dist2, int* idx1, int* idx2, void* ws,
                                size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(b >= 0 && n >= 0 && m >= 0, "chamfer_fwd: negative size");
  PCFM_CHECK_ARG(ws_bytes >= pcfm_chamfer_workspace_bytes(b, n, m),
                 "chamfer_fwd: workspace %zu < %zu bytes", ws_bytes,
                 pcfm_chamfer_workspace_bytes(b, n, m));
  if (b == 0) return PCFM_OK;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0 || m == 0) {
    // The reference leaves its zero-initialised outputs untouched.
    hipError_t e = hipSuccess;
    if (n) e = hipMemsetAsync(dist1, 0, (size_t)b * n * 4, st);
    if (n && e == hipSuccess) e = hipMemsetAsync(idx1, 0, (size_t)b * n * 4, st);
    if (m && e == hipSuccess) e = hipMemsetAsync(dist2, 0, (size_t)b * m * 4, st);
    if (m && e == hipSuccess) e = hipMemsetAsync(idx2, 0, (size_t)b * m * 4, st);
    if (e != hipSuccess) {
      set_error("chamfer_fwd: hipMemsetAsync: %s", hipGetErrorString(e));
      return (int)e;
    }
    return PCFM_OK;
  }
  const int splits = choose_splits(b, n, m);
  unsigned long long* key1 = nullptr;
  unsigned long long* key2 = nullptr;
  if (splits > 1) {
    key1 = (unsigned long long*)ws;
    key2 = key1 + (size_t)b * n;
    const size_t total = (size_t)b * ((size_t)n + m);
    hipLaunchKernelGGL(key_init_kernel, dim3(ceil_div((long long)total, 256)), dim3(256), 0, st,
                       key1, total);
  }
  dim3 grid(ceil_div(std::max(n, m), kPerBlock), splits, 2 * b);
  hipLaunchKernelGGL(nn_kernel, grid, dim3(kThreads), 0, st, xyz1, xyz2, b, n, m, splits, dist1,
                     idx1, dist2, idx2, key1, key2);
  if (splits > 1) {
    const size_t t1 = (size_t)b * n, t2 = (size_t)b * m;
    hipLaunchKernelGGL(key_unpack_kernel, dim3(ceil_div((long long)t1, 256)), dim3(256), 0, st,
                       key1, t1, dist1, idx1);
    hipLaunchKernelGGL(key_unpack_kernel, dim3(ceil_div((long long)t2, 256)), dim3(256), 0, st,
                       key2, t2, dist2, idx2);
  }
  return check_launch("chamfer_fwd");
}

extern "C" int pcfm_chamfer_bwd(const float* xyz1, const float* xyz2, int b, int n, int m,
                                const float* grad_dist1, const float* grad_dist2, const int* idx1,
                                const int* idx2, float* grad_xyz1, float* grad_xyz2,
                                void* stream) {
  PCFM_CHECK_ARG(b >= 0 && n >= 0 && m >= 0, "chamfer_bwd: negative size");
  if (b == 0 || n == 0 || m == 0) return PCFM_OK;
  dim3 grid(ceil_div(std::max(n, m), 256), 2 * b);
  hipLaunchKernelGGL(nn_grad_kernel, grid, dim3(256), 0, (hipStream_t)stream, xyz1, xyz2, b, n,
                     m, grad_dist1, grad_dist2, idx1, idx2, grad_xyz1, grad_xyz2);
  return check_launch("chamfer_bwd");
}
