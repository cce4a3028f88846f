// Ball query and grouping (include/pcfm.h).
//
// Reference semantics: third_party/pvcnn/modules/functional/src/ball_query/
// ball_query.cu:19-50 and src/grouping/grouping.cu:18-77.
#include "rows.hpp"
#include "segsum.hpp"

namespace pcfm {
namespace {

// One WAVE per center, 64 candidate points per step (lane = point): the hits
// of a step come out of one ballot, in index order, so the first u hits of the
// reference's sequential scan (ball_query.cu:33-47) are the first u set bits
// seen; the wave leaves as soon as it holds u.  The candidates stream through
// an LDS tile shared by the block's 16 waves (16 centers): each tile is read
// from global memory once per block instead of once per center, and a block
// stops loading tiles when all its centers are full (__syncthreads_count).
// Unfilled slots repeat the first hit (:40-45) or stay zero when there is none
// (the reference's torch::zeros output).  Distances: sqdist3 (dx = center -
// point), strict d2 < r2, as the oracle.
constexpr int kBQWaves = 16;      // centers per block
constexpr int kBQTile = 2048;     // candidate points per LDS tile (24 KiB)

__global__ void __launch_bounds__(kBQWaves * 64)
    ball_query_kernel(const float* __restrict__ centers, const float* __restrict__ points,
                      int m, int n, float r2, int u, int* __restrict__ out) {
  __shared__ float sx[kBQTile], sy[kBQTile], sz[kBQTile];
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = blockIdx.x * kBQWaves + w;
  const bool active = j < m;
  const float* cb = centers + (size_t)b * 3 * m;
  const float* __restrict__ pb = points + (size_t)b * 3 * n;
  const float cx = active ? cb[j] : 0.0f;
  const float cy = active ? cb[j + m] : 0.0f;
  const float cz = active ? cb[j + 2 * m] : 0.0f;
  int* o = out + ((size_t)b * m + (active ? j : 0)) * u;
  int cnt = 0, first = 0;
  bool open = active;
  for (int k0 = 0; k0 < n; k0 += kBQTile) {
    if (__syncthreads_count(open ? 1 : 0) == 0) break;  // every center of the block is full
    const int len = min(kBQTile, n - k0);
    for (int e = threadIdx.x; e < len; e += kBQWaves * 64) {
      sx[e] = pb[k0 + e];
      sy[e] = pb[(size_t)n + k0 + e];
      sz[e] = pb[(size_t)2 * n + k0 + e];
    }
    __syncthreads();
    for (int c0 = 0; open && c0 < len; c0 += 64) {
      const int e = c0 + lane;
      bool hit = false;
      if (e < len) {
        const float d2 = sqdist3(cx - sx[e], cy - sy[e], cz - sz[e]);
        hit = d2 < r2;
      }
      const unsigned long long bal = __ballot(hit);
      if (bal) {
        if (cnt == 0) first = k0 + c0 + __ffsll((long long)bal) - 1;
        const int pos = cnt + __popcll(bal & ((1ull << lane) - 1ull));
        if (hit && pos < u) o[pos] = k0 + e;
        cnt += __popcll(bal);
        open = cnt < u;
      }
    }
  }
  if (active) {
    const int fill = cnt > 0 ? first : 0;
    for (int v = min(cnt, u) + lane; v < u; v += 64) o[v] = fill;
  }
}

}  // namespace
}  // namespace pcfm

using namespace pcfm;

extern "C" int pcfm_ball_query(const float* centers, const float* points, int b, int m, int n,
                               float radius, int u, int* idx, void* stream) {
  PCFM_CHECK_ARG(b >= 0 && m >= 0 && n >= 0 && u >= 0, "ball_query: negative size");
  if (b == 0 || m == 0 || u == 0) return PCFM_OK;
  const float r2 = radius * radius;  // host float product, as ball_query.cpp:25
  dim3 grid(ceil_div(m, kBQWaves), b);
  hipLaunchKernelGGL(ball_query_kernel, grid, dim3(kBQWaves * 64), 0, (hipStream_t)stream, centers,
                     points, m, n, r2, u, idx);
  return check_launch("ball_query");
}

extern "C" int pcfm_grouping_fwd(const float* feat, const int* idx, int b, int c, int n, int m,
                                 int u, float* out, void* stream) {
  PCFM_CHECK_ARG(b >= 0 && c >= 0 && n >= 0 && m >= 0 && u >= 0, "grouping_fwd: negative size");
  const long long mu = (long long)m * u;
  PCFM_CHECK_ARG(mu < (1LL << 31), "grouping_fwd: m*u too large");
  if (c == 0) return PCFM_OK;
  return launch_gather(feat, out, b, c, n, (int)mu, ProvIdx1{idx, nullptr, (int)mu, n},
                       (hipStream_t)stream, "grouping_fwd");
}

extern "C" size_t pcfm_grouping_bwd_workspace_bytes(int b, int c, int n, int m, int u) {
  if (b < 0 || c < 0 || n < 0 || m < 0 || u < 0) return 0;
  const long long mu = (long long)m * u;
  if (mu >= (1LL << 31)) return 0;
  return seg_ws_bytes(b, c, (int)mu, n, 1);
}

extern "C" int pcfm_grouping_bwd(const float* grad_y, const int* idx, int b, int c, int n, int m,
                                 int u, float* grad_x, void* ws, size_t ws_bytes, void* stream) {
  PCFM_CHECK_ARG(b >= 0 && c >= 0 && n >= 0 && m >= 0 && u >= 0, "grouping_bwd: negative size");
  const long long mu = (long long)m * u;
  PCFM_CHECK_ARG(mu < (1LL << 31), "grouping_bwd: m*u too large");
  const size_t need = pcfm_grouping_bwd_workspace_bytes(b, c, n, m, u);
  PCFM_CHECK_ARG(ws_bytes >= need, "grouping_bwd: workspace %zu < %zu bytes", ws_bytes, need);
  // grad_x[c, i] = sum of grad_y over the (center, slot) pairs whose index is i
  return seg_scatter<1>(grad_y, idx, mu, false, nullptr, 0, b, c, (int)mu, n, nullptr, grad_x,
                        ws, (hipStream_t)stream, "grouping_bwd");
}
