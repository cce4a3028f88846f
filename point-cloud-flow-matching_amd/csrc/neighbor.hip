// Ball query and grouping (include/pcfm.h).
//
// Reference semantics: third_party/pvcnn/modules/functional/src/ball_query/
// ball_query.cu:19-50 and src/grouping/grouping.cu:18-77.
#include "rows.hpp"
#include "segsum.hpp"

namespace pcfm {
namespace {

// One lane per center; the point scan is wave-uniform (the same point k for
// all 64 lanes), so the three coordinates come in through scalar loads and the
// wave leaves the scan as soon as every lane holds u hits.  Hits are written
// in index order; unfilled slots repeat the first hit (ball_query.cu:40-45) or
// stay zero when there is none (the reference's torch::zeros output).
__global__ void __launch_bounds__(256)
    ball_query_kernel(const float* __restrict__ centers, const float* __restrict__ points,
                      int m, int n, float r2, int u, int* __restrict__ out) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = j < m;
  const float* cb = centers + (size_t)b * 3 * m;
  const float* __restrict__ pb = points + (size_t)b * 3 * n;
  const float cx = active ? cb[j] : 0.0f;
  const float cy = active ? cb[j + m] : 0.0f;
  const float cz = active ? cb[j + 2 * m] : 0.0f;
  int* o = out + ((size_t)b * m + (active ? j : 0)) * u;
  int cnt = 0, first = 0;
  bool open = active && u > 0;
  for (int k0 = 0; k0 < n; k0 += 64) {
    if (!__any(open)) break;
    const int kend = min(n, k0 + 64);
    for (int k = k0; k < kend; ++k) {
      const float dx = cx - pb[k];
      const float dy = cy - pb[k + n];
      const float dz = cz - pb[k + 2 * n];
      const float d2 = sqdist3(dx, dy, dz);
      if (open && d2 < r2) {
        if (cnt == 0) first = k;
        o[cnt] = k;
        ++cnt;
        open = cnt < u;
      }
    }
  }
  if (active) {
    const int fill = cnt > 0 ? first : 0;
    for (int v = cnt; v < u; ++v) o[v] = fill;
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
  dim3 grid(ceil_div(m, 256), b);
  hipLaunchKernelGGL(ball_query_kernel, grid, dim3(256), 0, (hipStream_t)stream, centers, points,
                     m, n, r2, u, idx);
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
