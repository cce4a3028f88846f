// PVConv voxel path: average voxelization and trilinear devoxelization,
// forward and backward (include/pcfm.h).
//
// Reference semantics: third_party/pvcnn/modules/functional/src/voxelization/
// vox.cu:18-126 and src/interpolate/trilinear_devox.cu:21-162.
#include "rows.hpp"
#include "segsum.hpp"

namespace pcfm {
namespace {

// ind[b, i] = x*r^2 + y*r + z (vox.cu:31); the histogram is built by the sort.
__global__ void __launch_bounds__(256)
    vox_ind_kernel(const int* __restrict__ coords, int n, int r, int* __restrict__ ind) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int* cb = coords + (size_t)b * 3 * n;
  ind[(size_t)b * n + i] = cb[i] * r * r + cb[i + n] * r + cb[i + 2 * n];
}

bool cube_fits(int r, int* s) {
  if (r < 1) return false;
  const long long c = (long long)r * r * r;
  if (c > (1LL << 30)) return false;
  *s = (int)c;
  return true;
}

// out[r] = scale * sum_v a[r][v] * (b ? b[r][v] : 1): one block per row,
// fixed per-thread order + tree, deterministic.  Accumulated in fp64 (the
// products of two floats are exact in fp64): SE3d's channel mean and its scale
// gradient sum_v grid * g cancel heavily, and an fp32 sum over R^3 voxels
// would carry its rounding times that cancellation into the SE weights'
// gradients.  The row is read once either way (HBM-bound, the fp64 adds are
// free beside the loads).
__global__ void __launch_bounds__(256)
    rows_dot_kernel(const float* __restrict__ a, const float* __restrict__ b, int len, float scale,
                    float* __restrict__ out) {
  const size_t r = blockIdx.x;
  const float* ar = a + r * len;
  const float* br = b != nullptr ? b + r * len : nullptr;
  double acc = 0.0;
  if ((len & 3) == 0) {
    const float4* a4 = reinterpret_cast<const float4*>(ar);
    const float4* b4 = reinterpret_cast<const float4*>(br);
    for (int v = threadIdx.x; v < (len >> 2); v += 256) {
      const float4 x = a4[v];
      if (br != nullptr) {
        const float4 y = b4[v];
        acc = __builtin_fma((double)x.x, (double)y.x, acc);
        acc = __builtin_fma((double)x.y, (double)y.y, acc);
        acc = __builtin_fma((double)x.z, (double)y.z, acc);
        acc = __builtin_fma((double)x.w, (double)y.w, acc);
      } else {
        acc += ((double)x.x + (double)x.y) + ((double)x.z + (double)x.w);
      }
    }
  } else {
    for (int v = threadIdx.x; v < len; v += 256)
      acc = br != nullptr ? __builtin_fma((double)ar[v], (double)br[v], acc) : acc + (double)ar[v];
  }
  __shared__ double red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[r] = (float)(red[0] * (double)scale);
}

// x[r][v] = s[r] * x[r][v] + t[r]  (in place; t may be null).  Runs after
// rows_dot over the same rows (SE3d's backward): blocks in reverse order.
__global__ void __launch_bounds__(256)
    rows_affine_kernel(float* __restrict__ x, const float* __restrict__ s,
                       const float* __restrict__ t, int len4, int per_row_blocks) {
  const unsigned blk = rev_order(blockIdx.x, gridDim.x);
  const size_t r = blk / per_row_blocks;
  const int v = (blk % per_row_blocks) * 256 + threadIdx.x;
  if (v >= len4) return;
  const float sv = s[r], tv = t != nullptr ? t[r] : 0.0f;
  float4* x4 = reinterpret_cast<float4*>(x) + r * len4;
  float4 q = x4[v];
  q.x = __builtin_fmaf(sv, q.x, tv);
  q.y = __builtin_fmaf(sv, q.y, tv);
  q.z = __builtin_fmaf(sv, q.z, tv);
  q.w = __builtin_fmaf(sv, q.w, tv);
  x4[v] = q;
}

// Diagnosis: recompute scale * devox(feat) + add for every (b, c, i) in the
// plainest form (one thread per output, global reads, no LDS, no batching) and
// compare bit for bit with what the gather stored; training mode also checks
// the stored inds / wgts.  rec[0] counts mismatches, rec[1] counts points whose
// stored weights do not sum to 1 within 1e-5; rec[2 + 8k ..] holds up to 16
// records {kind, b, c, i, got bits, want bits, lane, i / 64}.
constexpr int kVerifyRecs = 16;
// bn / abn (mean != nullptr): the grid rows / the add operand enter as
// act(bn(.)) (pcfm_trilinear_devoxelize_bn_scale_add_fwd's RowBn transforms)
__global__ void __launch_bounds__(256)
    devox_verify_kernel(const float* __restrict__ coords, const float* __restrict__ feat,
                        const float* __restrict__ scale, const float* __restrict__ add,
                        const float* __restrict__ out, const int* __restrict__ inds,
                        const float* __restrict__ wgts, int C, int n, int r, int* __restrict__ rec,
                        RowBn bn = {}, RowBn abn = {}) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (t >= (long long)C * n) return;
  const int c = (int)(t / n), i = (int)(t % n);
  const int s = r * r * r;
  ProvDevox prov{coords, n, r, r * r, s, nullptr, nullptr};
  int id[8];
  float w[8];
  prov.get(b, i, false, id, w);
  const float* row = feat + ((size_t)b * C + c) * s;
  float a;
  if (bn.mean != nullptr) {  // tap_sum's order on the transformed values
    const RowBnC tc = row_bn_at(bn, c);
    a = w[1] * tc(row[id[1]]);
    a = __builtin_fmaf(w[0], tc(row[id[0]]), a);
    for (int k = 2; k < 8; ++k) a = __builtin_fmaf(w[k], tc(row[id[k]]), a);
  } else {
    a = tap_sum<8>(row, id, w);
  }
  if (scale != nullptr) a *= scale[(size_t)b * C + c];
  if (add != nullptr) {
    const float av = add[((size_t)b * C + c) * n + i];
    a += abn.mean != nullptr ? row_bn_at(abn, c)(av) : av;
  }
  const float got = out[((size_t)b * C + c) * n + i];
  auto note = [&](int kind, float gv, float wv) {
    const int k = atomicAdd(rec, 1);
    if (k < kVerifyRecs) {
      int* e = rec + 2 + 8 * k;
      e[0] = kind; e[1] = b; e[2] = c; e[3] = i;
      e[4] = __float_as_int(gv); e[5] = __float_as_int(wv); e[6] = i & 63; e[7] = i >> 6;
    }
  };
  if (__float_as_int(got) != __float_as_int(a)) note(0, got, a);
  if (c == 0 && inds != nullptr) {
    // the stored pairs are the unclamped ones (trilinear_devox.cu:64-75): compare
    // where the recomputed corner is inside the volume with a non-zero weight
    float sum = 0.0f;
    for (int k = 0; k < 8; ++k) {
      const size_t o = ((size_t)b * 8 + k) * n + i;
      sum += wgts[o];
      if ((unsigned)inds[o] < (unsigned)s && inds[o] != id[k] && w[k] != 0.0f)
        note(1, __int_as_float(inds[o]), __int_as_float(id[k]));
      if ((unsigned)id[k] < (unsigned)s && w[k] != 0.0f &&
          __float_as_int(wgts[o]) != __float_as_int(w[k]))
        note(2, wgts[o], w[k]);
    }
    if (fabsf(sum - 1.0f) > 1e-5f) atomicAdd(rec + 1, 1);
  }
}

}  // namespace
}  // namespace pcfm

using namespace pcfm;

extern "C" int pcfm_debug_devox_verify(const float* coords, const float* feat, const float* scale,
                                       const float* add, const float* out, const int* inds,
                                       const float* wgts, int b, int c, int n, int r, int* rec,
                                       void* stream) {
  int s = 0;
  PCFM_CHECK_ARG(b >= 0 && c >= 0 && n >= 0 && cube_fits(r, &s) && rec != nullptr,
                 "debug_devox_verify: bad arguments");
  if ((long long)b * c * n == 0) return PCFM_OK;
  hipLaunchKernelGGL(devox_verify_kernel, dim3(ceil_div((long long)c * n, 256), b), dim3(256), 0,
                     (hipStream_t)stream, coords, feat, scale, add, out, inds, wgts, c, n, r, rec);
  return check_launch("debug_devox_verify");
}

extern "C" int pcfm_debug_devox_verify_bn(const float* coords, const float* feat,
                                          const float* bn_mean, const float* bn_invstd,
                                          const float* bn_gamma, const float* bn_beta,
                                          float slope, const float* scale, const float* add,
                                          const float* add_mean, const float* add_invstd,
                                          const float* add_gamma, const float* add_beta,
                                          float add_slope, const float* out, const int* inds,
                                          const float* wgts, int b, int c, int n, int r, int* rec,
                                          void* stream) {
  int s = 0;
  PCFM_CHECK_ARG(b >= 0 && c >= 0 && n >= 0 && cube_fits(r, &s) && rec != nullptr &&
                     bn_mean != nullptr && bn_invstd != nullptr && bn_gamma != nullptr &&
                     bn_beta != nullptr,
                 "debug_devox_verify_bn: bad arguments");
  PCFM_CHECK_ARG(add_mean == nullptr || (add != nullptr && add_invstd != nullptr &&
                                         add_gamma != nullptr && add_beta != nullptr),
                 "debug_devox_verify_bn: incomplete BatchNorm operands of add");
  if ((long long)b * c * n == 0) return PCFM_OK;
  const RowBn bn{bn_mean, bn_invstd, bn_gamma, bn_beta, slope};
  const RowBn abn{add_mean, add_invstd, add_gamma, add_beta, add_slope};
  hipLaunchKernelGGL(devox_verify_kernel, dim3(ceil_div((long long)c * n, 256), b), dim3(256), 0,
                     (hipStream_t)stream, coords, feat, scale, add, out, inds, wgts, c, n, r, rec,
                     bn, abn);
  return check_launch("debug_devox_verify_bn");
}

extern "C" size_t pcfm_avg_voxelize_fwd_workspace_bytes(int b, int c, int n, int r) {
  int s = 0;
  if (b < 0 || c < 0 || n < 0 || !cube_fits(r, &s)) return 0;
  return seg_ws_bytes(b, c, n, s, 1);
}

extern "C" int pcfm_avg_voxelize_fwd(const float* feat, const int* coords, int b, int c, int n,
                                     int r, float* out, int* ind, int* cnt, void* ws,
                                     size_t ws_bytes, void* stream) {
  int s = 0;
  PCFM_CHECK_ARG(b >= 0 && c >= 0 && n >= 0, "avg_voxelize_fwd: negative size b=%d c=%d n=%d",
                 b, c, n);
  PCFM_CHECK_ARG(cube_fits(r, &s), "avg_voxelize_fwd: bad resolution %d", r);
  const size_t need = pcfm_avg_voxelize_fwd_workspace_bytes(b, c, n, r);
  PCFM_CHECK_ARG(ws_bytes >= need, "avg_voxelize_fwd: workspace %zu < %zu bytes", ws_bytes, need);
  if (b == 0) return PCFM_OK;
  hipStream_t st = (hipStream_t)stream;
  if (n > 0)
    hipLaunchKernelGGL(vox_ind_kernel, dim3(ceil_div(n, 256), b), dim3(256), 0, st, coords, n, r,
                       ind);
  // cnt = histogram of ind; out[c, v] = sum_{i in voxel v} feat[c, i] * (1/cnt[v])
  // (per-term product, vox.cu:68)
  return seg_scatter<1>(feat, ind, n, true, nullptr, r, b, c, n, s, cnt, out, ws, st,
                        "avg_voxelize_fwd");
}

extern "C" int pcfm_avg_voxelize_bwd(const float* grad_y, const int* ind, const int* cnt, int b,
                                     int c, int n, int s, float* grad_x, void* stream) {
  PCFM_CHECK_ARG(b >= 0 && c >= 0 && n >= 0 && s >= 0,
                 "avg_voxelize_bwd: negative size b=%d c=%d n=%d s=%d", b, c, n, s);
  if (c == 0) return PCFM_OK;
  return launch_gather(grad_y, grad_x, b, c, s, n, ProvVoxBwd{ind, cnt, n, s},
                       (hipStream_t)stream, "avg_voxelize_bwd");
}

// grad_x = avg_voxelize_bwd(grad_y) + add: the voxelization's input gradient
// summed with the point branch's (PVConv feeds features to both) in the gather
extern "C" int pcfm_avg_voxelize_bwd_add(const float* grad_y, const int* ind, const int* cnt,
                                         const float* add, int b, int c, int n, int s,
                                         float* grad_x, void* stream) {
  PCFM_CHECK_ARG(b >= 0 && c >= 0 && n >= 0 && s > 0,
                 "avg_voxelize_bwd_add: bad size b=%d c=%d n=%d s=%d", b, c, n, s);
  if (c == 0) return PCFM_OK;
  GatherEpi epi;
  epi.add = add;
  return launch_gather(grad_y, grad_x, b, c, s, n, ProvVoxBwd{ind, cnt, n, s},
                       (hipStream_t)stream, "avg_voxelize_bwd_add", epi);
}

extern "C" int pcfm_trilinear_devoxelize_fwd(const float* coords, const float* feat, int b, int c,
                                             int n, int r, int training, float* out, int* inds,
                                             float* wgts, void* stream) {
  int s = 0;
  PCFM_CHECK_ARG(b >= 0 && c >= 0 && n >= 0, "trilinear_devoxelize_fwd: negative size");
  PCFM_CHECK_ARG(cube_fits(r, &s), "trilinear_devoxelize_fwd: bad resolution %d", r);
  PCFM_CHECK_ARG(!training || (long long)b * n == 0 || (inds != nullptr && wgts != nullptr),
                 "trilinear_devoxelize_fwd: training needs inds/wgts buffers");
  ProvDevox prov{coords, n, r, r * r, s, training ? inds : nullptr, training ? wgts : nullptr};
  return launch_gather(feat, out, b, c, s, n, prov, (hipStream_t)stream,
                       "trilinear_devoxelize_fwd");
}

extern "C" size_t pcfm_trilinear_devoxelize_bwd_workspace_bytes(int b, int c, int n, int r) {
  int s = 0;
  if (b < 0 || c < 0 || n < 0 || !cube_fits(r, &s)) return 0;
  return seg_ws_bytes(b, c, n, s, 8);
}

extern "C" int pcfm_trilinear_devoxelize_bwd(const float* grad_y, const int* inds,
                                             const float* wgts, int b, int c, int n, int r,
                                             float* grad_x, void* ws, size_t ws_bytes,
                                             void* stream) {
  int s = 0;
  PCFM_CHECK_ARG(b >= 0 && c >= 0 && n >= 0, "trilinear_devoxelize_bwd: negative size");
  PCFM_CHECK_ARG(cube_fits(r, &s), "trilinear_devoxelize_bwd: bad resolution %d", r);
  const size_t need = pcfm_trilinear_devoxelize_bwd_workspace_bytes(b, c, n, r);
  PCFM_CHECK_ARG(ws_bytes >= need, "trilinear_devoxelize_bwd: workspace %zu < %zu bytes",
                 ws_bytes, need);
  // Points grouped by their base cell inds[b, 0, i]; corner k of a point in
  // cell q lands on q + (dx r^2 + dy r + dz).  When a fraction is 0 the
  // reference folds that corner onto the low cell with weight exactly 0
  // (trilinear_devox.cu:64-75), so both placements add the same zeros.
  return seg_scatter<8>(grad_y, inds, 8LL * n, false, wgts, r, b, c, n, s, nullptr, grad_x, ws,
                        (hipStream_t)stream, "trilinear_devoxelize_bwd");
}

// ---------------------------------------------------------------------------
// SE3d folded into the devoxelization (modules/se.py over pvconv.py:35-39):
// devox(grid * s) + point branch == s * devox(grid) + point branch, so the
// scaled grid is never written.  Backward: g = devox_bwd(dout) then
// d grid = s * g + d mean / V (rows_affine) and d s = sum_v grid * g (rows_dot).
// ---------------------------------------------------------------------------
extern "C" int pcfm_trilinear_devoxelize_scale_add_fwd(const float* coords, const float* feat,
                                                       const float* scale, const float* add,
                                                       int b, int c, int n, int r, int training,
                                                       float* out, int* inds, float* wgts,
                                                       void* stream) {
  int s = 0;
  PCFM_CHECK_ARG(b >= 0 && c >= 0 && n >= 0, "trilinear_devoxelize_scale_add_fwd: negative size");
  PCFM_CHECK_ARG(cube_fits(r, &s), "trilinear_devoxelize_scale_add_fwd: bad resolution %d", r);
  PCFM_CHECK_ARG(!training || (long long)b * n == 0 || (inds != nullptr && wgts != nullptr),
                 "trilinear_devoxelize_scale_add_fwd: training needs inds/wgts buffers");
  ProvDevox prov{coords, n, r, r * r, s, training ? inds : nullptr, training ? wgts : nullptr};
  GatherEpi epi;
  epi.scale = scale;
  epi.add = add;
  return launch_gather(feat, out, b, c, s, n, prov, (hipStream_t)stream,
                       "trilinear_devoxelize_scale_add_fwd", epi);
}

// scale[b, c] * devox(act(bn(x)))[b, c, i] + add'[b, c, i]: PVConv's second
// BatchNorm3d + LeakyReLU applied to the conv output x as the gather stages its
// rows (rows.hpp RowBn), so the activation is never written (norm.hip,
// pcfm_bn_act_fwd_rowmean); add' = add, or act(bn(add)) with its own BatchNorm
// operands (the point branch's BatchNorm1d + ReLU, SharedMLP's activation
// never written either).
extern "C" int pcfm_trilinear_devoxelize_bn_scale_add_fwd(
    const float* coords, const float* x, const float* bn_mean, const float* bn_invstd,
    const float* gamma, const float* beta, float slope, const float* scale, const float* add,
    const float* add_mean, const float* add_invstd, const float* add_gamma,
    const float* add_beta, float add_slope, int b, int c, int n, int r, int training, float* out,
    int* inds, float* wgts, void* stream) {
  int s = 0;
  PCFM_CHECK_ARG(b >= 0 && c >= 0 && n >= 0, "trilinear_devoxelize_bn_scale_add_fwd: negative size");
  PCFM_CHECK_ARG(cube_fits(r, &s), "trilinear_devoxelize_bn_scale_add_fwd: bad resolution %d", r);
  PCFM_CHECK_ARG(bn_mean != nullptr && bn_invstd != nullptr && gamma != nullptr && beta != nullptr,
                 "trilinear_devoxelize_bn_scale_add_fwd: BatchNorm operands missing");
  PCFM_CHECK_ARG(!training || (long long)b * n == 0 || (inds != nullptr && wgts != nullptr),
                 "trilinear_devoxelize_bn_scale_add_fwd: training needs inds/wgts buffers");
  PCFM_CHECK_ARG(s <= 32 * 1024, "trilinear_devoxelize_bn_scale_add_fwd: r^3 = %d > 32768", s);
  ProvDevox prov{coords, n, r, r * r, s, training ? inds : nullptr, training ? wgts : nullptr};
  PCFM_CHECK_ARG(add_mean == nullptr ||
                     (add != nullptr && add_invstd != nullptr && add_gamma != nullptr &&
                      add_beta != nullptr),
                 "trilinear_devoxelize_bn_scale_add_fwd: incomplete BatchNorm operands of add");
  GatherEpi epi;
  epi.scale = scale;
  epi.add = add;
  epi.add_mean = add_mean;
  epi.add_invstd = add_invstd;
  epi.add_gamma = add_gamma;
  epi.add_beta = add_beta;
  epi.add_slope = add_slope;
  RowBn bn;
  bn.mean = bn_mean;
  bn.invstd = bn_invstd;
  bn.gamma = gamma;
  bn.beta = beta;
  bn.slope = slope;
  return launch_gather(x, out, b, c, s, n, prov, (hipStream_t)stream,
                       "trilinear_devoxelize_bn_scale_add_fwd", epi, bn);
}

// ---------------------------------------------------------------------------
// Segment plans (include/pcfm.h): the scatter's sort + work units built once
// and applied to every feature tensor over the same points.
// ---------------------------------------------------------------------------
static bool plan_taps_ok(int taps) { return taps == 1 || taps == 8; }

extern "C" size_t pcfm_seg_plan_bytes(int b, int n, int r, int taps) {
  int s = 0;
  if (b < 0 || n < 0 || !cube_fits(r, &s) || !plan_taps_ok(taps)) return 0;
  return seg_plan_bytes(b, n, s, taps);
}

extern "C" size_t pcfm_seg_apply_workspace_bytes(int b, int c, int n, int r, int taps) {
  int s = 0;
  if (b < 0 || c < 0 || n < 0 || !cube_fits(r, &s) || !plan_taps_ok(taps)) return 0;
  return seg_apply_bytes(b, c, n, s, taps);
}

extern "C" int pcfm_avg_voxelize_plan(const int* coords, int b, int n, int r, int* ind, int* cnt,
                                      void* plan, size_t plan_bytes, void* stream) {
  int s = 0;
  PCFM_CHECK_ARG(b >= 0 && n >= 0, "avg_voxelize_plan: negative size b=%d n=%d", b, n);
  PCFM_CHECK_ARG(cube_fits(r, &s), "avg_voxelize_plan: bad resolution %d", r);
  PCFM_CHECK_ARG(plan != nullptr && plan_bytes >= seg_plan_bytes(b, n, s, 1),
                 "avg_voxelize_plan: plan buffer too small");
  if (b == 0) return PCFM_OK;
  hipStream_t st = (hipStream_t)stream;
  if (n > 0)
    hipLaunchKernelGGL(vox_ind_kernel, dim3(ceil_div(n, 256), b), dim3(256), 0, st, coords, n, r,
                       ind);
  const int e = seg_plan_build<1>(ind, n, true, nullptr, r, b, n, s, cnt,
                                  seg_plan_carve(plan, b, n, s, 1), st);
  return e ? e : check_launch("avg_voxelize_plan");
}

extern "C" int pcfm_avg_voxelize_fwd_planned(const float* feat, const void* plan, int b, int c,
                                             int n, int r, float* out, void* ws, size_t ws_bytes,
                                             void* stream) {
  int s = 0;
  PCFM_CHECK_ARG(b >= 0 && c >= 0 && n >= 0, "avg_voxelize_fwd_planned: negative size");
  PCFM_CHECK_ARG(cube_fits(r, &s), "avg_voxelize_fwd_planned: bad resolution %d", r);
  PCFM_CHECK_ARG(plan != nullptr && ws_bytes >= seg_apply_bytes(b, c, n, s, 1),
                 "avg_voxelize_fwd_planned: workspace too small");
  if (b == 0) return PCFM_OK;
  const int e = seg_apply<1>(feat, seg_plan_carve(const_cast<void*>(plan), b, n, s, 1), true, r, b,
                             c, n, s, out, seg_apply_carve(ws, b, c, n, s, 1), (hipStream_t)stream);
  return e ? e : check_launch("avg_voxelize_fwd_planned");
}

extern "C" int pcfm_trilinear_devoxelize_bwd_plan(const int* inds, const float* wgts, int b, int n,
                                                  int r, void* plan, size_t plan_bytes,
                                                  void* stream) {
  int s = 0;
  PCFM_CHECK_ARG(b >= 0 && n >= 0, "trilinear_devoxelize_bwd_plan: negative size");
  PCFM_CHECK_ARG(cube_fits(r, &s), "trilinear_devoxelize_bwd_plan: bad resolution %d", r);
  PCFM_CHECK_ARG(plan != nullptr && plan_bytes >= seg_plan_bytes(b, n, s, 8),
                 "trilinear_devoxelize_bwd_plan: plan buffer too small");
  if (b == 0) return PCFM_OK;
  const int e = seg_plan_build<8>(inds, 8LL * n, false, wgts, r, b, n, s, nullptr,
                                  seg_plan_carve(plan, b, n, s, 8), (hipStream_t)stream);
  return e ? e : check_launch("trilinear_devoxelize_bwd_plan");
}

extern "C" int pcfm_trilinear_devoxelize_bwd_planned(const float* grad_y, const void* plan, int b,
                                                     int c, int n, int r, float* grad_x, void* ws,
                                                     size_t ws_bytes, void* stream) {
  int s = 0;
  PCFM_CHECK_ARG(b >= 0 && c >= 0 && n >= 0, "trilinear_devoxelize_bwd_planned: negative size");
  PCFM_CHECK_ARG(cube_fits(r, &s), "trilinear_devoxelize_bwd_planned: bad resolution %d", r);
  PCFM_CHECK_ARG(plan != nullptr && ws_bytes >= seg_apply_bytes(b, c, n, s, 8),
                 "trilinear_devoxelize_bwd_planned: workspace too small");
  if (b == 0) return PCFM_OK;
  const int e = seg_apply<8>(grad_y, seg_plan_carve(const_cast<void*>(plan), b, n, s, 8), false,
                             r, b, c, n, s, grad_x, seg_apply_carve(ws, b, c, n, s, 8),
                             (hipStream_t)stream);
  return e ? e : check_launch("trilinear_devoxelize_bwd_planned");
}

// ---------------------------------------------------------------------------
// SE3d's channel MLP (modules/se.py: s = sigmoid(W2 relu(W1 m)), m the pooled
// grid, bias-free Linears) and its backward, each ONE single-block launch: the
// products are B x C x C/r multiply-adds (8 x 256 x 32 at C2), which as torch
// ops were ~12 launches of a few microseconds per PVConv.  Fixed summation
// order (deterministic); fp32 like the module.
// ---------------------------------------------------------------------------
// Every operand is staged in LDS first (coalesced loads by the whole block;
// read straight from global memory, the dependent loads of the reduction loops
// took 17-20 us per launch); W2 transposed (w2t [h][c]).  Long reductions
// (over c) are one 16-lane group per output with the lanes splitting c (a fixed
// xor tree); short ones (over h or b) one thread per output.
__device__ __forceinline__ float se_group_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(1024)
    se_mlp_fwd_kernel(const float* __restrict__ m, const float* __restrict__ w1,
                      const float* __restrict__ w2, int b, int c, int h, float* __restrict__ hid,
                      float* __restrict__ s) {
  extern __shared__ float sh[];  // m [b][c], w1 [h][c], w2t [h][c], hid [b][h]
  float* ms = sh;
  float* w1s = ms + b * c;
  float* w2t = w1s + h * c;
  float* hs = w2t + h * c;
  const int l16 = threadIdx.x & 15, grp = threadIdx.x >> 4, ng = blockDim.x >> 4;
  for (int e = threadIdx.x; e < b * c; e += blockDim.x) ms[e] = m[e];
  for (int e = threadIdx.x; e < h * c; e += blockDim.x) {
    w1s[e] = w1[e];
    const int k = e / h, j = e - k * h;
    w2t[j * c + k] = w2[e];
  }
  __syncthreads();
  for (int e0 = 0; e0 < b * h; e0 += ng) {  // hid = relu(m . W1^T): 16 lanes over c
    const int e = e0 + grp, ec = min(e, b * h - 1);
    const int bi = ec / h, j = ec - bi * h;
    float acc = 0.0f;
    for (int k = l16; k < c; k += 16) acc = __builtin_fmaf(ms[bi * c + k], w1s[j * c + k], acc);
    const float v = fmaxf(se_group_sum(acc), 0.0f);
    if (l16 == 0 && e < b * h) {
      hs[e] = v;
      hid[e] = v;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < b * c; e += blockDim.x) {  // s = sigmoid(hid . W2^T)
    const int bi = e / c, k = e - bi * c;
    float acc = 0.0f;
    for (int j = 0; j < h; ++j) acc = __builtin_fmaf(hs[bi * h + j], w2t[j * c + k], acc);
    s[e] = 1.0f / (1.0f + expf(-acc));
  }
}

// ds -> dm (scaled by dm_scale: the pooling's 1/V folded in), dW1, dW2.
__global__ void __launch_bounds__(1024)
    se_mlp_bwd_kernel(const float* __restrict__ m, const float* __restrict__ hid,
                      const float* __restrict__ s, const float* __restrict__ ds,
                      const float* __restrict__ w1, const float* __restrict__ w2, int b, int c,
                      int h, float dm_scale, float* __restrict__ dm, float* __restrict__ dw1,
                      float* __restrict__ dw2) {
  // dz2 [b][c], m [b][c], w1 [h][c], w2t [h][c], hid [b][h], dz1 [b][h]
  extern __shared__ float sh[];
  float* dz2 = sh;
  float* ms = dz2 + b * c;
  float* w1s = ms + b * c;
  float* w2t = w1s + h * c;
  float* hs = w2t + h * c;
  float* dz1 = hs + b * h;
  const int l16 = threadIdx.x & 15, grp = threadIdx.x >> 4, ng = blockDim.x >> 4;
  for (int e = threadIdx.x; e < b * c; e += blockDim.x) {
    const float sv = s[e];
    dz2[e] = ds[e] * (1.0f - sv) * sv;  // torch's sigmoid backward expression
    ms[e] = m[e];
  }
  for (int e = threadIdx.x; e < h * c; e += blockDim.x) {
    w1s[e] = w1[e];
    const int k = e / h, j = e - k * h;
    w2t[j * c + k] = w2[e];
  }
  for (int e = threadIdx.x; e < b * h; e += blockDim.x) hs[e] = hid[e];
  __syncthreads();
  for (int e = threadIdx.x; e < c * h; e += blockDim.x) {  // dW2 [c][h]: over b
    const int k = e / h, j = e - k * h;
    float acc = 0.0f;
    for (int bi = 0; bi < b; ++bi) acc = __builtin_fmaf(dz2[bi * c + k], hs[bi * h + j], acc);
    dw2[e] = acc;
  }
  for (int e0 = 0; e0 < b * h; e0 += ng) {  // dh = dz2 . W2, relu backward: 16 lanes over c
    const int e = e0 + grp, ec = min(e, b * h - 1);
    const int bi = ec / h, j = ec - bi * h;
    float acc = 0.0f;
    for (int k = l16; k < c; k += 16) acc = __builtin_fmaf(dz2[bi * c + k], w2t[j * c + k], acc);
    acc = se_group_sum(acc);
    if (l16 == 0 && e < b * h) dz1[e] = hs[e] > 0.0f ? acc : 0.0f;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < h * c; e += blockDim.x) {  // dW1 [h][c]: over b
    const int j = e / c, k = e - j * c;
    float acc = 0.0f;
    for (int bi = 0; bi < b; ++bi) acc = __builtin_fmaf(dz1[bi * h + j], ms[bi * c + k], acc);
    dw1[e] = acc;
  }
  for (int e = threadIdx.x; e < b * c; e += blockDim.x) {  // dm [b][c]: over h
    const int bi = e / c, k = e - bi * c;
    float acc = 0.0f;
    for (int j = 0; j < h; ++j) acc = __builtin_fmaf(dz1[bi * h + j], w1s[j * c + k], acc);
    dm[e] = acc * dm_scale;
  }
}

static bool se_mlp_ok(int b, int c, int h) {  // LDS: 2 (b + h) c + 2 b h floats <= 128 KiB
  return b > 0 && c > 0 && h > 0 && 2 * ((long long)b + h) * c + 2LL * b * h <= 32768;
}

extern "C" int pcfm_se_mlp_fwd(const float* m, const float* w1, const float* w2, int b, int c,
                               int h, float* hid, float* s, void* stream) {
  PCFM_CHECK_ARG(se_mlp_ok(b, c, h), "se_mlp_fwd: unsupported size b=%d c=%d h=%d", b, c, h);
  const size_t lds = ((size_t)b * c + 2 * (size_t)h * c + (size_t)b * h) * sizeof(float);
  int e = allow_big_lds((const void*)se_mlp_fwd_kernel);
  if (e) return e;
  hipLaunchKernelGGL(se_mlp_fwd_kernel, dim3(1), dim3(1024), lds, (hipStream_t)stream, m, w1, w2,
                     b, c, h, hid, s);
  return check_launch("se_mlp_fwd");
}

extern "C" int pcfm_se_mlp_bwd(const float* m, const float* hid, const float* s, const float* ds,
                               const float* w1, const float* w2, int b, int c, int h,
                               float dm_scale, float* dm, float* dw1, float* dw2, void* stream) {
  PCFM_CHECK_ARG(se_mlp_ok(b, c, h), "se_mlp_bwd: unsupported size b=%d c=%d h=%d", b, c, h);
  const size_t lds = (2 * (size_t)b * c + 2 * (size_t)h * c + 2 * (size_t)b * h) * sizeof(float);
  int e = allow_big_lds((const void*)se_mlp_bwd_kernel);
  if (e) return e;
  hipLaunchKernelGGL(se_mlp_bwd_kernel, dim3(1), dim3(1024), lds, (hipStream_t)stream, m, hid, s,
                     ds, w1, w2, b, c, h, dm_scale, dm, dw1, dw2);
  return check_launch("se_mlp_bwd");
}

extern "C" int pcfm_rows_dot(const float* a, const float* b, long long rows, int len, float scale,
                             float* out, void* stream) {
  PCFM_CHECK_ARG(rows >= 0 && rows < (1LL << 31) && len >= 0, "rows_dot: bad size %lld x %d",
                 rows, len);
  if (rows == 0) return PCFM_OK;
  hipLaunchKernelGGL(rows_dot_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, a,
                     b, len, scale, out);
  return check_launch("rows_dot");
}

extern "C" int pcfm_rows_affine(float* x, const float* s, const float* t, long long rows, int len,
                                void* stream) {
  PCFM_CHECK_ARG(rows >= 0 && len >= 0 && (len & 3) == 0, "rows_affine: bad size %lld x %d",
                 rows, len);
  if (rows == 0 || len == 0) return PCFM_OK;
  const int per = ceil_div(len / 4, 256);
  PCFM_CHECK_ARG(rows * per < (1LL << 31), "rows_affine: too many rows %lld", rows);
  hipLaunchKernelGGL(rows_affine_kernel, dim3((unsigned)(rows * per)), dim3(256), 0,
                     (hipStream_t)stream, x, s, t, len / 4, per);
  return check_launch("rows_affine");
}
