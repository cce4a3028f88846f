/*
 * pcfm.h -- C ABI of the MI355X-native point-cloud flow-matching hot path.
 *
 * One shared library (point-cloud-flow-matching_amd/csrc/libpcfm_hip.so, built
 * for gfx950) exports every entry point below.  Conventions:
 *
 *   - every pointer is a DEVICE pointer (hipMalloc / torch CUDA tensor storage),
 *     dense and contiguous in the layout written next to it;
 *   - sizes are plain ints; `stream` is a hipStream_t passed as void* (NULL =
 *     the legacy default stream) -- no HIP or torch type appears in this header;
 *   - functions never allocate; scratch memory is passed as `ws` with the byte
 *     count returned by the matching *_workspace_bytes() query;
 *   - return value 0 = success, PCFM_EINVAL = bad argument (nothing launched),
 *     any other positive value = the hipError_t of the failed launch.  The
 *     reference backend calls exit(-1) on a launch failure
 *     (third_party/pvcnn/modules/functional/src/cuda_utils.cuh:28-37); here the
 *     caller decides (the Python layer raises RuntimeError, like TORCH_CHECK).
 *     pcfm_last_error() returns a thread-local description of the last failure.
 *
 * Each function names the reference entry point it replaces (file:line under
 * the reference tree).  Output ownership differs from the reference in one
 * way only: the reference allocates zero-filled outputs inside the binding
 * (torch::zeros); here the caller passes them in and the function writes every
 * element (no pre-zeroing needed), except where "ACCUMULATES" is stated.
 */
#ifndef PCFM_H
#define PCFM_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCFM_OK 0
#define PCFM_EINVAL -1

/* ABI version: bumped on any signature change (4: voxel and pointwise convolution;
 * 5: per-point head kernels; 6: conv3d_igemm workspace,
 * split-operand convolution entry points; fused BatchNorm + activation;
 * 7: channel-segmented pointwise GEMMs, SE3d folded into the devoxelization;
 * 8: per-batch input bias of the head FiLM kernels; 9: split-K workspace of
 * pcfm_conv3d_igemm_cl; 10: fused AdamW + clip + EMA parameter update; 11: segment
 * plans shared by scatters over the same points; 12: the BatchNorm forward entry
 * points take the module's num_batches_tracked counter; 13: occupancy-masked
 * voxel convolution entry points; 14: voxel-list form of the voxel convolution;
 * 15: the head FiLM backward takes shift and recomputes u; 16: devoxelization
 * self-check entry point; 17: BatchNorm statistics from the pointwise GEMM's
 * epilogue; 18: fused EMD approxmatch + matchcost, SE3d MLP kernels; 19: PVConv's
 * second BatchNorm fused with SE3d and the devoxelization; 20: the PV block's
 * post BatchNorm + ReLU fused into its GroupNorm-FiLM residual, the devoxelization
 * self-check of the BatchNorm-transformed gather). */
int pcfm_abi_version(void);
/* Thread-local text of the last non-zero return code. */
const char* pcfm_last_error(void);

/* ------------------------------------------------------------------------
 * PVConv voxel path
 * ---------------------------------------------------------------------- */

/* Scratch bytes pcfm_avg_voxelize_fwd needs for (b, c, n, r). */
size_t pcfm_avg_voxelize_fwd_workspace_bytes(int b, int c, int n, int r);

/* Average-pool voxelization, forward.
 * Replaces avg_voxelize_forward (third_party/pvcnn/modules/functional/src/
 * voxelization/vox.cpp:17-43) -> grid_stats_kernel + avg_voxelize_kernel
 * (vox.cu:18-72).
 *   feat   f32 [b, c, n]        coords i32 [b, 3, n]   (voxel coords in [0, r))
 *   out    f32 [b, c, r^3]      out[c, v] = sum_{i: ind[i]=v} feat[c, i] * (1/cnt[v])
 *   ind    i32 [b, n]           ind[i] = x*r*r + y*r + z
 *   cnt    i32 [b, r^3]         points per voxel                                  */
int pcfm_avg_voxelize_fwd(const float* feat, const int* coords, int b, int c, int n,
                          int r, float* out, int* ind, int* cnt, void* ws,
                          size_t ws_bytes, void* stream);

/* Average-pool voxelization, backward.
 * Replaces avg_voxelize_backward (vox.cpp:54-76) -> avg_voxelize_grad_kernel
 * (vox.cu:86-110).
 *   grad_y f32 [b, c, s]   ind i32 [b, n]   cnt i32 [b, s]   grad_x f32 [b, c, n]   */
int pcfm_avg_voxelize_bwd(const float* grad_y, const int* ind, const int* cnt, int b,
                          int c, int n, int s, float* grad_x, void* stream);

/* grad_x = avg_voxelize_bwd(grad_y) + add (add f32 [b][c][n]): PVConv's
 * feature gradient, voxel branch plus point branch (pvconv.py:35-39), in one
 * gather. */
int pcfm_avg_voxelize_bwd_add(const float* grad_y, const int* ind, const int* cnt,
                              const float* add, int b, int c, int n, int s, float* grad_x,
                              void* stream);

/* Trilinear devoxelization, forward.
 * Replaces trilinear_devoxelize_forward (src/interpolate/trilinear_devox.cpp:18-55)
 * -> trilinear_devoxelize_kernel (trilinear_devox.cu:21-105).
 *   coords f32 [b, 3, n] in [0, r-1]   feat f32 [b, c, r^3]   out f32 [b, c, n]
 *   training != 0: also writes inds i32 [b, 8, n] and wgts f32 [b, 8, n];
 *   training == 0: inds/wgts are ignored (may be NULL).                         */
int pcfm_trilinear_devoxelize_fwd(const float* coords, const float* feat, int b, int c,
                                  int n, int r, int training, float* out, int* inds,
                                  float* wgts, void* stream);

/* out = scale[b, c] * devox(feat)[b, c, i] + add[b, c, i] (either may be NULL):
 * SE3d (modules/se.py:6-17) and the point-branch sum of PVConv.forward
 * (pvconv.py:35-39) folded into the devoxelization; inds/wgts as above. */
int pcfm_trilinear_devoxelize_scale_add_fwd(const float* coords, const float* feat,
                                            const float* scale, const float* add, int b, int c,
                                            int n, int r, int training, float* out, int* inds,
                                            float* wgts, void* stream);

/* pcfm_trilinear_devoxelize_scale_add_fwd of act(bn(x)): x [b][c][r^3] is a
 * PVConv's second voxel-conv output, bn_mean / bn_invstd its batch statistics
 * (pcfm_bn_act_fwd_rowmean), act(t) = t > 0 ? t : slope * t -- BatchNorm3d +
 * LeakyReLU (pvconv.py:20-30) applied while the rows are staged, so the
 * activation is never written.  With add_mean != NULL the add operand is
 * likewise act(bn(add)) with its own statistics and affine (the point branch's
 * pre-BatchNorm1d output, shared_mlp.py:15-27; add_slope 0 = ReLU).
 * r^3 <= 32768. */
int pcfm_trilinear_devoxelize_bn_scale_add_fwd(
    const float* coords, const float* x, const float* bn_mean, const float* bn_invstd,
    const float* gamma, const float* beta, float slope, const float* scale, const float* add,
    const float* add_mean, const float* add_invstd, const float* add_gamma,
    const float* add_beta, float add_slope, int b, int c, int n, int r, int training, float* out,
    int* inds, float* wgts, void* stream);

/* Diagnosis only (not a reference interface): recompute scale * devox(feat) + add
 * per output in the plainest form and compare bit for bit with `out` (and, when
 * inds / wgts are given, the stored corners).  rec i32 [2 + 16 * 8], zeroed by the
 * caller: rec[0] mismatches, rec[1] points whose stored weights do not sum to 1,
 * then up to 16 records {kind (0 out, 1 ind, 2 wgt), b, c, i, got, want, lane, wave}. */
int pcfm_debug_devox_verify(const float* coords, const float* feat, const float* scale,
                            const float* add, const float* out, const int* inds,
                            const float* wgts, int b, int c, int n, int r, int* rec,
                            void* stream);
/* pcfm_debug_devox_verify for pcfm_trilinear_devoxelize_bn_scale_add_fwd: the
 * grid rows enter as act(bn(feat)) and, with add_mean non-NULL, the add operand
 * as act(bn(add)) -- the same transforms, bit for bit. */
int pcfm_debug_devox_verify_bn(const float* coords, const float* feat, const float* bn_mean,
                               const float* bn_invstd, const float* bn_gamma,
                               const float* bn_beta, float slope, const float* scale,
                               const float* add, const float* add_mean, const float* add_invstd,
                               const float* add_gamma, const float* add_beta, float add_slope,
                               const float* out, const int* inds, const float* wgts, int b, int c,
                               int n, int r, int* rec, void* stream);

/* SE3d's channel MLP (modules/se.py over pvconv.py:35-39; se.py:9-19):
 *   hid [b][h] = relu(m [b][c] . W1^T), W1 [h][c];  s [b][c] = sigmoid(hid . W2^T), W2 [c][h]
 * and its backward from ds [b][c]: dm [b][c] (times dm_scale), dW1 [h][c], dW2 [c][h].
 * One single-block launch each; 2 (b + h) c + 2 b h <= 32768 (else PCFM_EINVAL). */
int pcfm_se_mlp_fwd(const float* m, const float* w1, const float* w2, int b, int c, int h,
                    float* hid, float* s, void* stream);
int pcfm_se_mlp_bwd(const float* m, const float* hid, const float* s, const float* ds,
                    const float* w1, const float* w2, int b, int c, int h, float dm_scale,
                    float* dm, float* dw1, float* dw2, void* stream);

/* out[r] = scale * sum_v a[r][v] * b[r][v] (b NULL: plain row sum), rows of
 * `len` floats; deterministic.  (SE3d pooling and its scale gradient.) */
int pcfm_rows_dot(const float* a, const float* b, long long rows, int len, float scale,
                  float* out, void* stream);

/* x[r][v] = s[r] * x[r][v] + t[r] in place (t may be NULL); len % 4 == 0. */
int pcfm_rows_affine(float* x, const float* s, const float* t, long long rows, int len,
                     void* stream);

size_t pcfm_trilinear_devoxelize_bwd_workspace_bytes(int b, int c, int n, int r);

/* Trilinear devoxelization, backward.
 * Replaces trilinear_devoxelize_backward (trilinear_devox.cpp:67-91) ->
 * trilinear_devoxelize_grad_kernel (trilinear_devox.cu:119-162).
 *   grad_y f32 [b, c, n]  inds i32 [b, 8, n]  wgts f32 [b, 8, n]
 *   grad_x f32 [b, c, r^3]                                                      */
int pcfm_trilinear_devoxelize_bwd(const float* grad_y, const int* inds, const float* wgts,
                                  int b, int c, int n, int r, float* grad_x, void* ws,
                                  size_t ws_bytes, void* stream);

/* Ball query.  Replaces ball_query_forward (src/ball_query/ball_query.cpp:6-30)
 * -> ball_query_kernel (ball_query.cu:19-50).
 *   centers f32 [b, 3, m]  points f32 [b, 3, n]  idx i32 [b, m, u]
 *   idx[j, 0..k) = the first k (<= u) point indices with |c - p|^2 < radius^2 in
 *   index order; the remaining slots repeat the first hit; all zeros if none.     */
int pcfm_ball_query(const float* centers, const float* points, int b, int m, int n,
                    float radius, int u, int* idx, void* stream);

/* Grouping forward.  Replaces grouping_forward (src/grouping/grouping.cpp:6-22)
 * -> grouping_kernel (grouping.cu:18-36).
 *   feat f32 [b, c, n]  idx i32 [b, m, u]  out f32 [b, c, m, u]                   */
int pcfm_grouping_fwd(const float* feat, const int* idx, int b, int c, int n, int m,
                      int u, float* out, void* stream);

size_t pcfm_grouping_bwd_workspace_bytes(int b, int c, int n, int m, int u);

/* Grouping backward.  Replaces grouping_backward (grouping.cpp:24-44) ->
 * grouping_grad_kernel (grouping.cu:58-77).
 *   grad_y f32 [b, c, m, u]  idx i32 [b, m, u]  grad_x f32 [b, c, n]              */
int pcfm_grouping_bwd(const float* grad_y, const int* idx, int b, int c, int n, int m,
                      int u, float* grad_x, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Chamfer-3D
 * ---------------------------------------------------------------------- */

size_t pcfm_chamfer_workspace_bytes(int b, int n, int m);

/* Chamfer forward, both directions.  Replaces chamfer_forward
 * (third_party/ChamferDistancePytorch/chamfer3D/chamfer_cuda.cpp:17-19) ->
 * chamfer_cuda_forward / NmDistanceKernel (chamfer3D.cu:12-154).
 *   xyz1 f32 [b, n, 3]  xyz2 f32 [b, m, 3]
 *   dist1 f32 [b, n], idx1 i32 [b, n]: squared distance / index of the nearest
 *   point of xyz2 (ties -> lowest index); dist2/idx2 the same from xyz2 to xyz1.
 *   Squared distance contract: d = fma(dz, dz, fma(dx, dx, dy*dy)), dx = q - p.  */
int pcfm_chamfer_fwd(const float* xyz1, const float* xyz2, int b, int n, int m,
                     float* dist1, float* dist2, int* idx1, int* idx2, void* ws,
                     size_t ws_bytes, void* stream);

/* Chamfer backward.  Replaces chamfer_backward (chamfer_cuda.cpp:22-27) ->
 * NmDistanceGradKernel (chamfer3D.cu:155-195).  ACCUMULATES into grad_xyz1
 * [b, n, 3] and grad_xyz2 [b, m, 3] (callers zero them, as the reference's do). */
int pcfm_chamfer_bwd(const float* xyz1, const float* xyz2, int b, int n, int m,
                     const float* grad_dist1, const float* grad_dist2, const int* idx1,
                     const int* idx2, float* grad_xyz1, float* grad_xyz2, void* stream);

/* ------------------------------------------------------------------------
 * Approximate EMD (approxmatch + matchcost), float and double like the
 * reference's AT_DISPATCH_FLOATING_TYPES (PyTorchEMD/cuda/emd_kernel.cu).
 * ---------------------------------------------------------------------- */

/* elem_bytes = 4 (float) or 8 (double). */
size_t pcfm_emd_workspace_bytes(int b, int n, int m, int elem_bytes);

/* Replaces ApproxMatchForward (emd_kernel.cu:169-191) -> approxmatch (:24-156).
 *   xyz1 [b, n, 3]  xyz2 [b, m, 3]  match [b, m, n]                              */
int pcfm_emd_approxmatch_f32(const float* xyz1, const float* xyz2, int b, int n, int m,
                             float* match, void* ws, size_t ws_bytes, void* stream);
int pcfm_emd_approxmatch_f64(const double* xyz1, const double* xyz2, int b, int n, int m,
                             double* match, void* ws, size_t ws_bytes, void* stream);

/* Replaces MatchCostForward (emd_kernel.cu:255-277) -> matchcost (:199-241).
 *   cost [b] = sum_{k,l} |xyz1[k] - xyz2[l]|^2 * match[l, k]                      */
int pcfm_emd_matchcost_f32(const float* xyz1, const float* xyz2, const float* match, int b,
                           int n, int m, float* cost, void* ws, size_t ws_bytes,
                           void* stream);
int pcfm_emd_matchcost_f64(const double* xyz1, const double* xyz2, const double* match,
                           int b, int n, int m, double* cost, void* ws, size_t ws_bytes,
                           void* stream);

/* ApproxMatchForward + MatchCostForward in one call (the forward of the
 * reference's EarthMoverDistanceFunction, PyTorchEMD/emd.py:14-19): the cost
 * is summed from the match kernel's own values, so match is not read back.
 * match may be NULL (cost only, match not written: a forward whose inputs
 * need no gradient).  cost [b].  Same workspace as approxmatch.             */
int pcfm_emd_approxmatch_cost_f32(const float* xyz1, const float* xyz2, int b, int n, int m,
                                  float* match, float* cost, void* ws, size_t ws_bytes,
                                  void* stream);
int pcfm_emd_approxmatch_cost_f64(const double* xyz1, const double* xyz2, int b, int n, int m,
                                  double* match, double* cost, void* ws, size_t ws_bytes,
                                  void* stream);

/* Replaces MatchCostBackward (emd_kernel.cu:371-396) -> matchcostgrad1/2
 * (:285-353).  grad1 [b, n, 3], grad2 [b, m, 3] fully written.                   */
int pcfm_emd_matchcost_bwd_f32(const float* grad_cost, const float* xyz1, const float* xyz2,
                               const float* match, int b, int n, int m, float* grad1,
                               float* grad2, void* ws, size_t ws_bytes, void* stream);
int pcfm_emd_matchcost_bwd_f64(const double* grad_cost, const double* xyz1,
                               const double* xyz2, const double* match, int b, int n, int m,
                               double* grad1, double* grad2, void* ws, size_t ws_bytes,
                               void* stream);

/* ------------------------------------------------------------------------
 * Voxel convolution (PVConv's Conv3d, kernel 3, stride 1, padding 1;
 * third_party/pvcnn/modules/pvconv.py:20-24 -> torch nn.Conv3d / cuDNN).
 * Implicit GEMM on the bf16 matrix cores with a three-term split of every
 * fp32 operand (hi + lo bf16; products hi*hi + hi*lo + lo*hi accumulated in
 * fp32): ~2^-16 relative error per product, vs 2^-11 for the TF32 the
 * reference's cuDNN path uses by default.  Tensors are NCDHW fp32.
 * ---------------------------------------------------------------------- */

/* Bytes of a split weight image for a (cout, cin, 3, 3, 3) kernel. */
size_t pcfm_conv3d_weight_bytes(int cout, int cin);

/* Split + rearrange w f32 [cout][cin][27] into `wsplit`.  transpose = 0: the
 * forward image [27][cout][cin]; transpose = 1: the backward-data image
 * [27][cin][cout] with the taps mirrored. */
int pcfm_conv3d_prep_weight(const float* w, int cout, int cin, int transpose, void* wsplit,
                            void* stream);

/* 1 if pcfm_conv3d_igemm handles (b, cin, cout, r): cin % 64, cout % 128 and
 * r^3 % 128 must all be 0. */
int pcfm_conv3d_supported(int b, int cin, int cout, int r);

/* y[b, cout, r^3] = conv3x3x3(x[b, cin, r^3], w) (+ bias[cout] if non-NULL),
 * zero padding.  With the transpose=1 image of a (C_out, C_in) kernel and
 * x = grad_y (cin = C_out, cout = C_in) this is the backward-data pass.
 * Fully writes y. */
int pcfm_conv3d_igemm(const float* x, const void* wsplit, const float* bias, int b, int cin,
                      int cout, int r, float* y, void* ws, size_t ws_bytes, void* stream);

/* Scratch bytes for pcfm_conv3d_igemm (the channels-last bf16 hi/lo copy of x
 * plus the split-K partials);
 * 0 = unsupported shape (cin % 64 is needed). */
size_t pcfm_conv3d_igemm_workspace_bytes(int b, int cin, int cout, int r);

/* Channels-last split operand of the convolution GEMMs: xs = [hi | lo], each
 * bf16 [b][r^3][c] with hi = bf16(x), lo = bf16(x - hi), from x f32
 * [b][c][r^3] (NCDHW).  pcfm_conv3d_split_bytes = its size (0: unsupported,
 * c % 64 and r^3 % 64 are needed).  A split operand is reusable: the forward
 * keeps split(x) for the weight gradient, the backward-data pass's split(dY)
 * feeds it too. */
size_t pcfm_conv3d_split_bytes(int b, int c, int r);
int pcfm_conv3d_split(const float* x, int b, int c, int r, void* xs, void* stream);

/* pcfm_conv3d_igemm on an already split input xs (= split(x)); ws holds the
 * split-K partials of small grids (pcfm_conv3d_igemm_cl_workspace_bytes). */
size_t pcfm_conv3d_igemm_cl_workspace_bytes(int b, int cin, int cout, int r);
int pcfm_conv3d_igemm_cl(const void* xs, const void* wsplit, const float* bias, int b, int cin,
                         int cout, int r, float* y, void* ws, size_t ws_bytes, void* stream);

/* pcfm_conv3d_wgrad on split operands xs = split(x), gys = split(grad_y);
 * same workspace query (pcfm_conv3d_wgrad_workspace_bytes). */
int pcfm_conv3d_wgrad_cl(const void* xs, const void* gys, int b, int cin, int cout, int r,
                         float* grad_w, void* ws, size_t ws_bytes, void* stream);

/* Empty-voxel skipping for PVConv's first convolution (pvconv.py:20-27: its
 * input is the voxelization, exactly 0 in every voxel no point falls into, and
 * its input gradient is read back only at occupied voxels, vox.cu:86-110).
 * pcfm_conv3d_occupancy: from the voxelization's counts cnt i32 [b][r^3]
 * (> 0 = occupied) writes masks (pcfm_conv3d_occupancy_bytes(b, r); 0 =
 * unsupported: r^3 % 256 != 0): per 256-voxel tile the taps whose shifted tile
 * holds an occupied voxel (bits 0-26) and whether the tile holds one (bit 31);
 * then per 64-voxel chunk the (dx, dy) pairs whose shifted rows hold one;
 * then per 16-voxel group the taps at which some voxel of the group has an
 * occupied neighbour (bits 0-26). */
size_t pcfm_conv3d_occupancy_bytes(int b, int r);
int pcfm_conv3d_occupancy(const int* cnt, int b, int r, unsigned* masks, void* stream);
/* pcfm_conv3d_igemm_cl skipping exact-zero work: mode 1 (forward over a
 * voxelized input x: taps that read only empty voxels are skipped, bit-identical
 * to pcfm_conv3d_igemm_cl), mode 2 (backward-data into a voxelized grid: only
 * tiles holding an occupied voxel are computed, the others are written 0 --
 * equal to pcfm_conv3d_igemm_cl at every occupied voxel). */
int pcfm_conv3d_igemm_cl_occ(const void* xs, const void* wsplit, const float* bias, int b,
                             int cin, int cout, int r, const unsigned* masks, int mode, float* y,
                             void* ws, size_t ws_bytes, void* stream);
/* Chunk and voxel lists of a voxelized grid (the same counts cnt i32 [b][r^3];
 * a chunk = 32 consecutive voxels): list 0 = the chunks holding an occupied
 * voxel, list 1 = the chunks holding a voxel with an occupied voxel in its
 * 3x3x3 neighbourhood, as chunk indices (b r^3 + v) / 32; lists 2 / 3 = the
 * occupied / neighbourhood-occupied voxels themselves, b r^3 + v; all
 * ascending.  The four device-side counts lead the buffer
 * (pcfm_conv3d_vlist_bytes; 0 = unsupported: r^3 % 256 != 0 or b r^3 >= 2^31). */
size_t pcfm_conv3d_vlist_bytes(int b, int r);
int pcfm_conv3d_vlist(const int* cnt, int b, int r, int* lists, void* stream);
/* pcfm_conv3d_igemm_cl computed at the listed voxels only (GEMM tiles of 256
 * listed voxels, their B rows the voxels' neighbours): which 1 (forward over a
 * voxelized input x, list 3: elsewhere the output is exactly the bias, written
 * as such -- bit-identical to pcfm_conv3d_igemm_cl everywhere), which 0
 * (backward-data into a voxelized grid, bias NULL, list 2: equal to
 * pcfm_conv3d_igemm_cl at every occupied voxel, 0 at every other voxel).  Env
 * PCFM_LIST_VOX (bit 0: which 0, bit 1: which 1; default 3) -- a cleared bit
 * runs that direction over the chunk list (0 / 1) instead: 8 chunks per tile,
 * the same values at the voxels the contract names.  Shapes without the list
 * form (split-K grids, r = 8 at the C2 sizes) run the dense GEMM.
 * Fully writes y; same workspace as pcfm_conv3d_igemm_cl. */
int pcfm_conv3d_igemm_cl_list(const void* xs, const void* wsplit, const float* bias, int b,
                              int cin, int cout, int r, const int* cnt, const int* lists,
                              int which, float* y, void* ws, size_t ws_bytes, void* stream);
/* pcfm_conv3d_wgrad_cl with x a voxelized grid: steps whose X rows are all
 * empty voxels are skipped (bit-identical to pcfm_conv3d_wgrad_cl); workspace
 * pcfm_conv3d_wgrad_occ_workspace_bytes (adds the per-split chunk lists). */
size_t pcfm_conv3d_wgrad_occ_workspace_bytes(int b, int cin, int cout, int r);
int pcfm_conv3d_wgrad_cl_occ(const void* xs, const void* gys, int b, int cin, int cout, int r,
                             const unsigned* masks, float* grad_w, void* ws, size_t ws_bytes,
                             void* stream);

/* Scratch bytes for pcfm_conv3d_wgrad (0 = unsupported shape: cin % 128 is
 * needed in addition to pcfm_conv3d_supported). */
size_t pcfm_conv3d_wgrad_workspace_bytes(int b, int cin, int cout, int r);

/* grad_w f32 [cout][cin][27] = sum_{b, v} grad_y[b, co, v] * x[b, ci, v + off(tap)]
 * (the weight gradient of the padding-1 conv; bf16x3 products, fp32 sums).
 * Fully writes grad_w (no accumulation). */
int pcfm_conv3d_wgrad(const float* x, const float* grad_y, int b, int cin, int cout, int r,
                      float* grad_w, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Pointwise convolution: SharedMLP's Conv1d(C_in, C_out, 1)
 * (third_party/pvcnn/modules/shared_mlp.py:15-27; cuDNN/TF32 in the
 * reference) as bf16x3 GEMMs.  Tensors (B, C, N) fp32; any sizes.
 * ---------------------------------------------------------------------- */

/* Bytes of a split weight image (either orientation) for w [cout][cin]. */
size_t pcfm_pointwise_weight_bytes(int cout, int cin);

/* transpose = 0: forward image of w f32 [cout][cin]; 1: backward-data image. */
int pcfm_pointwise_prep_weight(const float* w, int cout, int cin, int transpose, void* wsplit,
                               void* stream);

/* y[b, cout, n] = W x[b, cin, n] (+ bias).  With the transpose = 1 image of a
 * (C_out, C_in) weight, x = grad_y (cin = C_out) and cout = C_in this is the
 * backward-data pass.  Fully writes y. */
int pcfm_pointwise_gemm(const float* x, const void* wsplit, const float* bias, int b, int cin,
                        int cout, int n, float* y, void* stream);

size_t pcfm_pointwise_wgrad_workspace_bytes(int b, int cin, int cout, int n);

/* grad_w f32 [cout][cin] = sum_{b, p} grad_y[b, co, p] * x[b, ci, p]; fully written. */
int pcfm_pointwise_wgrad(const float* x, const float* grad_y, int b, int cin, int cout, int n,
                         float* grad_w, void* ws, size_t ws_bytes, void* stream);

/* Channel-segmented variants (ContextNet's head_pre over the channel concat of
 * the stage outputs, models.py:460-466, read in place instead of torch.cat).
 * Input part i is an f32 (b, xw[i], n) tensor holding channels
 * [sum xw[<i], sum xw[<=i]) of the logical input; 1..4 parts, every width but
 * the last a multiple of 32.  Output parts likewise, widths a multiple of 128.
 * bias_per_batch = 1: bias is f32 [b][cout] (a per-cloud bias, e.g. the
 * global-feature columns of the weight applied to the broadcast feature). */
int pcfm_pointwise_gemm_parts(int nx, const float* const* x, const int* xw, const void* wsplit,
                              const float* bias, int bias_per_batch, int b, int n, int ny,
                              float* const* y, const int* yw, void* stream);

/* grad_w f32 [cout][sum xw] over a segmented x (any part widths); workspace
 * as pcfm_pointwise_wgrad_workspace_bytes(b, sum xw, cout, n). */
int pcfm_pointwise_wgrad_parts(int nx, const float* const* x, const int* xw, const float* grad_y,
                               int b, int cout, int n, float* grad_w, void* ws, size_t ws_bytes,
                               void* stream);

/* ------------------------------------------------------------------------
 * Per-point head (models.py:62-153, 546-601: the Linear layers of
 * VelocityNetWithContext / ShapeEncoder run under bf16 autocast on
 * rows = B*N points; torch's autocast mm -> cuBLAS in the reference).
 * ---------------------------------------------------------------------- */

size_t pcfm_rows_wgrad_workspace_bytes(long long rows, int m, int n);

/* Weight gradient of a bf16 Linear over `rows` rows (the backward of
 * F.linear's weight under autocast, i.e. mm(grad_y^T, x) in bf16):
 *   a   bf16 [rows][lda]  (grad_y; columns 0..m)
 *   b   bf16 [rows][ldb]  (x; columns 0..n)
 *   out bf16 [m][n] = bf16( sum_r a[r][i] * b[r][j] )  (fp32 accumulation,
 *   split over rows, partials added in a fixed order: deterministic).
 * Fully writes out. */
int pcfm_rows_wgrad_bf16(const void* a, int lda, const void* b, int ldb, long long rows, int m,
                         int n, void* out, void* ws, size_t ws_bytes, void* stream);

size_t pcfm_rows_max_workspace_bytes(int b, int n, int c);

/* ShapeEncoder's global pooling h.max(dim=1) (models.py:156-187) over
 * h bf16 [b][n][c] (c even): values bf16 [b][c] and indices i32 [b][c]
 * (argmax over n, lowest index on ties; NaN propagates). */
int pcfm_rows_max_bf16(const void* h, int b, int n, int c, void* values, int* indices, void* ws,
                       size_t ws_bytes, void* stream);

size_t pcfm_rows_colsum_workspace_bytes(int b, long long rows, int c);

/* out f32 [b][c] = sum over r of x[b][r][c], x bf16 (bf16 = 1) or f32 [b][rows][c],
 * c even and <= 512; deterministic (fixed partial order).  The per-point
 * Linears' bias gradients and the gradient of a per-cloud row broadcast over
 * the points (models.py:594-601 t-gate blend). */
int pcfm_rows_colsum(const void* x, int bf16, int b, long long rows, int c, float* out, void* ws,
                     size_t ws_bytes, void* stream);

/* ContextNet's t-gate blend (models.py:533-541) fused with head_out's permute:
 * out f32 [b][n][c] = alpha[b] * head[b][c][n] + (1 - alpha[b]) * glb[b][c];
 * backward dhead f32 [b][c][n] = alpha[b] * dout[b][n][c] (glb's gradient is
 * (1 - alpha[b]) * pcfm_rows_colsum(dout)). */
int pcfm_tgate_fwd(const float* head, const float* glb, const float* alpha, int b, int c, int n,
                   float* out, void* stream);
int pcfm_tgate_bwd(const float* dout, const float* alpha, int b, int c, int n, float* dhead,
                   void* stream);

/* Trunk rows of VelocityNetWithContext / VelocityNet (models.py:62-79 FiLMBlock,
 * :107-116 residual loop), W = 256 or 512 channels, rows = b*n (batch-major).
 * bf16 tensors are passed as void* (raw 16-bit bf16 bits).
 * h of a block = h16 (bf16 [b*n][w], the input Linear's output) if non-NULL,
 * else uprev + gprev (fp32 + bf16: the previous block's residual sum).
 * hbias (f32 [b][w], may be NULL, used with h16 only): h = bf16(h16 + hbias[b]),
 * the input Linear's batch-constant embedding columns folded out of its GEMM.
 * Forward of one FiLM block:
 *   y = LayerNorm(h; gamma, beta, eps)   u = y * sp1[b] + shift[b]
 *   (sp1 = bf16(1 + scale), shift: bf16 [b][w], per batch element)
 *   writes u f32 [b*n][w], a = bf16(SiLU(u)) [b*n][w], mean/rstd f32 [b*n]. */
int pcfm_head_film_fwd(const void* h16, const float* hbias, const float* uprev,
                       const void* gprev, const float* gamma, const float* beta, const void* sp1,
                       const void* shift, int b, int n, int w, float eps, float* u, void* a,
                       float* mean, float* rstd, void* stream);

/* Output layer's input: a = bf16(SiLU(uprev + gprev)). */
int pcfm_head_silu_fwd(const float* uprev, const void* gprev, int b, int n, int w, void* a,
                       void* stream);

size_t pcfm_head_bwd_workspace_bytes(int b, int n, int w);

/* Backward of one FiLM block given dh_next = dL/dh_{i+1} (f32) and
 * da16 = dL/da (bf16, = dL/dg @ W of the block's Linear):
 *   du = dh_next + da * SiLU'(u);  d sp1[b] = sum_rows du*y;  d shift[b] = sum du;
 *   dy = du * sp1;  d gamma = sum dy*xhat;  d beta = sum dy;
 *   dh = LayerNorm backward (f32, written if dh != NULL) and bf16(dh) -> dh16;
 *   dbias = sum_rows bf16(dh) (the bias gradient of the Linear that produced h),
 *   dbias_b[b] = the same sum per batch element (the hbias rows' gradient).
 * dsp1/dshift/dbias_b f32 [b][w], dgamma/dbeta/dbias f32 [w]; any may be NULL.
 * u (the forward's f32 output) may be NULL when shift (bf16 [b][w]) is given: u
 * is then recomputed from h, mean, rstd, gamma, beta, sp1, shift with the
 * forward's expression -- bit-identical, 2 fewer bytes read per element (ABI 15). */
int pcfm_head_film_bwd(const float* dh_next, const void* da16, const float* u, const void* h16,
                       const float* hbias, const float* uprev, const void* gprev,
                       const float* mean, const float* rstd, const float* gamma,
                       const float* beta, const void* sp1, const void* shift, int b, int n, int w,
                       float* dh,
                       void* dh16, float* dsp1, float* dshift, float* dgamma, float* dbeta,
                       float* dbias, float* dbias_b, void* ws, size_t ws_bytes, void* stream);

/* Backward of a = bf16(SiLU(uprev + gprev)): dh = da * SiLU'(h) -> dh (f32),
 * dh16 (bf16), dbias = sum_rows bf16(dh). */
int pcfm_head_silu_bwd(const void* da16, const float* uprev, const void* gprev, int b, int n,
                       int w, float* dh, void* dh16, float* dbias, void* ws, size_t ws_bytes,
                       void* stream);

/* ------------------------------------------------------------------------
 * BatchNorm (batch statistics, training mode) fused with the activation
 * after it: SharedMLP's BN1d + ReLU (shared_mlp.py:15-27, slope = 0) and
 * PVConv's BN3d + LeakyReLU(0.1) (pvconv.py:20-30, slope = 0.1), over
 * x f32 [b][c][s] (s % 4 == 0).  torch.nn.functional.batch_norm semantics.
 * ---------------------------------------------------------------------- */

size_t pcfm_bn_workspace_bytes(int b, int c, int s);

/* y = act((x - mean) * invstd * gamma + beta), act(v) = v > 0 ? v : slope * v,
 * mean / invstd = batch statistics over (b, s) per channel (biased variance,
 * invstd = 1/sqrt(var + eps)), written to mean / invstd [c].  If running_mean
 * and running_var are non-NULL they are updated in place:
 * r = (1 - momentum) * r + momentum * stat (unbiased variance for running_var).
 * If num_batches_tracked (one int64 on the device) is non-NULL it is incremented
 * by 1 -- the nn.BatchNorm counter torch's batch_norm path advances with a
 * separate launch. */
int pcfm_bn_act_fwd(const float* x, const float* gamma, const float* beta, int b, int c, int s,
                    float eps, float slope, float momentum, float* running_mean,
                    float* running_var, long long* num_batches_tracked, float* y, float* mean,
                    float* invstd, void* ws, size_t ws_bytes, void* stream);

/* SharedMLP layer forward with the BatchNorm statistics produced by the GEMM
 * (shared_mlp.py:21-25: Conv1d -> BatchNorm1d -> ReLU).  For the shapes where
 * pcfm_pointwise_bnstats_groups(b, cin, cout, n) = P > 0,
 * pcfm_pointwise_gemm_bnstats writes y = W x + bias as pcfm_pointwise_gemm and
 * stats f32 [cout][P][2]: per point group (mean, centred sum of squares) --
 * 64-point groups (P = b * ceil(n / 64)) from the 256-row tiles, 32-point
 * groups (P = b * ceil(n / 32)) from the 128-row streaming form (the group size
 * follows from P); pcfm_bn_act_fwd_parts then finalizes them (fixed order, deterministic) and
 * applies the BatchNorm + activation like pcfm_bn_act_fwd, without a
 * statistics pass over y. */
int pcfm_pointwise_bnstats_groups(int b, int cin, int cout, int n);
int pcfm_pointwise_gemm_bnstats(const float* x, const void* wsplit, const float* bias, int b,
                                int cin, int cout, int n, float* y, float* stats, void* stream);
int pcfm_bn_act_fwd_parts(const float* x, const float* part, int P, const float* gamma,
                          const float* beta, int b, int c, int s, float eps, float slope,
                          float momentum, float* running_mean, float* running_var,
                          long long* num_batches_tracked, float* y, float* mean, float* invstd,
                          void* stream);

/* Backward of pcfm_bn_act_fwd given dz = dL/dy: dx [b][c][s] and
 * dgamma / dbeta [c] (all fully written); if dbias_in is non-NULL it receives
 * sum_{b,s} dx [c] -- the bias gradient of the convolution that produced x. */
int pcfm_bn_act_bwd(const float* dz, const float* x, const float* gamma, const float* beta,
                    const float* mean, const float* invstd, int b, int c, int s, float slope,
                    float* dx, float* dgamma, float* dbeta, float* dbias_in, void* ws,
                    size_t ws_bytes, void* stream);

/* pcfm_bn_act_fwd whose output only feeds a voxel convolution: y is written
 * directly as the channels-last bf16 hi/lo split of pcfm_conv3d_split (ys:
 * pcfm_conv3d_split_bytes(b, c, r) bytes, r^3 = s; c, s multiples of 64), not
 * as fp32.  Workspace: pcfm_bn_workspace_bytes(b, c, s). */
int pcfm_bn_act_fwd_split(const float* x, const float* gamma, const float* beta, int b, int c,
                          int s, float eps, float slope, float momentum, float* running_mean,
                          float* running_var, long long* num_batches_tracked, void* ys,
                          float* mean, float* invstd, void* ws, size_t ws_bytes, void* stream);

/* PVConv's second voxel BatchNorm + LeakyReLU fused with SE3d and the
 * devoxelization (pvconv.py:20-39, se.py:6-17), z = act(bn(x)) never written.
 * Forward: pcfm_bn_act_fwd_rowmean = the batch statistics (as pcfm_bn_act_fwd,
 * running stats updated) and rowmean [b][c] = mean over s of z (SE's pooling);
 * then pcfm_trilinear_devoxelize_bn_scale_add_fwd.
 * Backward, from g = devox_bwd(dout) [b][c][s]: with dz = se_scale * g + dmv
 * (dmv [b][c] = SE's pooling gradient dm / s), pcfm_bn_se_bwd_stats writes
 * rowstats [5][b][c] = (sum z g, sum a g, sum a, sum a g xhat, sum a xhat) per
 * row, a = act'; rowstats[0] is SE's ds.  pcfm_bn_se_bwd_apply_split then writes
 * dx as pcfm_bn_act_bwd_split does (conv split operand, dgamma, dbeta,
 * dbias_in).  c, s multiples of 64.  Deterministic. */
/* BatchNorm batch statistics only (mean, invstd; running stats and the counter
 * updated as pcfm_bn_act_fwd): from x by a statistics pass (part NULL; workspace
 * pcfm_bn_workspace_bytes), or finalized from a producer's epilogue statistics
 * part [c][P] (pcfm_pointwise_gemm_bnstats, P = b * ceil(s / 64) or b * ceil(s / 32)). */
int pcfm_bn_fwd_stats(const float* x, const float* part, int P, int b, int c, int s, float eps,
                      float momentum, float* running_mean, float* running_var,
                      long long* num_batches_tracked, float* mean, float* invstd, void* ws,
                      size_t ws_bytes, void* stream);
size_t pcfm_bn_act_fwd_rowmean_workspace_bytes(int b, int c, int s);
int pcfm_bn_act_fwd_rowmean(const float* x, const float* gamma, const float* beta, int b, int c,
                            int s, float eps, float slope, float momentum, float* running_mean,
                            float* running_var, long long* num_batches_tracked, float* rowmean,
                            float* mean, float* invstd, void* ws, size_t ws_bytes, void* stream);
size_t pcfm_bn_se_bwd_workspace_bytes(int b, int c, int s);
int pcfm_bn_se_bwd_stats(const float* g, const float* x, const float* mean, const float* invstd,
                         const float* gamma, const float* beta, int b, int c, int s, float slope,
                         float* rowstats, void* ws, size_t ws_bytes, void* stream);
int pcfm_bn_se_bwd_apply_split(const float* g, const float* x, const float* mean,
                               const float* invstd, const float* gamma, const float* beta,
                               const float* se_scale, const float* dmv, const float* rowstats,
                               int b, int c, int s, float slope, void* dxs, float* dgamma,
                               float* dbeta, float* dbias_in, void* ws, size_t ws_bytes,
                               void* stream);

/* pcfm_bn_act_bwd for a voxel convolution's output x [b][c][s] (c, s multiples
 * of 64) whose dx only feeds that convolution's backward: dx is written
 * directly as the channels-last bf16 hi/lo split of pcfm_conv3d_split
 * (dxs: pcfm_conv3d_split_bytes(b, c, r) bytes, r^3 = s), not as fp32.
 * dgamma / dbeta / dbias_in as pcfm_bn_act_bwd (dbias_in summed per 64-voxel
 * tile, then over tiles in a fixed order). */
size_t pcfm_bn_act_bwd_split_workspace_bytes(int b, int c, int s);
int pcfm_bn_act_bwd_split(const float* dz, const float* x, const float* gamma, const float* beta,
                          const float* mean, const float* invstd, int b, int c, int s,
                          float slope, void* dxs, float* dgamma, float* dbeta, float* dbias_in,
                          void* ws, size_t ws_bytes, void* stream);

/* GroupNorm + FiLM + residual of the hybrid backbone's PV blocks
 * (models.py:322-346 _FiLM1d(norm="group"), :349-368 _PVBlock):
 *   out = x + (GroupNorm(x; groups, w, bias, eps) * (1 + gamma[b]) + beta[b])
 * x f32 [b][c][n] (n % 4 == 0, c <= 1024), gamma / beta f32 [b][c];
 * mean / rstd f32 [b][groups] saved for the backward. */
size_t pcfm_gn_film_workspace_bytes(int b, int c, int n, int groups);
int pcfm_gn_film_res_fwd(const float* x, const float* w, const float* bias, const float* gamma,
                         const float* beta, int b, int c, int n, int groups, float eps,
                         float* out, float* mean, float* rstd, void* ws, size_t ws_bytes,
                         void* stream);
/* dx [b][c][n], dw / dbias [c], dgamma / dbeta [b][c] from dout = dL/dout. */
int pcfm_gn_film_res_bwd(const float* dout, const float* x, const float* w, const float* bias,
                         const float* gamma, const float* mean, const float* rstd, int b, int c,
                         int n, int groups, float* dx, float* dw, float* dbias, float* dgamma,
                         float* dbeta, void* ws, size_t ws_bytes, void* stream);

/* The PV block's post SharedMLP activation fused into its GroupNorm + FiLM +
 * residual (models.py:349-368; shared_mlp.py:15-27 for the BatchNorm + ReLU):
 * the GroupNorm's input is z = act(bn(y)) for y f32 [b][c][n], the post 1x1
 * conv's output, with the BatchNorm's batch statistics bn_mean / bn_invstd,
 * affine bn_gamma / bn_beta and act(v) = v > 0 ? v : slope v (slope 0: ReLU)
 * -- z is computed as pcfm_bn_act_fwd does, bit for bit, and never written:
 *   out = z + (GroupNorm(z) * (1 + gamma[b]) + beta[b]).
 * Same workspace as pcfm_gn_film_res_*.  Replaces pcfm_bn_act_fwd(y) followed
 * by pcfm_gn_film_res_fwd(z). */
int pcfm_gn_film_res_fwd_bnin(const float* y, const float* bn_mean, const float* bn_invstd,
                              const float* bn_gamma, const float* bn_beta, float slope,
                              const float* w, const float* bias, const float* gamma,
                              const float* beta, int b, int c, int n, int groups, float eps,
                              float* out, float* mean, float* rstd, void* ws, size_t ws_bytes,
                              void* stream);
/* Backward: dz = dL/dz f32 [b][c][n] and the GroupNorm / FiLM gradients as
 * pcfm_gn_film_res_bwd, plus the BatchNorm backward statistics of
 * g = dz * act'(bn(y)) -- bnpart f32 [c][P][2] = (sum g, sum g * xhat) over
 * P = pcfm_gn_bnin_parts(b, n) blocks per channel -- for
 * pcfm_bn_act_bwd_apply_parts (no separate statistics pass over (dz, y)). */
int pcfm_gn_bnin_parts(int b, int n);
int pcfm_gn_film_res_bwd_bnin(const float* dout, const float* y, const float* bn_mean,
                              const float* bn_invstd, const float* bn_gamma, const float* bn_beta,
                              float slope, const float* w, const float* bias, const float* gamma,
                              const float* mean, const float* rstd, int b, int c, int n,
                              int groups, float* dz, float* dw, float* dbias, float* dgamma,
                              float* dbeta, float* bnpart, void* ws, size_t ws_bytes,
                              void* stream);
/* pcfm_bn_act_bwd's apply pass on given statistics part f32 [c][P][2]
 * (sum g, sum g * xhat per block): dx, dgamma, dbeta and, when dbias_in is
 * non-NULL, the producer's bias gradient (ws: pcfm_bn_workspace_bytes). */
int pcfm_bn_act_bwd_apply_parts(const float* dz, const float* x, const float* gamma,
                                const float* beta, const float* mean, const float* invstd,
                                const float* part, int P, int b, int c, int s, float slope,
                                float* dx, float* dgamma, float* dbeta, float* dbias_in, void* ws,
                                size_t ws_bytes, void* stream);

/* SiLU(GroupNorm(x; w, bias, groups, eps)) over x f32 [b][c][n] (ContextNet's
 * head_norm + head_act, models.py:460-466); mean/rstd f32 [b][groups]; same
 * workspace as pcfm_gn_film_res_*.  Backward: dx, dw, dbias from dout. */
int pcfm_gn_silu_fwd(const float* x, const float* w, const float* bias, int b, int c, int n,
                     int groups, float eps, float* out, float* mean, float* rstd, void* ws,
                     size_t ws_bytes, void* stream);
int pcfm_gn_silu_bwd(const float* dout, const float* x, const float* w, const float* bias,
                     const float* mean, const float* rstd, int b, int c, int n, int groups,
                     float* dx, float* dw, float* dbias, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Segment plans.  avg_voxelize_fwd and trilinear_devoxelize_bwd are scatters:
 * a stable sort of the points by target voxel + a list of work units (the
 * plan), then the deterministic segment sums of the features (the apply).  The
 * plan depends on the coordinates only, and the hybrid backbone runs two PVConv
 * blocks per stage on the SAME points (models.py:371-389 _PVStage: PVConv
 * passes `coords` through, pvconv.py:35-38), so it is built once per
 * (points, resolution) and applied to every block's features.  The one-shot
 * entry points above are plan + apply in one workspace; results are identical.
 * taps: 1 (voxelization: key = voxel of the rounded coordinate) or 8
 * (devoxelization backward: key = base cell inds[b][0][i], 8 trilinear taps).
 * ---------------------------------------------------------------------- */
size_t pcfm_seg_plan_bytes(int b, int n, int r, int taps);
size_t pcfm_seg_apply_workspace_bytes(int b, int c, int n, int r, int taps);
/* Voxelization plan from integer coords [b][3][n]: also writes ind [b][n] and
 * cnt [b][r^3] exactly as pcfm_avg_voxelize_fwd does. */
int pcfm_avg_voxelize_plan(const int* coords, int b, int n, int r, int* ind, int* cnt,
                           void* plan, size_t plan_bytes, void* stream);
/* out [b][c][r^3] of pcfm_avg_voxelize_fwd on a voxelization plan. */
int pcfm_avg_voxelize_fwd_planned(const float* feat, const void* plan, int b, int c, int n, int r,
                                  float* out, void* ws, size_t ws_bytes, void* stream);
/* Devoxelization-backward plan from the forward's inds i32 / wgts f32 [b][8][n]. */
int pcfm_trilinear_devoxelize_bwd_plan(const int* inds, const float* wgts, int b, int n, int r,
                                       void* plan, size_t plan_bytes, void* stream);
/* grad_x [b][c][r^3] of pcfm_trilinear_devoxelize_bwd on a devoxelization plan. */
int pcfm_trilinear_devoxelize_bwd_planned(const float* grad_y, const void* plan, int b, int c,
                                          int n, int r, float* grad_x, void* ws, size_t ws_bytes,
                                          void* stream);

/* ------------------------------------------------------------------------
 * Parameter update of the train step (reference train.py:652-661):
 * GradScaler.unscale_ -> clip_grad_norm_(all parameters) -> AdamW.step
 * (torch.optim.AdamW, train.py:249-253; its foreach arithmetic) -> EMA update
 * of the new parameters (util.py:17-21) -- three launches over a device table
 * of parameters instead of torch's per-list multi-tensor passes.
 * ---------------------------------------------------------------------- */
#define PCFM_ADAMW_CHUNK 4096     /* elements per block of the update kernels */
#define PCFM_ADAMW_MAX_GROUPS 8   /* optimizer parameter groups */
/* flags */
#define PCFM_ADAMW_VEC4 1  /* every pointer 16-B aligned and n % 4 == 0 */
#define PCFM_ADAMW_SKIP 2  /* no gradient (grad None): no update, not in the norm */
#define PCFM_ADAMW_EMA 4   /* ema points at the parameter's EMA shadow */
typedef struct {
  float* p;        /* parameter f32 [n] */
  const float* g;  /* gradient f32 [n] (scaled by the GradScaler scale) */
  float* m;        /* AdamW exp_avg f32 [n] */
  float* v;        /* AdamW exp_avg_sq f32 [n] */
  float* ema;      /* EMA shadow f32 [n] or NULL */
  long long n;
  int group;       /* parameter group (lr, weight decay) */
  int flags;
} pcfm_adamw_tensor;

/* Chunk length (PCFM_ADAMW_CHUNK) and scratch of pcfm_adamw_grad_norm. */
int pcfm_adamw_chunk_elems(void);
size_t pcfm_adamw_workspace_bytes(int nchunks);
/* tensors: device table [ntensors]; chunks: device int [nchunks][2] = (tensor
 * index, first element), one per PCFM_ADAMW_CHUNK elements of every tensor.
 * scale: device f32 [1] GradScaler scale or NULL; max_norm <= 0: no clipping.
 * steps: device f32 [ntensors] per-tensor AdamW step counts (+1 for every tensor
 * with a gradient unless found_inf).  state: device f32 [4]: [0] total gradient
 * norm (clip_grad_norm_'s return value), [1] gradient multiplier (1/scale * clip
 * coefficient), [2] found_inf (GradScaler: skip the step). */
int pcfm_adamw_grad_norm(const pcfm_adamw_tensor* tensors, int ntensors, const int* chunks,
                         int nchunks, const float* scale, float max_norm, float* steps,
                         float* state, void* ws, size_t ws_bytes, void* stream);
/* AdamW step with the state pcfm_adamw_grad_norm wrote (no update when found_inf),
 * then shadow = shadow * d + (1 - d) * p for the entries with an EMA shadow (also
 * when the step is skipped).  lr / weight_decay: HOST arrays [ngroups]. */
int pcfm_adamw_ema_step(const pcfm_adamw_tensor* tensors, const int* chunks, int nchunks,
                        const float* steps, const float* state, int ngroups, const double* lr,
                        const double* weight_decay, double beta1, double beta2, double eps,
                        double ema_decay, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PCFM_H */
