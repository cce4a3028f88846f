"""BatchNorm (training-mode batch statistics) fused with the activation that
follows it on the PVConv path: SharedMLP's BN1d + ReLU
(third_party/pvcnn/modules/shared_mlp.py:15-27) and PVConv's BN3d +
LeakyReLU(0.1) (third_party/pvcnn/modules/pvconv.py:20-30).

`bn_act(x, bn, slope)` computes act(bn(x)) with the nn.BatchNorm module's own
parameters and buffers: on a HIP device in training mode it runs pcfm's fused
kernels (csrc/norm.hip; running_mean / running_var / num_batches_tracked
updated as torch does); otherwise (eval mode, CPU, momentum=None) the module
and the activation run as in the reference.
"""
import torch
import torch.nn.functional as F

__all__ = ["bn_act", "conv_bn_act", "gn_film_residual", "post_gn_film_residual"]

# PCFM_DEBUG_CHECKS=1: assert the preconditions of the exact-skip fast paths
_DEBUG_CHECKS = __import__("os").environ.get("PCFM_DEBUG_CHECKS") == "1"
# SharedMLP BatchNorm statistics from the GEMM epilogue (PCFM_BN_FROM_GEMM=0: separate pass)
_BN_FROM_GEMM = __import__("os").environ.get("PCFM_BN_FROM_GEMM", "1") != "0"


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, nbt, eps, momentum, slope):
        from pcfm import ops
        y, mean, invstd = ops.bn_act_forward(x, weight, bias, eps, slope, momentum, running_mean,
                                             running_var, nbt)
        ctx.save_for_backward(x, weight, bias, mean, invstd)
        ctx.slope = slope
        return y

    @staticmethod
    def backward(ctx, dy):
        from pcfm import ops
        x, weight, bias, mean, invstd = ctx.saved_tensors
        dx, dgamma, dbeta, _ = ops.bn_act_backward(dy, x, weight, bias, mean, invstd, ctx.slope)
        return dx, dgamma, dbeta, None, None, None, None, None, None


def _fusable(x: torch.Tensor, bn) -> bool:
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() >= 3 and bn.training
            and bn.affine and bn.track_running_stats and bn.momentum is not None
            and bn.running_mean is not None and not torch.is_autocast_enabled("cuda")):
        return False
    s = x[0, 0].numel()
    # one value per channel: torch's batch_norm raises ("Expected more than 1 value
    # per channel"), so such a call takes the module path and raises the same way
    return (s % 4 == 0 and x.shape[0] * x.shape[1] < 65536 and x.numel() > 0
            and x.shape[0] * s > 1)


def bn_act(x: torch.Tensor, bn, slope: float) -> torch.Tensor:
    """act(bn(x)) with act(v) = v if v > 0 else slope * v (slope 0: ReLU)."""
    if _fusable(x, bn):  # num_batches_tracked += 1 inside the kernel (no extra launch)
        return _BNAct.apply(x.contiguous(), bn.weight, bn.bias, bn.running_mean, bn.running_var,
                            _nbt(bn), float(bn.eps), float(bn.momentum), float(slope))
    y = bn(x)
    return F.relu(y, inplace=True) if slope == 0 else F.leaky_relu(y, slope, inplace=True)


class _PwBnAct(torch.autograd.Function):
    """SharedMLP layer: act(BN(Conv1d_1x1(x))) in one autograd node, so the
    conv's bias gradient comes out of the BN backward pass (sum of dBN/dy)."""

    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, rmean, rvar, nbt, eps, momentum, slope):
        from pcfm import ops
        # the 256-row GEMM hands the BatchNorm its statistics (no pass over y)
        ys = ops.pointwise_forward_bnstats(x, w, b) if _BN_FROM_GEMM else None
        if ys is not None:
            y, stats = ys
            z, mean, invstd = ops.bn_act_forward_parts(y, stats, gamma, beta, eps, slope,
                                                       momentum, rmean, rvar, nbt)
        else:
            y = ops.pointwise_forward(x, w, b)
            z, mean, invstd = ops.bn_act_forward(y, gamma, beta, eps, slope, momentum, rmean,
                                                 rvar, nbt)
        ctx.save_for_backward(x, w, y, gamma, beta, mean, invstd)
        ctx.slope, ctx.has_bias = slope, b is not None
        return z

    @staticmethod
    def backward(ctx, dz):
        from pcfm import ops
        x, w, y, gamma, beta, mean, invstd = ctx.saved_tensors
        dy, dgamma, dbeta, db = ops.bn_act_backward(dz, y, gamma, beta, mean, invstd, ctx.slope,
                                                    want_dbias_in=ctx.has_bias)
        dx = ops.pointwise_backward_data(dy, w) if ctx.needs_input_grad[0] else None
        dw = ops.pointwise_backward_weight(x, dy).view_as(w) if ctx.needs_input_grad[1] else None
        return dx, dw, db, dgamma, dbeta, None, None, None, None, None, None


class _Conv3dBnAct(torch.autograd.Function):
    """PVConv voxel layer: act(BN3d(Conv3d(x))) in one autograd node: split(x)
    kept for the weight gradient, the conv bias gradient from the BN backward."""

    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, rmean, rvar, nbt, eps, momentum, slope):
        from pcfm import ops
        bsz, cin, r = x.shape[0], x.shape[1], x.shape[2]
        cout = w.shape[0]
        xs = ops.conv3d_split(x)
        y = ops.conv3d_igemm_split(xs, ops.conv3d_prep_weight(w, False), b, bsz, cin, cout, r,
                                   "conv3d_fwd")
        z, mean, invstd = ops.bn_act_forward(y, gamma, beta, eps, slope, momentum, rmean, rvar,
                                             nbt)
        ctx.save_for_backward(xs, w, y, gamma, beta, mean, invstd)
        ctx.slope, ctx.has_bias, ctx.dims = slope, b is not None, (bsz, cin, cout, r)
        return z

    @staticmethod
    def backward(ctx, dz):
        from pcfm import ops
        xs, w, y, gamma, beta, mean, invstd = ctx.saved_tensors
        bsz, cin, cout, r = ctx.dims
        # BN backward writes d(conv output) straight into the split layout the
        # conv's backward GEMMs read (no fp32 dy pass)
        gys, dgamma, dbeta, db = ops.bn_act_backward_split(dz, y, gamma, beta, mean, invstd,
                                                           ctx.slope, want_dbias_in=ctx.has_bias)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = ops.conv3d_igemm_split(gys, ops.conv3d_prep_weight(w, True), None, bsz, cout, cin,
                                        r, "conv3d_bwd_data")
        if ctx.needs_input_grad[1]:
            dw = ops.conv3d_wgrad_split(xs, gys, bsz, cin, cout, r)
        return dx, dw, db, dgamma, dbeta, None, None, None, None, None, None


def _pair_head(x, w1, b1, g1, bt1, rm1, rv1, nbt1, w2, b2, eps1, mom1, slope1, occ):
    """Conv1 -> BN1 + act (written only as Conv2's split input) -> Conv2:
    -> (xs, y1, m1, is1, z1s, y2), y2 the second conv's pre-BatchNorm output."""
    from pcfm import ops
    bsz, cin, r = x.shape[0], x.shape[1], x.shape[2]
    cmid, cout = w1.shape[0], w2.shape[0]
    xs = ops.conv3d_split(x)
    masks, vl, cnt = (occ.masks, occ.lists, occ.cnt) if occ is not None else (None, None, None)
    y1 = ops.conv3d_igemm_split(xs, ops.conv3d_prep_weight(w1, False), b1, bsz, cin, cmid,
                                r, "conv3d_fwd", occ=masks, occ_mode=1, vlists=vl, cnt=cnt)
    z1s, m1, is1 = ops.bn_act_forward_split(y1, g1, bt1, eps1, slope1, mom1, rm1, rv1, nbt1)
    y2 = ops.conv3d_igemm_split(z1s, ops.conv3d_prep_weight(w2, False), b2, bsz, cmid, cout,
                                r, "conv3d_fwd")
    return xs, y1, m1, is1, z1s, y2


def _pair_tail(gys2, xs, w1, y1, g1, bt1, m1, is1, z1s, w2, slope1, has_bias1, dims, occ,
               needs_dx):
    """Backward of _pair_head from split(d y2): -> (dx, dw1, db1, dg1, dbt1, dw2)."""
    from pcfm import ops
    bsz, cin, cmid, cout, r = dims
    dz1 = ops.conv3d_igemm_split(gys2, ops.conv3d_prep_weight(w2, True), None, bsz, cout,
                                 cmid, r, "conv3d_bwd_data")
    dw2 = ops.conv3d_wgrad_split(z1s, gys2, bsz, cmid, cout, r)
    del gys2
    gys1, dg1, dbt1, db1 = ops.bn_act_backward_split(dz1, y1, g1, bt1, m1, is1, slope1,
                                                     want_dbias_in=has_bias1)
    del dz1
    dx = None
    masks, vl, cnt = (occ.masks, occ.lists, occ.cnt) if occ is not None else (None, None, None)
    if needs_dx:
        dx = ops.conv3d_igemm_split(gys1, ops.conv3d_prep_weight(w1, True), None, bsz, cmid,
                                    cin, r, "conv3d_bwd_data", occ=masks, occ_mode=2,
                                    vlists=vl, cnt=cnt)
    dw1 = ops.conv3d_wgrad_split(xs, gys1, bsz, cin, cmid, r, occ=masks)
    return dx, dw1, db1, dg1, dbt1, dw2


class _Conv3dBnActPair(torch.autograd.Function):
    """PVConv's two voxel layers act2(BN2(Conv2(act1(BN1(Conv1(x)))))) in one
    autograd node, so the inner activation lives only as Conv2's channels-last
    split input (bn_act_forward_split) and its gradient only as Conv1's split
    grad (bn_act_backward_split): no fp32 pass over either.

    `occ` (PVConv, x = the voxelization's grid: pcfm.plans.conv_occupancy)
    skips Conv1's exact-zero work: its forward is computed at the voxels with
    an occupied voxel in their 3x3x3 neighbourhood only (elsewhere the output
    is exactly the bias; with voxel lists, else per tile and tap), its weight
    gradient skips steps that read only empty voxels (bit-identical), and its
    input gradient is computed at the occupied voxels only (the voxelization's
    backward reads it there only, vox.cu:86-110; the returned dx is 0 at the
    other voxels, or in the other tiles without lists)."""

    @staticmethod
    def forward(ctx, x, w1, b1, g1, bt1, rm1, rv1, nbt1, w2, b2, g2, bt2, rm2, rv2, nbt2, eps1,
                mom1, slope1, eps2, mom2, slope2, occ=None):
        from pcfm import ops
        xs, y1, m1, is1, z1s, y2 = _pair_head(x, w1, b1, g1, bt1, rm1, rv1, nbt1, w2, b2, eps1,
                                              mom1, slope1, occ)
        z2, m2, is2 = ops.bn_act_forward(y2, g2, bt2, eps2, slope2, mom2, rm2, rv2, nbt2)
        ctx.save_for_backward(xs, w1, y1, g1, bt1, m1, is1, z1s, w2, y2, g2, bt2, m2, is2)
        ctx.occ = occ
        ctx.slopes = (slope1, slope2)
        ctx.has_bias = (b1 is not None, b2 is not None)
        ctx.dims = (x.shape[0], x.shape[1], w1.shape[0], w2.shape[0], x.shape[2])
        return z2

    @staticmethod
    def backward(ctx, dz2):
        from pcfm import ops
        xs, w1, y1, g1, bt1, m1, is1, z1s, w2, y2, g2, bt2, m2, is2 = ctx.saved_tensors
        gys2, dg2, dbt2, db2 = ops.bn_act_backward_split(dz2, y2, g2, bt2, m2, is2,
                                                         ctx.slopes[1],
                                                         want_dbias_in=ctx.has_bias[1])
        dx, dw1, db1, dg1, dbt1, dw2 = _pair_tail(gys2, xs, w1, y1, g1, bt1, m1, is1, z1s, w2,
                                                  ctx.slopes[0], ctx.has_bias[0], ctx.dims,
                                                  ctx.occ, ctx.needs_input_grad[0])
        return (dx, dw1, db1, dg1, dbt1, None, None, None, dw2, db2, dg2, dbt2, None, None,
                None, None, None, None, None, None, None, None)


def pair_fusable(conv1, bn1, conv2, bn2, x: torch.Tensor) -> bool:
    """Whether conv_bn_act_pair runs its two layers as one fused GPU node."""
    from modules.shared_mlp import PointwiseConv1d
    ok = (not isinstance(conv1, PointwiseConv1d) and not isinstance(conv2, PointwiseConv1d)
          and _fusable_pre(bn1) and _fusable_pre(bn2) and hasattr(conv1, "x3_ok")
          and hasattr(conv2, "x3_ok") and conv1.x3_ok(x) and conv1.bias is not None
          and conv2.bias is not None and conv1.out_channels % 64 == 0
          and x[0, 0].numel() % 64 == 0 and x.shape[0] * conv2.out_channels < 65536
          and x.shape[0] * conv1.out_channels < 65536 and x.shape[0] * x[0, 0].numel() > 1)
    if ok:
        from pcfm import ops
        # shape / dtype / device stand-in for conv1's output (no allocation)
        probe = x.new_empty(()).expand((x.shape[0], conv1.out_channels) + tuple(x.shape[2:]))
        ok = conv2.x3_ok(probe) and ops.conv3d_split_supported(probe)
    return ok


def conv_bn_act_pair(conv1, bn1, slope1: float, conv2, bn2, slope2: float,
                     x: torch.Tensor, voxelized_input_occ=None) -> torch.Tensor:
    """act2(bn2(conv2(act1(bn1(conv1(x)))))) for two VoxelConv3d layers: one
    autograd node on the GPU path when both layers qualify, else two
    conv_bn_act calls.

    voxelized_input_occ (pcfm.plans.conv_occupancy of the points x was
    voxelized from; PVConv only): x must be exactly 0 at every empty voxel, and
    the returned input gradient is then computed at the OCCUPIED voxels only
    (0 elsewhere) -- correct for the voxelization's backward, which reads it
    there only (vox.cu:86-110), wrong for any other consumer of dx.  With
    PCFM_DEBUG_CHECKS=1 the zero-outside-occupancy precondition is asserted."""
    occ = voxelized_input_occ
    if occ is not None and _DEBUG_CHECKS and x.is_cuda:
        empty = (occ.cnt == 0).view(x.shape[0], 1, -1).expand(-1, x.shape[1], -1)
        if bool((x.reshape(x.shape[0], x.shape[1], -1)[empty] != 0).any()):
            raise AssertionError("conv_bn_act_pair: voxelized_input_occ given but x is non-zero "
                                 "at an empty voxel")
    if not pair_fusable(conv1, bn1, conv2, bn2, x):
        x = conv_bn_act(conv1, bn1, x, slope1)
        return conv_bn_act(conv2, bn2, x, slope2)
    return _Conv3dBnActPair.apply(
        x.contiguous(), conv1.weight, conv1.bias, bn1.weight, bn1.bias, bn1.running_mean,
        bn1.running_var, _nbt(bn1), conv2.weight, conv2.bias, bn2.weight, bn2.bias,
        bn2.running_mean, bn2.running_var, _nbt(bn2), float(bn1.eps), float(bn1.momentum),
        float(slope1), float(bn2.eps), float(bn2.momentum), float(slope2), occ)


def conv_bn_act(conv, bn, x: torch.Tensor, slope: float) -> torch.Tensor:
    """act(bn(conv(x))) for a PointwiseConv1d / VoxelConv3d `conv`: one fused
    autograd node on the GPU path, the modules' own forwards otherwise."""
    if _fusable_pre(bn) and hasattr(conv, "x3_ok") and conv.x3_ok(x) and conv.bias is not None:
        out_shape_ok = (x[0, 0].numel() % 4 == 0 and x.shape[0] * conv.out_channels < 65536
                        and x.shape[0] * x[0, 0].numel() > 1)
        if out_shape_ok:
            from modules.shared_mlp import PointwiseConv1d
            fn = _PwBnAct if isinstance(conv, PointwiseConv1d) else _Conv3dBnAct
            return fn.apply(x.contiguous(), conv.weight, conv.bias, bn.weight, bn.bias,
                            bn.running_mean, bn.running_var, _nbt(bn), float(bn.eps),
                            float(bn.momentum), float(slope))
    return bn_act(conv(x), bn, slope)


def _nbt(bn):
    """bn.num_batches_tracked for the fused kernels to increment (channel 0's
    statistics publisher adds 1, as torch's batch_norm path does with a separate
    add_ launch); None when the module has no int64 counter on the device."""
    t = getattr(bn, "num_batches_tracked", None)
    if t is None or t.dtype != torch.int64 or t.numel() != 1 or not t.is_cuda:
        return None
    return t


def _fusable_pre(bn) -> bool:
    return (bn.training and bn.affine and bn.track_running_stats and bn.momentum is not None
            and bn.running_mean is not None)


class _GNFiLMRes(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta, groups, eps):
        from pcfm import ops
        out, mean, rstd = ops.gn_film_res_forward(x, weight, bias, gamma, beta, groups, eps)
        ctx.save_for_backward(x, weight, bias, gamma, mean, rstd)
        ctx.groups = groups
        return out

    @staticmethod
    def backward(ctx, dout):
        from pcfm import ops
        x, weight, bias, gamma, mean, rstd = ctx.saved_tensors
        dx, dw, db, dg, dbt = ops.gn_film_res_backward(dout, x, weight, bias, gamma, mean, rstd,
                                                       ctx.groups)
        return dx, dw, db, dg, dbt, None, None


class _GNSiLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, groups, eps):
        from pcfm import ops
        out, mean, rstd = ops.gn_silu_forward(x, weight, bias, groups, eps)
        ctx.save_for_backward(x, weight, bias, mean, rstd)
        ctx.groups = groups
        return out

    @staticmethod
    def backward(ctx, dout):
        from pcfm import ops
        x, weight, bias, mean, rstd = ctx.saved_tensors
        dx, dw, db = ops.gn_silu_backward(dout, x, weight, bias, mean, rstd, ctx.groups)
        return dx, dw, db, None, None


def gn_silu(x: torch.Tensor, norm) -> torch.Tensor:
    """SiLU(norm(x)) for a GroupNorm `norm` (ContextNet's head_norm + head_act,
    reference models.py:460-466); fused on a HIP device in fp32."""
    fused = (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3
             and isinstance(norm, torch.nn.GroupNorm) and norm.affine
             and x.shape[2] % 4 == 0 and x.shape[1] <= 1024 and x.shape[0] * x.shape[1] < 65536
             and not torch.is_autocast_enabled("cuda"))
    if fused:
        return _GNSiLU.apply(x.contiguous(), norm.weight, norm.bias, int(norm.num_groups),
                             float(norm.eps))
    return torch.nn.functional.silu(norm(x))


def gn_film_residual(x: torch.Tensor, norm, gamma: torch.Tensor, beta: torch.Tensor):
    """x + (norm(x) * (1 + gamma[:, :, None]) + beta[:, :, None]) for a GroupNorm
    `norm` (reference models.py:322-368); fused on a HIP device in fp32."""
    fused = (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3
             and isinstance(norm, torch.nn.GroupNorm) and norm.affine
             and x.shape[2] % 4 == 0 and x.shape[1] <= 1024 and x.shape[0] * x.shape[1] < 65536
             and gamma.dtype == torch.float32 and beta.dtype == torch.float32
             and not torch.is_autocast_enabled("cuda"))
    if fused:
        return _GNFiLMRes.apply(x.contiguous(), norm.weight, norm.bias, gamma, beta,
                                int(norm.num_groups), float(norm.eps))
    y = norm(x)
    return x + (y * (1.0 + gamma[:, :, None]) + beta[:, :, None])


# PCFM_POST_GN_FUSED=0: the PV block's post SharedMLP and GroupNorm-FiLM residual
# as two nodes (the post activation written, its BatchNorm backward statistics a
# separate pass)
_POST_GN_FUSED = __import__("os").environ.get("PCFM_POST_GN_FUSED", "1") != "0"


class _PostGNFiLMRes(torch.autograd.Function):
    """The PV block's tail (models.py:349-368) as one autograd node:
    z = ReLU(BN(Conv1d_1x1(x))) (SharedMLP, shared_mlp.py:15-27), then
    out = z + GroupNorm(z) (1 + gamma) + beta.  z is never written -- the
    GroupNorm kernels compute it from the conv output y as bn_act_forward does,
    bit for bit -- and the GroupNorm backward's apply pass also sums the
    BatchNorm's backward statistics, so of the unfused form's passes the
    BatchNorm apply (read y, write z) and the BatchNorm backward statistics
    (read dL/dz, y) are gone."""

    @staticmethod
    def forward(ctx, x, w, b, g_bn, bt_bn, rm, rv, nbt, eps, momentum, slope, gn_w, gn_b, gamma,
                beta, groups, gn_eps):
        from pcfm import ops
        ys = ops.pointwise_forward_bnstats(x, w, b) if _BN_FROM_GEMM else None
        if ys is not None:
            y, stats = ys
            mean, invstd = ops.bn_forward_stats(y, eps, momentum, rm, rv, nbt, parts=stats)
        else:
            y = ops.pointwise_forward(x, w, b)
            mean, invstd = ops.bn_forward_stats(y, eps, momentum, rm, rv, nbt)
        out, gm, grs = ops.gn_film_res_forward_bnin(y, mean, invstd, g_bn, bt_bn, slope, gn_w,
                                                    gn_b, gamma, beta, groups, gn_eps)
        ctx.save_for_backward(x, w, y, g_bn, bt_bn, mean, invstd, gn_w, gn_b, gamma, gm, grs)
        ctx.slope, ctx.groups, ctx.has_bias = slope, groups, b is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        from pcfm import ops
        x, w, y, g_bn, bt_bn, mean, invstd, gn_w, gn_b, gamma, gm, grs = ctx.saved_tensors
        dz, dgnw, dgnb, dgamma, dbeta, bnpart = ops.gn_film_res_backward_bnin(
            dout, y, mean, invstd, g_bn, bt_bn, ctx.slope, gn_w, gn_b, gamma, gm, grs, ctx.groups)
        dy, dg_bn, db_bn, db = ops.bn_act_backward_parts(dz, y, g_bn, bt_bn, mean, invstd, bnpart,
                                                         ctx.slope, want_dbias_in=ctx.has_bias)
        del dz
        dx = ops.pointwise_backward_data(dy, w) if ctx.needs_input_grad[0] else None
        dw = ops.pointwise_backward_weight(x, dy).view_as(w) if ctx.needs_input_grad[1] else None
        return (dx, dw, db, dg_bn, db_bn, None, None, None, None, None, None, dgnw, dgnb, dgamma,
                dbeta, None, None)


def post_gn_film_residual(post, norm, x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor):
    """z + GroupNorm(z) (1 + gamma) + beta with z = post(x) for a one-layer
    SharedMLP `post` (conv, BN, ReLU) and a GroupNorm `norm`: one fused node on
    the GPU training path (_PostGNFiLMRes), else the two modules' paths."""
    layers = post.layers
    conv, bn = layers[0], layers[1]
    fused = (_POST_GN_FUSED and len(layers) == 3 and isinstance(layers[2], torch.nn.ReLU)
             and x.is_cuda and x.dtype == torch.float32 and x.dim() == 3
             and _fusable_pre(bn) and hasattr(conv, "x3_ok") and conv.x3_ok(x)
             and conv.bias is not None and isinstance(norm, torch.nn.GroupNorm) and norm.affine
             and x.shape[2] % 4 == 0 and conv.out_channels <= 1024
             and x.shape[0] * conv.out_channels < 65536 and x.shape[0] * x.shape[2] > 1
             and conv.out_channels % norm.num_groups == 0
             and gamma.dtype == torch.float32 and beta.dtype == torch.float32)
    if not fused:
        return gn_film_residual(post(x), norm, gamma, beta)
    return _PostGNFiLMRes.apply(
        x.contiguous(), conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean,
        bn.running_var, _nbt(bn), float(bn.eps), float(bn.momentum), 0.0, norm.weight, norm.bias,
        gamma, beta, int(norm.num_groups), float(norm.eps))
