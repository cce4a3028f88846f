"""PVConv: point-voxel convolution block.

Reference: third_party/pvcnn/modules/pvconv.py:11-39.  Voxelize (gfx950 scatter
kernel) -> two Conv3d/BN3d/LeakyReLU(0.1) stages (+ SE; the 3x3x3 convs run on
the bf16x3 matrix-core kernels of modules/voxel_conv.py) -> trilinear
devoxelize (gfx950 gather kernel) -> + pointwise SharedMLP branch.  Modules are
created in the reference's order, so a given torch seed yields the same
initial weights, and the state_dict keys (voxel_layers.{0,1,3,4,6.fc.*},
point_features.layers.*) are the reference's.
"""
import torch
import torch.nn as nn
import torch.nn.functional as TF

import modules.functional as F
from modules.norm_act import (_BN_FROM_GEMM, _fusable_pre, _nbt, _pair_head, _pair_tail,
                              conv_bn_act_pair, pair_fusable)
from modules.se import SE3d
from modules.shared_mlp import SharedMLP
from modules.voxel_conv import VoxelConv3d
from modules.voxelization import Voxelization

__all__ = ["PVConv"]


def _conv_bn_lrelu(cin, cout, kernel_size):
    return [
        VoxelConv3d(cin, cout, kernel_size, stride=1, padding=kernel_size // 2),
        nn.BatchNorm3d(cout, eps=1e-4),
        nn.LeakyReLU(0.1, True),
    ]


# SE3d's MLP as one kernel each way (PCFM_SE_FUSED=0: torch ops, A/B knob)
_SE_FUSED = __import__("os").environ.get("PCFM_SE_FUSED", "1") != "0"


def _se_scale(m, w1, w2):
    return torch.sigmoid(TF.linear(TF.relu(TF.linear(m, w1)), w2))


class _SEDevoxAdd(torch.autograd.Function):
    """devox(SE3d(grid)) + point branch in one gather (pcfm_trilinear_devoxelize_
    scale_add_fwd): SE's channel scale is linear in the grid, so it is applied to
    the devoxelized values, and the SE-scaled grid is never materialised.

    Backward: g = devox_bwd(dout); ds = sum_v grid * g (rows_dot) feeds the SE
    MLP's gradient; d grid = s * g + d mean / V in place (rows_affine)."""

    @staticmethod
    def forward(ctx, grid, coords, pf, w1, w2, r, training):
        from pcfm import ops, plans
        b, c = grid.shape[0], grid.shape[1]
        v = grid[0, 0].numel()
        rows = grid.contiguous().view(b * c, v)
        m = ops.rows_dot(rows, None, 1.0 / v).view(b, c)
        w1, w2 = w1.contiguous(), w2.contiguous()
        # the SE MLP as one kernel each way (pcfm_se_mlp_*), torch ops beyond its size
        fused = _SE_FUSED and ops.se_mlp_ok(m, w1)
        if fused:
            s, hid = ops.se_mlp_forward(m, w1, w2)
        else:
            s, hid = _se_scale(m, w1, w2).contiguous(), m.new_empty(0)
        # the corner indices / weights depend on the points only: the second
        # block of a stage reuses the first one's (pcfm.plans) and skips writing
        shared = plans.devox_corners(coords, r) if training else None
        out, inds, wgts = ops.trilinear_devoxelize_scale_add(
            r, training and shared is None, coords, rows.view(b, c, v), s, pf)
        if shared is not None:
            inds, wgts = shared
        elif training:
            plans.put_devox_corners(coords, r, inds, wgts)
        if training:
            ctx.save_for_backward(rows, inds, wgts, m, s, w1, w2, hid)
            ctx.r, ctx.shape, ctx.fused = r, grid.shape, fused
            ctx.points = coords  # key of the shared backward plan (pcfm.plans)
        return out

    @staticmethod
    def backward(ctx, dout):
        from pcfm import ops
        from pcfm import plans
        rows, inds, wgts, m, s, w1, w2, hid = ctx.saved_tensors
        dout = dout.contiguous()
        if plans.ENABLED:
            plan = plans.devox_bwd_plan(ctx.points, inds, wgts, ctx.r)
            g = ops.trilinear_devoxelize_backward_planned(dout, plan).view_as(rows)
        else:
            g = ops.trilinear_devoxelize_backward(dout, inds, wgts, ctx.r).view_as(rows)
        ds = ops.rows_dot(rows, g, 1.0).view_as(s)
        if ctx.fused:  # d mean / V straight out of the MLP backward
            dmv, dw1, dw2 = ops.se_mlp_backward(m, hid, s, ds, w1, w2, 1.0 / rows.shape[1])
        else:
            with torch.enable_grad():
                m_ = m.detach().requires_grad_(True)
                w1_ = w1.detach().requires_grad_(True)
                w2_ = w2.detach().requires_grad_(True)
                dm, dw1, dw2 = torch.autograd.grad(_se_scale(m_, w1_, w2_), [m_, w1_, w2_], ds)
            dmv = (dm / rows.shape[1]).contiguous()
        ops.rows_affine_(g, s.view(-1), dmv.view(-1))
        return g.view(ctx.shape), None, dout, dw1, dw2, None, None


class _VoxelBranchSEDevox(torch.autograd.Function):
    """A PVConv with SE in one autograd node, voxel and point branches:
    devox(SE(act2(BN2(Conv2(act1(BN1(Conv1(grid)))))))) + ReLU(BN(W f + b))
    (pvconv.py:20-39, se.py:6-17, shared_mlp.py:15-27).  Neither act2(BN2(.))
    nor the point branch's ReLU(BN(.)) is ever written: BN2's batch statistics
    and SE's pooling come from one pass over Conv2's output y2
    (bn_act_forward_rowmean), the point branch's statistics from its GEMM's
    epilogue, and the devoxelization applies both BatchNorms + activations as it
    stages its rows and reads its add operand.  Backward from g = devox_bwd(dout):
    one pass over (g, y2) gives SE's ds and every BN2 sum (dz = s g + dm / V is
    linear in s and dm: bn_se_backward_stats), the SE MLP's backward gives dm,
    and the apply pass writes d y2 as Conv2's split operand
    (bn_se_backward_apply_split); the point branch's gradient is dout through
    its BatchNorm + ReLU and GEMM, as _PwBnAct.  Against _Conv3dBnActPair +
    _SEDevoxAdd + _PwBnAct: both activations' writes, both SE rows_dot passes,
    the rows_affine pass and BN2's backward statistics pass are gone."""

    @staticmethod
    def forward(ctx, x, w1, b1, g1, bt1, rm1, rv1, nbt1, w2, b2, g2, bt2, rm2, rv2, nbt2,
                sw1, sw2, coords, f, pw, pb, pg, pbt, prm, prv, pnbt, eps1, mom1, slope1, eps2,
                mom2, slope2, peps, pmom, r, occ=None):
        from pcfm import ops, plans
        # point branch: y_pf = W f + b, its BatchNorm statistics (the GEMM epilogue's
        # when the 256-row tile runs); ReLU(BN(y_pf)) is applied inside the gather
        ys = ops.pointwise_forward_bnstats(f, pw, pb) if _BN_FROM_GEMM else None
        if ys is not None:
            y_pf, parts = ys
        else:
            y_pf, parts = ops.pointwise_forward(f, pw, pb), None
        pm, pis = ops.bn_forward_stats(y_pf, peps, pmom, prm, prv, pnbt, parts=parts)
        xs, y1, m1, is1, z1s, y2 = _pair_head(x, w1, b1, g1, bt1, rm1, rv1, nbt1, w2, b2, eps1,
                                              mom1, slope1, occ)
        mse, m2, is2 = ops.bn_act_forward_rowmean(y2, g2, bt2, eps2, slope2, mom2, rm2, rv2,
                                                  nbt2)
        sw1, sw2 = sw1.contiguous(), sw2.contiguous()
        s, hid = ops.se_mlp_forward(mse, sw1, sw2)
        shared = plans.devox_corners(coords, r)
        out, inds, wgts = ops.trilinear_devoxelize_bn_scale_add(
            r, shared is None, coords, y2, m2, is2, g2, bt2, slope2, s, y_pf,
            add_bn=(pm, pis, pg, pbt, 0.0))
        if shared is not None:
            inds, wgts = shared
        else:
            plans.put_devox_corners(coords, r, inds, wgts)
        ctx.save_for_backward(xs, w1, y1, g1, bt1, m1, is1, z1s, w2, y2, g2, bt2, m2, is2,
                              inds, wgts, mse, s, hid, sw1, sw2, f, pw, y_pf, pg, pbt, pm, pis)
        ctx.points, ctx.r, ctx.occ = coords, r, occ
        ctx.slopes = (slope1, slope2)
        ctx.has_bias = (b1 is not None, b2 is not None, pb is not None)
        ctx.dims = (x.shape[0], x.shape[1], w1.shape[0], w2.shape[0], x.shape[2])
        return out

    @staticmethod
    def backward(ctx, dout):
        from pcfm import ops, plans
        (xs, w1, y1, g1, bt1, m1, is1, z1s, w2, y2, g2, bt2, m2, is2, inds, wgts, mse, s, hid,
         sw1, sw2, f, pw, y_pf, pg, pbt, pm, pis) = ctx.saved_tensors
        dout = dout.contiguous()
        # point branch (_PwBnAct's backward): ReLU + BatchNorm, then the GEMM's
        dy_pf, dpg, dpbt, dpb = ops.bn_act_backward(dout, y_pf, pg, pbt, pm, pis, 0.0,
                                                    want_dbias_in=ctx.has_bias[2])
        df = ops.pointwise_backward_data(dy_pf, pw) if ctx.needs_input_grad[18] else None
        dpw = ops.pointwise_backward_weight(f, dy_pf).view_as(pw)
        del dy_pf
        if plans.ENABLED:
            plan = plans.devox_bwd_plan(ctx.points, inds, wgts, ctx.r)
            g = ops.trilinear_devoxelize_backward_planned(dout, plan)
        else:
            g = ops.trilinear_devoxelize_backward(dout, inds, wgts, ctx.r)
        g = g.view(y2.shape)
        rowstats = ops.bn_se_backward_stats(g, y2, m2, is2, g2, bt2, ctx.slopes[1])
        v = y2[0, 0].numel()
        dmv, dsw1, dsw2 = ops.se_mlp_backward(mse, hid, s, rowstats[0], sw1, sw2, 1.0 / v)
        gys2, dg2, dbt2, db2 = ops.bn_se_backward_apply_split(
            g, y2, m2, is2, g2, bt2, s, dmv, rowstats, ctx.slopes[1],
            want_dbias_in=ctx.has_bias[1])
        del g
        dx, dw1, db1, dg1, dbt1, dw2 = _pair_tail(gys2, xs, w1, y1, g1, bt1, m1, is1, z1s, w2,
                                                  ctx.slopes[0], ctx.has_bias[0], ctx.dims,
                                                  ctx.occ, ctx.needs_input_grad[0])
        return (dx, dw1, db1, dg1, dbt1, None, None, None, dw2, db2, dg2, dbt2, None, None, None,
                dsw1, dsw2, None, df, dpw, dpb, dpg, dpbt, None, None, None, None, None, None,
                None, None, None, None, None, None, None)


# the voxel branch as one node (PCFM_PV_FUSED=0: the conv pair + the SE devoxelization
# as two nodes, the round-4 form; A/B knob)
_PV_FUSED = __import__("os").environ.get("PCFM_PV_FUSED", "1") != "0"


def _point_branch_fusable(layers, x) -> bool:
    """The point branch is one Conv1d(1x1) + BatchNorm1d + ReLU that the fused
    PVConv node can run (the _PwBnAct conditions of modules/norm_act.py)."""
    from modules.shared_mlp import PointwiseConv1d
    if len(layers) != 3 or not isinstance(layers[2], nn.ReLU):
        return False
    conv, bn = layers[0], layers[1]
    return (isinstance(conv, PointwiseConv1d) and isinstance(bn, nn.BatchNorm1d)
            and _fusable_pre(bn) and conv.x3_ok(x) and conv.bias is not None
            and x.shape[2] % 4 == 0 and x.shape[0] * conv.out_channels < 65536
            and x.shape[0] * x.shape[2] > 1)


def _se_fused_ok(b, c, w1) -> bool:
    """The SE MLP fits its one-block kernels (pcfm_se_mlp_fwd / _bwd)."""
    h = w1.shape[0]
    return _SE_FUSED and 2 * (b + h) * c + 2 * b * h <= 32768


def _se_devox_ok(se, grid, pf) -> bool:
    if not (grid.is_cuda and grid.dtype == torch.float32 and pf.dtype == torch.float32
            and isinstance(se, SE3d)):
        return False
    fc = se.fc
    return (len(fc) == 4 and isinstance(fc[0], nn.Linear) and fc[0].bias is None
            and isinstance(fc[1], nn.ReLU) and isinstance(fc[2], nn.Linear)
            and fc[2].bias is None and isinstance(fc[3], nn.Sigmoid)
            and grid[0, 0].numel() % 4 == 0 and not torch.is_autocast_enabled("cuda"))


class PVConv(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, resolution, with_se=False,
                 normalize=True, eps=0):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = kernel_size
        self.resolution = resolution
        self.voxelization = Voxelization(resolution, normalize=normalize, eps=eps)
        stages = _conv_bn_lrelu(in_channels, out_channels, kernel_size)
        stages += _conv_bn_lrelu(out_channels, out_channels, kernel_size)
        if with_se:
            stages.append(SE3d(out_channels))
        self.voxel_layers = nn.Sequential(*stages)
        self.point_features = SharedMLP(in_channels, out_channels)

    def forward(self, inputs):
        features, coords = inputs
        if (features.is_cuda and features.dtype == torch.float32 and features.requires_grad
                and torch.is_grad_enabled()):
            # the point branch reads the tee'd features: its input gradient is added
            # to the voxelization's inside the voxelization's backward gather
            grid, grid_coords, features = self.voxelization.forward_tee(features, coords)
        else:
            grid, grid_coords = self.voxelization(features, coords)
        layers = self.voxel_layers  # Conv3d, BN3d, LeakyReLU, Conv3d, BN3d, LeakyReLU[, SE3d]
        occ = None
        if grid.is_cuda:
            # the first conv's input is the voxelization: exact zeros off the
            # occupied voxels, and its gradient is read back only on them
            from pcfm import plans
            occ = plans.conv_occupancy(self.voxelization._coords(coords)[1], self.resolution)
        pm = self.point_features.layers
        if (_PV_FUSED and self.training and torch.is_grad_enabled() and len(layers) > 6
                and grid.is_cuda and pair_fusable(layers[0], layers[1], layers[3], layers[4], grid)
                and _point_branch_fusable(pm, features)):
            fc = layers[6].fc
            if (_se_devox_ok(layers[6], grid, features) and grid[0, 0].numel() <= 32768
                    and _se_fused_ok(grid.shape[0], layers[3].out_channels, fc[0].weight)):
                c1, n1, c2, n2 = layers[0], layers[1], layers[3], layers[4]
                out = _VoxelBranchSEDevox.apply(
                    grid.contiguous(), c1.weight, c1.bias, n1.weight, n1.bias, n1.running_mean,
                    n1.running_var, _nbt(n1), c2.weight, c2.bias, n2.weight, n2.bias,
                    n2.running_mean, n2.running_var, _nbt(n2), fc[0].weight, fc[2].weight,
                    grid_coords, features.contiguous(), pm[0].weight, pm[0].bias, pm[1].weight,
                    pm[1].bias, pm[1].running_mean, pm[1].running_var, _nbt(pm[1]),
                    float(n1.eps), float(n1.momentum), float(layers[2].negative_slope),
                    float(n2.eps), float(n2.momentum), float(layers[5].negative_slope),
                    float(pm[1].eps), float(pm[1].momentum), self.resolution, occ)
                return out, coords
        pf = None
        grid = conv_bn_act_pair(layers[0], layers[1], layers[2].negative_slope,
                                layers[3], layers[4], layers[5].negative_slope, grid,
                                voxelized_input_occ=occ)
        if pf is None:
            pf = self.point_features(features)
        if (len(layers) > 6 and _se_devox_ok(layers[6], grid, pf)
                and (self.training or not torch.is_grad_enabled())):
            fc = layers[6].fc
            out = _SEDevoxAdd.apply(grid, grid_coords, pf, fc[0].weight, fc[2].weight,
                                    self.resolution, self.training)
            return out, coords
        if len(layers) > 6:
            grid = layers[6](grid)
        voxel_branch = F.trilinear_devoxelize(grid, grid_coords, self.resolution, self.training)
        return voxel_branch + pf, coords
