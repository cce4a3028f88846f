"""avg_voxelize: autograd wrapper of the voxelization kernels.

Reference: third_party/pvcnn/modules/functional/voxelization.py:8-40.
"""
from torch.autograd import Function

from modules.functional import backend as _be

# On a HIP device the scatter runs on a shared segment plan (pcfm.plans): the
# second PVConv block of a stage voxelizes the same points with the first
# block's sort.


def _voxelize(feats, vox, r):
    if feats.is_cuda:
        from pcfm import ops, plans
        if plans.ENABLED:
            plan = plans.voxel_plan(vox, r)
            return ops.avg_voxelize_forward_planned(feats, plan), plan.ind, plan.cnt
    return _be._backend.avg_voxelize_forward(feats, vox, r)

__all__ = ["avg_voxelize", "avg_voxelize_tee"]


class AvgVoxelization(Function):
    """features f32 [B, C, N], coords i32 [B, 3, N] -> f32 [B, C, R, R, R]."""

    @staticmethod
    def forward(ctx, features, coords, resolution):
        feats = features.contiguous()
        vox = coords.int().contiguous()
        b, c = feats.shape[0], feats.shape[1]
        r = int(resolution)
        grid, ind, cnt = _voxelize(feats, vox, r)
        ctx.save_for_backward(ind, cnt)
        return grid.view(b, c, r, r, r)

    @staticmethod
    def backward(ctx, grad_output):
        ind, cnt = ctx.saved_tensors
        b, c = grad_output.shape[0], grad_output.shape[1]
        flat = grad_output.contiguous().view(b, c, -1)
        return _be._backend.avg_voxelize_backward(flat, ind, cnt), None, None


avg_voxelize = AvgVoxelization.apply


class AvgVoxelizationTee(Function):
    """(grid, features) from features: the voxelization plus a pass-through of its
    input for PVConv's point branch (pvconv.py:35-39 feeds `features` to both).
    The backward sums the two gradients inside the voxelization's gather
    (pcfm_avg_voxelize_bwd_add) instead of a separate add."""

    @staticmethod
    def forward(ctx, features, coords, resolution):
        feats = features.contiguous()
        vox = coords.int().contiguous()
        b, c = feats.shape[0], feats.shape[1]
        r = int(resolution)
        grid, ind, cnt = _voxelize(feats, vox, r)
        ctx.save_for_backward(ind, cnt)
        return grid.view(b, c, r, r, r), features.view_as(features)

    @staticmethod
    def backward(ctx, grad_grid, grad_feat):
        from pcfm import ops
        ind, cnt = ctx.saved_tensors
        b, c = grad_grid.shape[0], grad_grid.shape[1]
        flat = grad_grid.contiguous().view(b, c, -1)
        if grad_feat is None:
            return _be._backend.avg_voxelize_backward(flat, ind, cnt), None, None
        return ops.avg_voxelize_backward_add(flat, ind, cnt, grad_feat), None, None


avg_voxelize_tee = AvgVoxelizationTee.apply
