"""trilinear_devoxelize: autograd wrapper of the devoxelization kernels.

Reference: third_party/pvcnn/modules/functional/devoxelization.py:8-42.
"""
from torch.autograd import Function

from modules.functional import backend as _be

__all__ = ["trilinear_devoxelize"]


class TrilinearDevoxelization(Function):
    """features f32 [B, C, R, R, R], coords f32 [B, 3, N] in [0, R-1] -> f32 [B, C, N]."""

    @staticmethod
    def forward(ctx, features, coords, resolution, is_training=True):
        b, c = features.shape[0], features.shape[1]
        grid = features.contiguous().view(b, c, -1)
        r = int(resolution)
        outs, inds, wgts = _be._backend.trilinear_devoxelize_forward(
            r, bool(is_training), coords.contiguous(), grid)
        if is_training:
            ctx.save_for_backward(inds, wgts)
            ctx.r = r
        return outs

    @staticmethod
    def backward(ctx, grad_output):
        inds, wgts = ctx.saved_tensors
        r = ctx.r
        g = _be._backend.trilinear_devoxelize_backward(grad_output.contiguous(), inds, wgts, r)
        return g.view(grad_output.shape[0], grad_output.shape[1], r, r, r), None, None, None


trilinear_devoxelize = TrilinearDevoxelization.apply
