"""grouping: gather neighbour features, with a scatter-add backward.

Reference: third_party/pvcnn/modules/functional/grouping.py:8-31.
"""
from torch.autograd import Function

from modules.functional import backend as _be

__all__ = ["grouping"]


class Grouping(Function):
    """features f32 [B, C, N], indices i32 [B, M, U] -> f32 [B, C, M, U]."""

    @staticmethod
    def forward(ctx, features, indices):
        feats = features.contiguous()
        idx = indices.contiguous()
        ctx.save_for_backward(idx)
        ctx.num_points = feats.shape[-1]
        return _be._backend.grouping_forward(feats, idx)

    @staticmethod
    def backward(ctx, grad_output):
        (idx,) = ctx.saved_tensors
        g = _be._backend.grouping_backward(grad_output.contiguous(), idx, ctx.num_points)
        return g, None


grouping = Grouping.apply
