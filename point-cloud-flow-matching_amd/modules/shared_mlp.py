"""SharedMLP: a stack of pointwise (1x1) conv + BatchNorm + ReLU.

Reference: third_party/pvcnn/modules/shared_mlp.py:6-33.  Parameter names
(layers.{3k}, layers.{3k+1}) match, so reference checkpoints load unchanged.

The 1x1 Conv1d is evaluated as what it is, a GEMM over the channel axis
(y[b] = W x[b] + bias).  On the GPU in fp32 (the reference runs these layers
with autocast off, models.py:512-513) it goes through pcfm's bf16x3
matrix-core GEMMs (csrc/pointwise.hip; ~2^-16 relative error per product,
tighter than the TF32 cuDNN uses for the reference's Conv1d by default);
under autocast it stays a batched GEMM so torch's autocast casting applies.
"""
import torch
import torch.nn as nn

from modules.norm_act import conv_bn_act

__all__ = ["SharedMLP", "PointwiseConv1d"]


class _PointwiseX3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        from pcfm import ops
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return ops.pointwise_forward(x, weight, bias)

    @staticmethod
    def backward(ctx, gy):
        from pcfm import ops
        x, weight = ctx.saved_tensors
        gy = gy.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = ops.pointwise_backward_data(gy, weight)
        if ctx.needs_input_grad[1]:
            gw = ops.pointwise_backward_weight(x, gy).view_as(weight)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            # row sums on the rows kernel (torch's sum over dims (0, 2) of a
            # (8, 64, 20000) gradient ran at 0.8 TB/s), then over the batch
            bb, cc, nn_ = gy.shape
            gb = ops.rows_dot(gy.view(bb * cc, nn_), None, 1.0).view(bb, cc).sum(0)
        return gx, gw, gb


class PointwiseConv1d(nn.Conv1d):
    """nn.Conv1d(in, out, 1) whose forward is a channel GEMM (same parameters)."""

    exact_fp32 = False

    def _is_1x1(self) -> bool:
        return (self.kernel_size == (1,) and self.groups == 1 and self.stride == (1,)
                and self.padding in ((0,), "valid") and self.dilation == (1,))

    def x3_ok(self, x) -> bool:
        """True if forward(x) runs on the bf16x3 pointwise GEMM."""
        return (self._is_1x1() and x.dim() == 3 and x.is_cuda and x.dtype == torch.float32
                and self.weight.dtype == torch.float32 and not self.exact_fp32
                and not torch.is_autocast_enabled("cuda"))

    def forward(self, x):
        if not self._is_1x1() or x.dim() != 3:
            return super().forward(x)
        if self.x3_ok(x):
            return _PointwiseX3.apply(x, self.weight, self.bias)
        # bmm against the batch-broadcast weight: the result is a contiguous
        # (B, C_out, N) tensor (torch.matmul(2-D, 3-D) returns a transposed view,
        # which turns every following BatchNorm/ReLU/add into a strided kernel),
        # and the bias is folded into the GEMM's C operand.
        w = self.weight[:, :, 0].unsqueeze(0).expand(x.shape[0], -1, -1)
        if self.bias is None:
            return torch.bmm(w, x)
        return torch.baddbmm(self.bias[None, :, None], w, x)


_KINDS = {1: (PointwiseConv1d, nn.BatchNorm1d), 2: (nn.Conv2d, nn.BatchNorm2d)}


class SharedMLP(nn.Module):
    def __init__(self, in_channels, out_channels, dim=1):
        super().__init__()
        if dim not in _KINDS:
            raise ValueError(f"SharedMLP: dim must be 1 or 2, got {dim}")
        conv, norm = _KINDS[dim]
        widths = list(out_channels) if isinstance(out_channels, (list, tuple)) else [out_channels]
        stack = []
        prev = in_channels
        for w in widths:
            stack += [conv(prev, w, 1), norm(w), nn.ReLU(True)]
            prev = w
        self.layers = nn.Sequential(*stack)

    def _run(self, x):
        # (conv, BN, ReLU) triples; BN + ReLU fused on the GPU (modules/norm_act.py)
        layers = self.layers
        for i in range(0, len(layers), 3):
            x = conv_bn_act(layers[i], layers[i + 1], x, 0.0)
        return x

    def forward(self, inputs):
        # (features, coords, ...) tuples pass the trailing items through untouched
        if isinstance(inputs, (list, tuple)):
            return (self._run(inputs[0]), *inputs[1:])
        return self._run(inputs)
