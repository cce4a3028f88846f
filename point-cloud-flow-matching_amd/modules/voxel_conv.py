"""PVConv's voxel convolution, nn.Conv3d(C_in, C_out, 3, stride=1, padding=1)
(third_party/pvcnn/modules/pvconv.py:20-24), on the MI355X matrix cores.

`VoxelConv3d` keeps nn.Conv3d's parameters (same state_dict keys) and routes
the forward and the input gradient through pcfm's bf16x3 implicit GEMM
(include/pcfm.h, csrc/conv3d.hip): every fp32 operand is split into two bf16
terms and the three significant products are accumulated in fp32, ~2^-16
relative error per product -- tighter than the TF32 arithmetic cuDNN applies
to the reference's fp32 Conv3d by default (torch.backends.cudnn.allow_tf32).
The weight gradient is the same split GEMM over voxels.  Shapes the kernel
does not cover, or a module switched to `exact_fp32 = True`, use nn.Conv3d's
own (MIOpen fp32) path.
"""
import torch
import torch.nn as nn

__all__ = ["VoxelConv3d"]


class _Conv3dX3(torch.autograd.Function):
    """Forward keeps split(x) (channels-last bf16 hi/lo, the GEMM's B operand)
    instead of x; the backward splits dY once and uses it for both the
    backward-data GEMM and the weight gradient."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        from pcfm import ops
        x = x.contiguous()
        b, cin, r = x.shape[0], x.shape[1], x.shape[2]
        cout = weight.shape[0]
        xs = ops.conv3d_split(x)
        y = ops.conv3d_igemm_split(xs, ops.conv3d_prep_weight(weight, False), bias, b, cin, cout,
                                   r, "conv3d_fwd")
        ctx.save_for_backward(xs, weight)
        ctx.has_bias = bias is not None
        ctx.dims = (b, cin, cout, r)
        return y

    @staticmethod
    def backward(ctx, gy):
        from pcfm import ops
        xs, weight = ctx.saved_tensors
        b, cin, cout, r = ctx.dims
        gys = ops.conv3d_split(gy.contiguous())
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = ops.conv3d_igemm_split(gys, ops.conv3d_prep_weight(weight, True), None, b, cout,
                                        cin, r, "conv3d_bwd_data")
        if ctx.needs_input_grad[1]:
            gw = ops.conv3d_wgrad_split(xs, gys, b, cin, cout, r)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = gy.sum(dim=(0, 2, 3, 4))
        return gx, gw, gb


class VoxelConv3d(nn.Conv3d):
    exact_fp32 = False

    def x3_ok(self, x) -> bool:
        """True if forward(x) runs on the bf16x3 implicit GEMM."""
        if (self.exact_fp32 or not x.is_cuda or x.dtype != torch.float32
                or self.kernel_size != (3, 3, 3) or self.stride != (1, 1, 1)
                or self.padding != (1, 1, 1) or self.dilation != (1, 1, 1) or self.groups != 1
                or self.padding_mode != "zeros" or torch.is_autocast_enabled("cuda")):
            return False
        from pcfm import ops
        return ops.conv3d_supported(x, self.weight) and ops.conv3d_wgrad_supported(x, self.weight)

    def forward(self, x):
        if not self.x3_ok(x):
            return super().forward(x)
        return _Conv3dX3.apply(x, self.weight, self.bias)
