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
    @staticmethod
    def forward(ctx, x, weight, bias):
        from pcfm import ops
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return ops.conv3d_forward(x, weight, bias)

    @staticmethod
    def backward(ctx, gy):
        from pcfm import ops
        x, weight = ctx.saved_tensors
        gy = gy.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = ops.conv3d_backward_data(gy, weight)
        if ctx.needs_input_grad[1]:
            if ops.conv3d_wgrad_supported(x, weight):
                gw = ops.conv3d_backward_weight(x, gy)
            else:
                gw = torch.nn.grad.conv3d_weight(x, weight.shape, gy, stride=1, padding=1)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = gy.sum(dim=(0, 2, 3, 4))
        return gx, gw, gb


class VoxelConv3d(nn.Conv3d):
    exact_fp32 = False

    def forward(self, x):
        if (self.exact_fp32 or not x.is_cuda or x.dtype != torch.float32
                or self.kernel_size != (3, 3, 3) or self.stride != (1, 1, 1)
                or self.padding != (1, 1, 1) or self.dilation != (1, 1, 1) or self.groups != 1
                or self.padding_mode != "zeros"):
            return super().forward(x)
        from pcfm import ops
        if not ops.conv3d_supported(x, self.weight):
            return super().forward(x)
        return _Conv3dX3.apply(x, self.weight, self.bias)
