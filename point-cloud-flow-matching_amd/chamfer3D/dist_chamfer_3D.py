"""Chamfer-3D distance (drop-in for
third_party/ChamferDistancePytorch/chamfer3D/dist_chamfer_3D.py).

`chamfer_3D` is the native module (forward/backward write caller-allocated
tensors and return 1 on success, 0 on failure, like chamfer_cuda.cpp:17-32);
the autograd Function allocates its outputs directly on the device instead of
the reference's CPU torch.zeros + .to(device) round trip (:53-63, :77-81).
By default `chamfer_3D` is the ctypes binding (pcfm.ops.chamfer_3D, which also
runs CPU tensors); PCFM_TORCH_BACKEND=1 selects the torch C++ extension
`chamfer3D/chamfer_3D*.so` (csrc/torch_losses.cpp) for HIP tensors, CPU
tensors still going to the ctypes binding's CPU backend.
"""
import os

import torch
from torch import nn
from torch.autograd import Function

from pcfm.ops import chamfer_3D

if os.environ.get("PCFM_TORCH_BACKEND") == "1":
    from chamfer3D import chamfer_3D as _ext  # the torch-extension module
    from pcfm.ops import host_routed
    chamfer_3D = host_routed(_ext, chamfer_3D, ["forward", "backward"])

__all__ = ["chamfer_3D", "chamfer_3DFunction", "chamfer_3DDist", "chamfer_3DFunction_noGrad",
           "chamfer_3DDist_nograd"]


def _outputs(xyz1, xyz2):
    b, n, d1 = xyz1.shape
    _, m, d2 = xyz2.shape
    assert d1 == 3 and d2 == 3, \
        "Wrong last dimension for the chamfer distance 's input! Check with .size()"
    dev = xyz1.device
    return (torch.empty(b, n, device=dev), torch.empty(b, m, device=dev),
            torch.empty(b, n, dtype=torch.int32, device=dev),
            torch.empty(b, m, dtype=torch.int32, device=dev))


def _run_forward(xyz1, xyz2):
    dist1, dist2, idx1, idx2 = _outputs(xyz1, xyz2)
    if not chamfer_3D.forward(xyz1, xyz2, dist1, dist2, idx1, idx2):
        raise RuntimeError("chamfer_3D.forward failed")
    return dist1, dist2, idx1, idx2


class chamfer_3DFunction(Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, xyz1, xyz2):
        dist1, dist2, idx1, idx2 = _run_forward(xyz1, xyz2)
        ctx.save_for_backward(xyz1, xyz2, idx1, idx2)
        ctx.mark_non_differentiable(idx1, idx2)
        return dist1, dist2, idx1, idx2

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, graddist1, graddist2, gradidx1, gradidx2):
        xyz1, xyz2, idx1, idx2 = ctx.saved_tensors
        g1 = torch.zeros_like(xyz1)
        g2 = torch.zeros_like(xyz2)
        ok = chamfer_3D.backward(xyz1, xyz2, g1, g2, graddist1.contiguous(),
                                 graddist2.contiguous(), idx1, idx2)
        if not ok:
            raise RuntimeError("chamfer_3D.backward failed")
        return g1, g2


class chamfer_3DDist(nn.Module):
    def forward(self, input1, input2):
        return chamfer_3DFunction.apply(input1.contiguous(), input2.contiguous())


class chamfer_3DFunction_noGrad(Function):
    @staticmethod
    def forward(ctx, xyz1, xyz2):
        return _run_forward(xyz1, xyz2)


class chamfer_3DDist_nograd(nn.Module):
    def forward(self, input1, input2):
        return chamfer_3DFunction_noGrad.apply(input1.contiguous(), input2.contiguous())
