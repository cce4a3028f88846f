"""Approximate Earth Mover's Distance (drop-in for third_party/PyTorchEMD/emd.py).

`emd_cuda` is the native module (approxmatch_forward / matchcost_forward /
matchcost_backward, PyTorchEMD/cuda/emd.cpp:8-27) on the gfx950 library; float
and double inputs are both supported, like the reference's
AT_DISPATCH_FLOATING_TYPES.  CPU tensors run the pure-PyTorch backend
(pcfm.cpu_ops) where the reference asserts "Only support cuda currently."
(emd.py:13).  PCFM_TORCH_BACKEND=1 selects the torch C++ extension
`PyTorchEMD/emd_ext*.so` (csrc/torch_losses.cpp; the reference's extension name,
backend.py:11-12) as `emd_cuda` for HIP tensors, CPU tensors still going to the
CPU backend; the forward keeps the fused match + cost call.
"""
import os

import torch

from pcfm.ops import approxmatch_cost_forward

from pcfm.ops import emd_cuda

if os.environ.get("PCFM_TORCH_BACKEND") == "1":
    from PyTorchEMD.backend import emd_cuda_dynamic as _ext  # the torch-extension module
    from pcfm.ops import host_routed
    emd_cuda = host_routed(_ext, emd_cuda,
                           ["approxmatch_forward", "matchcost_forward", "matchcost_backward"])

__all__ = ["emd_cuda", "EarthMoverDistanceFunction", "earth_mover_distance"]


class EarthMoverDistanceFunction(torch.autograd.Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, xyz1, xyz2):
        xyz1 = xyz1.contiguous()
        xyz2 = xyz2.contiguous()
        # approxmatch + matchcost in one native call; match is kept only when a
        # gradient will need it (emd.py:14-19 computes both, then saves match)
        need = any(ctx.needs_input_grad)
        match, cost = approxmatch_cost_forward(xyz1, xyz2, want_match=need)
        ctx.save_for_backward(xyz1, xyz2, match if need else None)
        return cost

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, grad_cost):
        xyz1, xyz2, match = ctx.saved_tensors
        g1, g2 = emd_cuda.matchcost_backward(grad_cost.contiguous(), xyz1, xyz2, match)
        return g1, g2


def earth_mover_distance(xyz1, xyz2, transpose=True):
    """EMD (approx) per batch element, divided by the number of points of xyz1.

    xyz1, xyz2: (B, 3, N) if transpose else (B, N, 3); 2-D inputs get a batch
    dimension.  Returns cost (B,).  Reference: PyTorchEMD/emd.py:27-51.
    """
    if xyz1.dim() == 2:
        xyz1 = xyz1.unsqueeze(0)
    if xyz2.dim() == 2:
        xyz2 = xyz2.unsqueeze(0)
    if transpose:
        xyz1 = xyz1.transpose(1, 2)
        xyz2 = xyz2.transpose(1, 2)
    assert xyz1.shape[-1] == 3, f"require it to be B,N,3; get: {xyz1.shape}"
    return EarthMoverDistanceFunction.apply(xyz1, xyz2) / float(xyz1.shape[1])
