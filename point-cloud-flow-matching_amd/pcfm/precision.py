"""Arithmetic of the fp32 convolutions.

By default the PVConv Conv3d and the SharedMLP / head 1x1 Conv1d run on the
bf16x3 matrix-core kernels (modules/voxel_conv.py, modules/shared_mlp.py:
~2^-16 relative error per product -- tighter than the TF32 that cuDNN applies
to the reference's fp32 convolutions on H100).
`exact_fp32()` switches them to true fp32 arithmetic (MIOpen / hipBLASLt fp32,
TF32 disabled) for parity work: with it, the hybrid velocity and the train
step's losses match the reference's fp32 CPU execution within 1e-5 relative
(tests/test_gpu_model.py, tests/test_gpu_train_golden.py).  Every other
kernel on the path (voxelization, devoxelization, BatchNorm / GroupNorm
fusions, Chamfer, EMD) is fp32 in both modes.
"""
from __future__ import annotations

import contextlib

import torch

__all__ = ["exact_fp32", "set_exact_fp32", "is_exact_fp32"]


def _classes():
    from modules.shared_mlp import PointwiseConv1d
    from modules.voxel_conv import VoxelConv3d
    return VoxelConv3d, PointwiseConv1d


def set_exact_fp32(flag: bool) -> None:
    """Process-wide: fp32 convolutions on exact fp32 arithmetic (True) or on the
    bf16x3 matrix-core kernels (False, the default).  True also turns TF32 off."""
    for cls in _classes():
        cls.exact_fp32 = bool(flag)
    if flag:
        torch.backends.cuda.matmul.allow_tf32 = False
        torch.backends.cudnn.allow_tf32 = False


def is_exact_fp32() -> bool:
    return all(cls.exact_fp32 for cls in _classes())


@contextlib.contextmanager
def exact_fp32(flag: bool = True):
    """Scope in which the fp32 convolutions use exact fp32 arithmetic."""
    classes = _classes()
    old = ([cls.exact_fp32 for cls in classes], torch.backends.cuda.matmul.allow_tf32,
           torch.backends.cudnn.allow_tf32)
    set_exact_fp32(flag)
    try:
        yield
    finally:
        for cls, v in zip(classes, old[0]):
            cls.exact_fp32 = v
        torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32 = old[1], old[2]
