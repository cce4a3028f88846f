"""The native backend behind `modules.functional` (reference:
third_party/pvcnn/modules/functional/backend.py, which JIT-builds the CUDA
module `_pvcnn_backend` at import time).

Here `_backend` is the prebuilt gfx950 library bound through the C ABI
(pcfm.ops.backend); nothing is compiled at import.  Each function runs the
HIP kernels for tensors on a HIP device and the pure-PyTorch CPU backend
(pcfm.cpu_ops) for CPU tensors.  The functional wrappers look
`_backend` up on this module at call time, so a test may substitute another
object with the same function names (the CPU oracle does this in tests/ only).
"""
from pcfm.ops import backend as _backend

__all__ = ["_backend"]
