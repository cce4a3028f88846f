"""The native backend behind `modules.functional` (reference:
third_party/pvcnn/modules/functional/backend.py, which JIT-builds the CUDA
module `_pvcnn_backend` at import time).

Here `_backend` is the prebuilt gfx950 library bound through the C ABI
(pcfm.ops.backend); nothing is compiled at import.  Each function runs the
HIP kernels for tensors on a HIP device and the pure-PyTorch CPU backend
(pcfm.cpu_ops) for CPU tensors.  The functional wrappers look
`_backend` up on this module at call time, so a test may substitute another
object with the same function names (the CPU oracle does this in tests/ only).

`_torch_backend` is the same C ABI bound the reference's way: a torch C++
extension module `_pvcnn_backend` exporting the 12 names of its bindings.cpp
(csrc/torch_backend.cpp, built in-tree by __graft_entry__.build()), HIP tensors
only; None when it has not been built.  PCFM_TORCH_BACKEND=1 makes `_backend` the
extension for HIP tensors, with CPU tensors still sent to the pure-PyTorch
backend (pcfm.ops.host_routed).
"""
import os

from pcfm.ops import backend as _backend
from pcfm.ops import host_routed

try:
    from modules.functional import _pvcnn_backend as _torch_backend
except ImportError:  # not built (build_torch_backend.py)
    _torch_backend = None

if os.environ.get("PCFM_TORCH_BACKEND") == "1":
    if _torch_backend is None:
        raise ImportError("PCFM_TORCH_BACKEND=1 but modules/functional/_pvcnn_backend is not built "
                          "(python point-cloud-flow-matching_amd/csrc/build_torch_backend.py)")
    _backend = host_routed(_torch_backend, _backend,
                           [n for n in dir(_torch_backend) if not n.startswith("_")])

__all__ = ["_backend", "_torch_backend"]
