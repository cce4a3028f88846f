"""The EMD extension module (drop-in for third_party/PyTorchEMD/backend.py,
which JIT-builds `emd_ext` from cuda/emd.cpp + emd_kernel.cu at import and
exports it as `emd_cuda_dynamic`, backend.py:11-24).

Here `emd_ext` is prebuilt in-tree by __graft_entry__.build()
(csrc/build_torch_backend.py: csrc/torch_losses.cpp over libpcfm_hip.so, no
compile at import); HIP tensors only.  The same module also exists as
`PyTorchEMD.emd_cuda`.  Importing this file without the built extension raises
ImportError, as the reference's import does when its build fails."""
from PyTorchEMD import emd_ext as emd_cuda_dynamic  # noqa: F401

__all__ = ["emd_cuda_dynamic"]
