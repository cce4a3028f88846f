"""Build the torch-extension bindings of the C ABI in-tree, each next to the
Python package that mirrors the reference module it replaces:

    _pvcnn_backend  (csrc/torch_backend.cpp)  -> modules/functional/
    chamfer_3D      (csrc/torch_losses.cpp)   -> chamfer3D/
    emd_cuda        (csrc/torch_losses.cpp)   -> PyTorchEMD/
    emd_ext         (csrc/torch_losses.cpp)   -> PyTorchEMD/  (the reference's
                    extension name, PyTorchEMD/setup.py:26-29, backend.py:11-12)

    python point-cloud-flow-matching_amd/csrc/build_torch_backend.py [--force]

Plain g++ against torch's headers and libraries (no hipify, no device code: the
kernels are libpcfm_hip.so's, linked with an $ORIGIN-relative rpath).  Needs the
library built first (make -C csrc).  Skips a module whose output is newer than
its sources."""
import os
import subprocess
import sys
import sysconfig

import torch
from torch.utils import cpp_extension

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)

# name -> (source, output directory, extra defines)
MODULES = {
    "_pvcnn_backend": ("torch_backend.cpp", os.path.join(PKG, "modules", "functional"), []),
    "chamfer_3D": ("torch_losses.cpp", os.path.join(PKG, "chamfer3D"), ["-DPCFM_TORCH_MODULE=1"]),
    "emd_cuda": ("torch_losses.cpp", os.path.join(PKG, "PyTorchEMD"), ["-DPCFM_TORCH_MODULE=2"]),
    "emd_ext": ("torch_losses.cpp", os.path.join(PKG, "PyTorchEMD"), ["-DPCFM_TORCH_MODULE=2"]),
}


def output_path(name: str = "_pvcnn_backend") -> str:
    return os.path.join(MODULES[name][1], name + sysconfig.get_config_var("EXT_SUFFIX"))


def _command(name: str, force: bool):
    """(g++ command line or None when up to date, output path)"""
    src_name, out_dir, defs = MODULES[name]
    src = os.path.join(HERE, src_name)
    lib = os.path.join(HERE, "libpcfm_hip.so")
    hdr = os.path.join(os.path.dirname(PKG), "include", "pcfm.h")
    out = output_path(name)
    if not os.path.exists(lib):
        raise RuntimeError(f"{lib} missing: run make -C {HERE} first")
    if (not force and os.path.exists(out)
            and os.path.getmtime(out) >= max(os.path.getmtime(p) for p in (src, lib, hdr, __file__))):
        return None, out
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", src, "-o", out, *defs,
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-DTORCH_EXTENSION_NAME={name}",
           "-DTORCH_API_INCLUDE_EXTENSION_H", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           "-I" + sysconfig.get_paths()["include"], "-I/opt/rocm/include"]
    cmd += ["-I" + p for p in cpp_extension.include_paths()]
    for p in cpp_extension.library_paths():
        cmd += ["-L" + p, "-Wl,-rpath," + p]
    rel = os.path.relpath(HERE, out_dir)
    cmd += ["-L" + HERE, "-l:libpcfm_hip.so", f"-Wl,-rpath,$ORIGIN/{rel}",
            "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_python"]
    return cmd, out


def build(force: bool = False) -> list:
    """Compile the modules that are out of date, concurrently (one g++ each)."""
    jobs = [_command(name, force) for name in MODULES]
    procs = [(subprocess.Popen(cmd), cmd) for cmd, _ in jobs if cmd is not None]
    bad = [cmd for p, cmd in procs if p.wait() != 0]
    if bad:
        raise RuntimeError("torch-extension build failed: " + " ".join(bad[0]))
    return [out for _, out in jobs]


if __name__ == "__main__":
    for p in build(force="--force" in sys.argv):
        print(p)
