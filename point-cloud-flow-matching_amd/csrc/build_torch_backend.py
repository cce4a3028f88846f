"""Build the torch-extension binding `_pvcnn_backend` (csrc/torch_backend.cpp)
in-tree, next to modules/functional/backend.py:

    python point-cloud-flow-matching_amd/csrc/build_torch_backend.py

Plain g++ against torch's headers and libraries (no hipify, no device code: the
kernels are libpcfm_hip.so's, linked with an $ORIGIN-relative rpath).  Needs the
library built first (make -C csrc).  Skips the compile when the output is newer
than its sources."""
import os
import subprocess
import sys
import sysconfig

import torch
from torch.utils import cpp_extension

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
OUT_DIR = os.path.join(PKG, "modules", "functional")
NAME = "_pvcnn_backend"


def output_path() -> str:
    return os.path.join(OUT_DIR, NAME + sysconfig.get_config_var("EXT_SUFFIX"))


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "torch_backend.cpp")
    lib = os.path.join(HERE, "libpcfm_hip.so")
    hdr = os.path.join(os.path.dirname(PKG), "include", "pcfm.h")
    out = output_path()
    if not os.path.exists(lib):
        raise RuntimeError(f"{lib} missing: run make -C {HERE} first")
    if (not force and os.path.exists(out)
            and os.path.getmtime(out) >= max(os.path.getmtime(p) for p in (src, lib, hdr, __file__))):
        return out
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", src, "-o", out,
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-DTORCH_EXTENSION_NAME={NAME}",
           "-DTORCH_API_INCLUDE_EXTENSION_H", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           "-I" + sysconfig.get_paths()["include"], "-I/opt/rocm/include"]
    cmd += ["-I" + p for p in cpp_extension.include_paths()]
    for p in cpp_extension.library_paths():
        cmd += ["-L" + p, "-Wl,-rpath," + p]
    rel = os.path.relpath(HERE, OUT_DIR)
    cmd += ["-L" + HERE, "-l:libpcfm_hip.so", f"-Wl,-rpath,$ORIGIN/{rel}",
            "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_python"]
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
