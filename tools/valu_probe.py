"""Which VALU instruction classes return wrong results beside MFMA waves?
(tools/valu_probe.hip.)  For each aggressor (none,
conv3_wgrad3, pw_gemm256) loop it on a side stream from a Python thread and run
the probe kernel for every instruction class on the default stream; print one
JSON line per (aggressor, class) with the wrong-result counts per quarter wave.
The probe never dereferences what it computes, so wrong values cannot fault.

Build (CPU): hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/valu_probe.hip
             -o tools/libvalu_probe.so
Usage (GPU box): python tools/valu_probe.py [seconds per class] [aggressors,...]
                 [LDS bytes per probe block] [classes,...]"""
import ctypes
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import torch  # noqa: E402

from pcfm import ops  # noqa: E402

CLASSES = ["v_fma_f32", "v_pk_fma_f32", "v_lshl_add_u64", "v_mad_u64_u32", "v_add_co_u32+addc",
           "v_fma_f64"]
lib = ctypes.CDLL(os.path.join(REPO, "tools", "libvalu_probe.so"))
lib.valu_probe_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.c_int, ctypes.c_void_p]

seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
aggs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["none", "conv_wgrad", "pointwise"]
lds = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # bytes of LDS each probe block reserves
classes = [int(c) for c in sys.argv[4].split(",")] if len(sys.argv) > 4 else range(len(CLASSES))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)


def aggressor(name):
    if name == "pointwise":
        x = torch.randn(8, 256, 20000, device=dev, generator=g)
        w = torch.randn(256, 256, device=dev, generator=g) * 0.05
        return lambda: ops.pointwise_forward(x, w, None)
    if name == "conv_wgrad":
        xs = ops.conv3d_split(torch.randn(8, 256, 16, 16, 16, device=dev, generator=g))
        return lambda: ops.conv3d_wgrad_split(xs, xs, 8, 256, 256, 16)
    return None


for name in aggs:
    fn = aggressor(name)
    torch.cuda.synchronize(dev)
    stop = threading.Event()
    launched = [0]

    def run_side():
        side = torch.cuda.Stream(dev)
        with torch.cuda.stream(side):
            while not stop.is_set():
                fn()
                launched[0] += 1
                if launched[0] % 20 == 0:
                    side.synchronize()
            side.synchronize()

    th = threading.Thread(target=run_side, daemon=True) if fn is not None else None
    if th is not None:
        th.start()
    try:
        for cls in classes:
            cname = CLASSES[cls]
            bad = torch.zeros(len(CLASSES) * 4, dtype=torch.int64, device=dev)
            stream = torch.cuda.current_stream(dev).cuda_stream
            t0, n = time.time(), 0
            while time.time() - t0 < seconds:
                rc = lib.valu_probe_launch(cls, 1024, 4000, ctypes.c_void_p(bad.data_ptr()), lds,
                                           ctypes.c_void_p(stream))
                if rc != 0:
                    raise RuntimeError(f"valu_probe_launch: {rc}")
                n += 1
                if n % 8 == 0:
                    torch.cuda.synchronize(dev)
            torch.cuda.synchronize(dev)
            q = bad.view(len(CLASSES), 4)[cls].tolist()
            print(json.dumps({"aggressor": name, "class": cname, "launches": n,
                              "evaluations": n * 1024 * 256 * 4000, "wrong_by_quarter": q,
                              "aggressor_launches": launched[0], "lds": lds}), flush=True)
    finally:
        stop.set()
        if th is not None:
            th.join()
        torch.cuda.synchronize(dev)
