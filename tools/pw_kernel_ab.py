"""Kernel-only timing of the pointwise GEMM forms at the C2 shapes (dev tool):
the weight image is prepared once and only pcfm_pointwise_gemm is timed, with
HIP events around 50 back-to-back launches.  PCFM_PW_WST=0/1 picks the 256-row
tile / the weight-stationary form; PCFM_LIB=<variant> loads a measurement build.
One JSON line: python tools/pw_kernel_ab.py TAG"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm import _lib, ops  # noqa: E402

res = {"tag": sys.argv[1] if len(sys.argv) > 1 else "main", "wst": os.environ.get("PCFM_PW_WST", "1")}
g = torch.Generator(device="cuda").manual_seed(0)
for b, ci, co, n in ((8, 256, 256, 20000), (8, 128, 256, 20000)):
    x = torch.randn(b, ci, n, device="cuda", generator=g)
    w = torch.randn(co, ci, 1, device="cuda", generator=g) * ci ** -0.5
    bias = torch.randn(co, device="cuda", generator=g)
    img = ops.pointwise_prep_weight(w, False)
    y = torch.empty(b, co, n, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def launch():
        _lib.call("pcfm_pointwise_gemm", x.data_ptr(), img.data_ptr(), bias.data_ptr(), b, ci, co, n,
                  y.data_ptr(), st)
    for _ in range(5):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(50):
        launch()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    res[f"B{b}Ci{ci}Co{co}N{n}"] = {"fwd_us": round(us, 2),
                                    "TBps_xy": round(4 * b * n * (ci + co) / us / 1e6, 2)}
print(json.dumps(res), flush=True)
