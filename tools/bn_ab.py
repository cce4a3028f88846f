"""A/B timing of the fused BatchNorm + activation passes at the C2 train-step
shapes (dev tool): PCFM_LIB=<variant> python tools/bn_ab.py tag"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm import ops  # noqa: E402
from tools.scatter_ab import timeit  # noqa: E402

res = {"tag": sys.argv[1] if len(sys.argv) > 1 else "main"}
g = torch.Generator(device="cuda").manual_seed(0)
for b, c, s in ((8, 256, 20000), (8, 128, 20000), (8, 128, 32768), (8, 256, 4096)):
    x = torch.randn(b, c, s, device="cuda", generator=g)
    dz = torch.randn(b, c, s, device="cuda", generator=g)
    gm = torch.rand(c, device="cuda", generator=g) + 0.5
    bt = torch.randn(c, device="cuda", generator=g) * 0.1
    rm, rv = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
    _, mean, invstd = ops.bn_act_forward(x, gm, bt, 1e-5, 0.0, 0.1, rm, rv)
    res[f"B{b}C{c}S{s}"] = {
        "fwd_ms": timeit(lambda: ops.bn_act_forward(x, gm, bt, 1e-5, 0.0, 0.1, rm, rv)),
        "bwd_ms": timeit(lambda: ops.bn_act_backward(dz, x, gm, bt, mean, invstd, 0.0,
                                                     want_dbias_in=True))}
print(json.dumps(res), flush=True)
