"""A/B timing of the pointwise (1x1 conv) bf16x3 GEMMs at the C2 train-step
shapes (dev tool): PCFM_LIB=<variant> python tools/pw_ab.py tag"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm import ops  # noqa: E402
from tools.scatter_ab import timeit  # noqa: E402

OUT = {}
res = {"tag": sys.argv[1] if len(sys.argv) > 1 else "main"}
g = torch.Generator(device="cuda").manual_seed(0)
for b, ci, co, n in ((8, 256, 256, 20000), (8, 128, 256, 20000), (8, 128, 128, 20000)):
    x = torch.randn(b, ci, n, device="cuda", generator=g)
    w = torch.randn(co, ci, 1, device="cuda", generator=g) * ci ** -0.5
    bias = torch.randn(co, device="cuda", generator=g)
    dy = torch.randn(b, co, n, device="cuda", generator=g)
    res[f"B{b}Ci{ci}Co{co}N{n}"] = {
        "fwd_ms": timeit(lambda: ops.pointwise_forward(x, w, bias)),
        "bwd_data_ms": timeit(lambda: ops.pointwise_backward_data(dy, w)),
        "wgrad_ms": timeit(lambda: ops.pointwise_backward_weight(x, dy))}
    OUT[f"B{b}Ci{ci}Co{co}N{n}"] = (ops.pointwise_forward(x, w, bias).cpu(),
                                    ops.pointwise_backward_data(dy, w).cpu())
save = os.environ.get("PW_SAVE")  # outputs for a bitwise comparison across variants
if save:
    if os.path.exists(save):
        ref = torch.load(save, weights_only=True)
        res["bit_equal_to_saved"] = all(torch.equal(a, c) for k in OUT for a, c in zip(OUT[k], ref[k]))
    else:
        torch.save(OUT, save)
print(json.dumps(res), flush=True)
