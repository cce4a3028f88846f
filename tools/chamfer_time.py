"""Chamfer forward timing at C2 (8 x 20000 x 20000) and the published shape (dev tool)."""
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
for dist, (b, n, m) in (("randn", (8, 20000, 20000)), ("randn", (32, 2000, 1000)),
                        ("randn", (4, 100000, 100000)), ("rand", (4, 100000, 100000))):
    draw = torch.randn if dist == "randn" else torch.rand
    a = draw(b, n, 3, device="cuda", generator=g)
    c = draw(b, m, 3, device="cuda", generator=g)
    d1, d2 = torch.empty(b, n, device="cuda"), torch.empty(b, m, device="cuda")
    i1 = torch.empty(b, n, dtype=torch.int32, device="cuda")
    i2 = torch.empty(b, m, dtype=torch.int32, device="cuda")
    res[f"{dist}_{b}x{n}x{m}"] = timeit(lambda: ops.chamfer_3D.forward(a, c, d1, d2, i1, i2), it=10)
print(json.dumps(res), flush=True)
