"""Grid-tail probe of the 256-row pointwise GEMM (dev tool): forward and
backward-data time at B = 8 and point counts whose 128-point tile grid fills a
whole number of two-blocks-per-CU rounds (512 blocks) or not.  Time per
block-round shows whether the last, partly filled round costs a full one."""
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
b, ci, co = 8, 256, 256
w = torch.randn(co, ci, 1, device="cuda", generator=g) * ci ** -0.5
bias = torch.randn(co, device="cuda", generator=g)
for n in (8192, 12288, 16384, 18432, 20000, 20480, 24576):
    x = torch.randn(b, ci, n, device="cuda", generator=g)
    blocks = b * ((n + 127) // 128)
    f = timeit(lambda: ops.pointwise_forward(x, w, bias))
    d = timeit(lambda: ops.pointwise_backward_data(x, w))
    res[str(n)] = {"blocks": blocks, "rounds": blocks / 512.0, "fwd_ms": f, "bwd_data_ms": d,
                   "fwd_TBps": 2 * x.numel() * 4 / f / 1e9}
# the M <= 128 streaming form (pw_stream128) at N = 20000, with a shared bias
for ci, co in ((128, 128), (256, 128), (64, 128)):
    w2 = torch.randn(co, ci, 1, device="cuda", generator=g) * ci ** -0.5
    b2 = torch.randn(co, device="cuda", generator=g)
    x = torch.randn(b, ci, 20000, device="cuda", generator=g)
    dy = torch.randn(b, co, 20000, device="cuda", generator=g)
    res[f"s{ci}to{co}"] = {"fwd_ms": timeit(lambda: ops.pointwise_forward(x, w2, b2)),
                           "bwd_data_ms": timeit(lambda: ops.pointwise_backward_data(dy, w2))}
print(json.dumps(res), flush=True)
