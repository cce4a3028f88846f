"""Time the bf16x3 pointwise GEMMs vs torch fp32 bmm at the ContextNet shapes (dev tool)."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm import ops  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / iters


B, N = 8, 20000
for cin, cout in [(262, 128), (128, 256), (256, 256), (128, 128), (896, 256), (256, 64)]:
    x = torch.randn(B, cin, N, device="cuda")
    w = torch.randn(cout, cin, 1, device="cuda")
    gy = torch.randn(B, cout, N, device="cuda")
    wb = w[:, :, 0].unsqueeze(0).expand(B, -1, -1)
    flop = 2 * B * N * cin * cout
    t = [timeit(lambda: ops.pointwise_forward(x, w, None)),
         timeit(lambda: ops.pointwise_backward_data(gy, w)),
         timeit(lambda: ops.pointwise_backward_weight(x, gy)),
         timeit(lambda: torch.bmm(wb, x)),
         timeit(lambda: torch.bmm(wb.transpose(1, 2), gy)),
         timeit(lambda: torch.bmm(gy, x.transpose(1, 2)).sum(0))]
    print(f"{cin}->{cout}: x3 fwd/bd/wg " + " ".join(f"{v:.3f}" for v in t[:3]) +
          " ms | fp32 bmm " + " ".join(f"{v:.3f}" for v in t[3:]) +
          f" ms | x3 total {sum(t[:3]):.3f} vs {sum(t[3:]):.3f} ms ({3 * flop / sum(t[:3]) / 1e9:.0f}"
          f" vs {3 * flop / sum(t[3:]) / 1e9:.0f} TF)", flush=True)
