"""Time conv3d wgrad at the PVConv shapes (dev tool; run with PCFM_LIB variants)."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm import ops  # noqa: E402

for b, c, r in [(8, 128, 32), (8, 256, 16), (8, 256, 8)]:
    x = torch.randn(b, c, r, r, r, device="cuda")
    gy = torch.randn(b, c, r, r, r, device="cuda")
    for _ in range(2):
        ops.conv3d_backward_weight(x, gy)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        ops.conv3d_backward_weight(x, gy)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 100
    print(os.environ.get("PCFM_LIB", "default").split("/")[-1], f"C{c}R{r} wgrad {ms:.3f} ms "
          f"{2 * b * r ** 3 * c * c * 27 / ms / 1e9:.0f} TF", flush=True)
