"""Time the voxel-conv forward at the PVConv shapes (dev tool)."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm import ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / iters


for b, c, r in [(8, 128, 32), (8, 256, 16), (8, 256, 8)]:
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(b, c, r, r, r, device="cuda", generator=g)
    w = torch.randn(c, c, 3, 3, 3, device="cuda", generator=g)
    xs = ops.conv3d_split(x)
    img = ops.conv3d_prep_weight(w, False)
    flop = 2 * b * r ** 3 * c * c * 27
    tf = timeit(lambda: ops.conv3d_igemm_split(xs, img, None, b, c, c, r, "fwd"))
    print(f"C{c}R{r}: fwd {tf:.3f} ms ({flop / tf / 1e9:.0f} TF fp32-equiv)", flush=True)
