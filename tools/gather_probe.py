"""Time the LDS-staged gathers (devox fwd with SE scale + add, voxelize bwd with
add) at the PVConv shapes; PCFM_GATHER_BLOCKS overrides the block target (dev)."""
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


tag = os.environ.get("PCFM_GATHER_BLOCKS", "default")
b, n = 8, 20000
g = torch.Generator(device="cuda").manual_seed(0)
coords = torch.rand(b, 3, n, device="cuda", generator=g)
for c, r in [(128, 32), (256, 16), (256, 8)]:
    grid = torch.randn(b, c, r * r * r, device="cuda", generator=g)
    pf = torch.randn(b, c, n, device="cuda", generator=g)
    s = torch.rand(b, c, device="cuda", generator=g)
    cf = coords * (r - 1)
    vox = torch.round(cf).int()
    _, ind, cnt = ops.avg_voxelize_forward(pf, vox, r)
    t1 = timeit(lambda: ops.trilinear_devoxelize_scale_add(r, True, cf, grid, s, pf))
    t2 = timeit(lambda: ops.avg_voxelize_backward_add(grid, ind, cnt, pf))
    print(f"[{tag}] C{c}R{r}: devox fwd+SE+add {t1 * 1e3:.1f} us, vox bwd+add {t2 * 1e3:.1f} us",
          flush=True)
