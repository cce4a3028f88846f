"""Probe: the four voxel ops at the train-step shapes, for uniform coordinates
vs the concentrated coordinates the flow model produces (randn points through
Voxelization's normalisation).  Dev tool, not part of the product."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm import ops  # noqa: E402

B, N = 8, 20000
STAGES = [(128, 32), (256, 16), (256, 8)]


def norm_coords(kind, r, g):
    if kind == "uniform":
        return torch.rand(B, 3, N, device="cuda", generator=g) * (r - 1)
    x = torch.randn(B, 3, N, device="cuda", generator=g)
    x = x - x.mean(2, keepdim=True)
    x = x / (x.norm(dim=1, keepdim=True).max(dim=2, keepdim=True).values * 2.0 + 1e-6) + 0.5
    return torch.clamp(x * r, 0, r - 1)


def t(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6 / iters


g = torch.Generator(device="cuda").manual_seed(0)
for kind in ("uniform", "randn"):
    for c, r in STAGES:
        nc = norm_coords(kind, r, g)
        vc = torch.round(nc).to(torch.int32)
        feat = torch.randn(B, c, N, device="cuda", generator=g)
        grid = torch.randn(B, c, r ** 3, device="cuda", generator=g)
        out, ind, cnt = ops.avg_voxelize_forward(feat, vc, r)
        o, inds, wgts = ops.trilinear_devoxelize_forward(r, True, nc, grid)
        res = {
            "vox_fwd": t(lambda: ops.avg_voxelize_forward(feat, vc, r)),
            "vox_bwd": t(lambda: ops.avg_voxelize_backward(grid, ind, cnt)),
            "devox_fwd": t(lambda: ops.trilinear_devoxelize_forward(r, True, nc, grid)),
            "devox_bwd": t(lambda: ops.trilinear_devoxelize_backward(feat, inds, wgts, r)),
            "max_pts_per_voxel": int(cnt.max()), "occupied": int((cnt > 0).sum()) // B,
        }
        print(kind, f"C{c}R{r}", {k: (round(v, 1) if isinstance(v, float) else v)
                                  for k, v in res.items()}, flush=True)
