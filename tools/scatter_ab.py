"""A/B timing of the PVConv scatters (voxelize fwd, devoxelize bwd) at the C2
stage shapes (dev tool): PCFM_LIB=<variant> python tools/scatter_ab.py tag"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm import ops  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def main():
    res = {"tag": sys.argv[1] if len(sys.argv) > 1 else "main"}
    g = torch.Generator(device="cuda").manual_seed(0)
    b, n = 8, 20000
    for c, r in ((128, 32), (256, 16), (256, 8)):
        x = torch.randn(b, 3, n, device="cuda", generator=g)
        x = x - x.mean(2, keepdim=True)
        x = x / (x.norm(dim=1, keepdim=True).max(dim=2, keepdim=True).values * 2.0 + 1e-6) + 0.5
        nc = torch.clamp(x * r, 0, r - 1)
        vc = torch.round(nc).to(torch.int32)
        feat = torch.randn(b, c, n, device="cuda", generator=g)
        grid = torch.randn(b, c, r ** 3, device="cuda", generator=g)
        _, inds, wgts = ops.trilinear_devoxelize_forward(r, True, nc, grid)
        vplan = ops.avg_voxelize_plan(vc, r)
        dplan = ops.trilinear_devoxelize_backward_plan(inds, wgts, r)
        sc = torch.rand(b, c, device="cuda", generator=g)
        pf = torch.randn(b, c, n, device="cuda", generator=g)
        cnt = torch.randint(1, 4, (b, r ** 3), device="cuda", generator=g, dtype=torch.int32)
        ind = torch.randint(0, r ** 3, (b, n), device="cuda", generator=g, dtype=torch.int32)
        res[f"C{c}R{r}"] = {
            "devox_fwd_scale_add_ms": timeit(
                lambda: ops.trilinear_devoxelize_scale_add(r, True, nc, grid, sc, pf)),
            "vox_bwd_add_ms": timeit(lambda: ops.avg_voxelize_backward_add(grid, ind, cnt, pf)),
            "vox_fwd_ms": timeit(lambda: ops.avg_voxelize_forward(feat, vc, r)),
            "devox_bwd_ms": timeit(lambda: ops.trilinear_devoxelize_backward(feat, inds, wgts, r)),
            "vox_fwd_planned_ms": timeit(lambda: ops.avg_voxelize_forward_planned(feat, vplan)),
            "devox_bwd_planned_ms": timeit(
                lambda: ops.trilinear_devoxelize_backward_planned(feat, dplan))}
        if os.environ.get("SCATTER_SAVE"):  # outputs for a bitwise comparison across variants
            OUT[f"C{c}R{r}"] = (ops.avg_voxelize_forward_planned(feat, vplan).cpu(),
                                ops.trilinear_devoxelize_backward_planned(feat, dplan).cpu(),
                                ops.trilinear_devoxelize_scale_add(r, True, nc, grid, sc, pf)[0].cpu(),
                                ops.avg_voxelize_backward_add(grid, ind, cnt, pf).cpu())
    if os.environ.get("SCATTER_SAVE"):
        path = os.environ["SCATTER_SAVE"]
        if os.path.exists(path):
            ref = torch.load(path, weights_only=True)
            res["bit_equal_to_saved"] = all(torch.equal(a, b) for k in OUT
                                            for a, b in zip(OUT[k], ref[k]))
        else:
            torch.save(OUT, path)
    print(json.dumps(res), flush=True)


OUT = {}


if __name__ == "__main__":
    main()
