"""Dev probe: is trilinear_devoxelize_scale_add (the SE-scaled devoxelization
+ point-branch add, csrc/rows.hpp gather_rows_kernel) bitwise reproducible on
fixed inputs?  Runs it ITERS times per C2 stage shape and compares every
output with the first call's; on a mismatch reports which output, how many
elements and where.  Run two copies at once to put the GPU under contention.
Also runs the plain devoxelization and the voxelization backward gather the
same way (same kernel template).  JSON lines."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import torch  # noqa: E402

from pcfm import ops  # noqa: E402


def where(a, c):
    d = (a != c)
    if a.is_floating_point():
        d = d & ~(torch.isnan(a) & torch.isnan(c))
    idx = d.nonzero()
    return {"n_diff": int(d.sum()), "first": idx[:6].tolist(),
            "max_abs": float((a.double() - c.double()).abs().max()) if a.is_floating_point()
            else None, "last": idx[-3:].tolist()}


def main():
    dev = torch.device("cuda", 0)
    iters = int(os.environ.get("ITERS", "200"))
    b, n = int(os.environ.get("B", "8")), int(os.environ.get("N", "4096"))
    g = torch.Generator(device=dev).manual_seed(int(os.environ.get("SEED", "0")))
    for c, r in ((128, 32), (256, 16), (256, 8)):
        x = torch.randn(b, 3, n, device=dev, generator=g)
        x = x - x.mean(2, keepdim=True)
        x = x / (x.norm(dim=1, keepdim=True).max(dim=2, keepdim=True).values * 2.0 + 1e-6) + 0.5
        nc = torch.clamp(x * r, 0, r - 1).contiguous()
        grid = torch.randn(b, c, r ** 3, device=dev, generator=g)
        s = torch.rand(b, c, device=dev, generator=g)
        pf = torch.randn(b, c, n, device=dev, generator=g)
        cnt = torch.randint(1, 4, (b, r ** 3), device=dev, generator=g, dtype=torch.int32)
        ind = torch.randint(0, r ** 3, (b, n), device=dev, generator=g, dtype=torch.int32)
        cases = {
            "scale_add_train": lambda: ops.trilinear_devoxelize_scale_add(r, True, nc, grid, s, pf),
            "scale_add_eval": lambda: ops.trilinear_devoxelize_scale_add(r, False, nc, grid, s, pf)[:1],
            "devox_fwd": lambda: ops.trilinear_devoxelize_forward(r, True, nc, grid),
            "vox_bwd_add": lambda: [ops.avg_voxelize_backward_add(grid, ind, cnt, pf)],
        }
        for name, fn in cases.items():
            ref = [t.clone() for t in fn()]
            torch.cuda.synchronize()
            bad = []
            for it in range(iters):
                out = fn()
                for k, (a, o) in enumerate(zip(ref, out)):
                    if not torch.equal(a, o):
                        bad.append({"iter": it, "output": k, **where(a, o)})
                if len(bad) >= 4:
                    break
            torch.cuda.synchronize()
            print(json.dumps({"shape": f"C{c}R{r}", "case": name, "iters": iters,
                              "mismatches": len(bad), "first": bad[:4]}), flush=True)


if __name__ == "__main__":
    main()
