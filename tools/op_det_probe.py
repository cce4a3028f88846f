"""Dev probe: bitwise reproducibility of each PVConv-path op at the stage-2/3
shapes (C 256, R 16 / 8, B 8, N 20000) over repeated calls; run two copies
at once to put the GPU under contention.  Prints {op, r, mismatching_calls}."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import torch  # noqa: E402

from pcfm import _lib, ops  # noqa: E402


def main():
    _lib.load()
    reps = int(os.environ.get("REPS", "30"))
    b, n, c = 8, 20000, 256
    g = torch.Generator(device="cuda").manual_seed(0)
    pts = torch.randn(b, 3, n, device="cuda", generator=g)
    feats = torch.randn(b, c, n, device="cuda", generator=g)
    for r in (16, 8):
        c0 = pts - pts.mean(2, keepdim=True)
        unit = c0 / (2 * c0.norm(dim=1, keepdim=True).max(2, keepdim=True).values + 1e-6) + 0.5
        norm = torch.clamp(unit * r, 0, r - 1).contiguous()
        vox = torch.round(norm).int().contiguous()
        w = torch.randn(c, c, 3, 3, 3, device="cuda", generator=g) * 0.02
        bias = torch.randn(c, device="cuda", generator=g)
        gamma = torch.rand(c, device="cuda", generator=g) + 0.5
        beta = torch.randn(c, device="cuda", generator=g)
        img = ops.conv3d_prep_weight(w, False)
        s = torch.rand(b, c, device="cuda", generator=g)

        def f_plan():
            p = ops.avg_voxelize_plan(vox, r)
            return [p.ind, p.cnt]

        plan = ops.avg_voxelize_plan(vox, r)

        def f_vox():
            return [ops.avg_voxelize_forward_planned(feats, plan)]

        grid = ops.avg_voxelize_forward_planned(feats, plan).view(b, c, r, r, r).contiguous()

        def f_split():
            return [ops.conv3d_split(grid)]

        xs = ops.conv3d_split(grid)

        def f_conv():
            return [ops.conv3d_igemm_split(xs, img, bias, b, c, c, r, "x")]

        y = ops.conv3d_igemm_split(xs, img, bias, b, c, c, r, "x")

        def f_bn():
            z, m, i = ops.bn_act_forward(y, gamma, beta, 1e-4, 0.1, 0.1, None, None, None)
            return [z, m, i]

        def f_bn_split():
            z, m, i = ops.bn_act_forward_split(y, gamma, beta, 1e-4, 0.1, 0.1, None, None, None)
            return [z, m, i]

        rows = y.view(b * c, -1)

        def f_rowsdot():
            return [ops.rows_dot(rows, None, 1.0)]

        def f_devox():
            out, inds, wgts = ops.trilinear_devoxelize_scale_add(r, True, norm, y.view(b, c, -1),
                                                                 s, feats)
            return [out, inds, wgts]

        for name, fn in (("voxel_plan", f_plan), ("avg_voxelize_fwd", f_vox),
                         ("conv3d_split", f_split), ("conv3d_fwd", f_conv), ("bn_act_fwd", f_bn),
                         ("bn_act_fwd_split", f_bn_split), ("rows_dot", f_rowsdot),
                         ("devox_scale_add", f_devox)):
            ref = [t.clone() for t in fn()]
            bad = 0
            for _ in range(reps):
                got = fn()
                if not all(torch.equal(a, c_) for a, c_ in zip(ref, got)):
                    bad += 1
            torch.cuda.synchronize()
            print(json.dumps({"op": name, "r": r, "mismatching_calls": bad, "of": reps}),
                  flush=True)


if __name__ == "__main__":
    main()
