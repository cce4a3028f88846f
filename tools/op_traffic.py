"""HBM traffic per launch of the four PVConv voxel ops and the three voxel-conv
GEMMs (forward, backward-data, weight gradient; split operands as the train
step runs them) at the bench's stage
shapes, from rocprofv3 PMC counters (MI355X_MICROARCH.md, HBM section).

Two passes, one counter each (FETCH_SIZE and WRITE_SIZE cannot share a pass):

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT/fetch -o t -- python tools/op_traffic.py run
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d OUT/write -o t -- python tools/op_traffic.py run
    python tools/op_traffic.py summarize OUT/fetch OUT/write > profiles/r01_traffic.json

`run` executes, per stage (C, R) of the bench's ContextNet, each op K times,
separated by a marker kernel (torch.cumsum on a tiny tensor).  It also runs a
calibration copy of known bytes through seg_transpose (4-B-per-lane loads, the
access width of the voxel kernels): FETCH_SIZE is scaled by
known_bytes / FETCH_SIZE(calibration) before it is reported (the guide: gfx950
FETCH_SIZE under-reports wide reads; calibrate on your own access pattern).
Both counters are reported by rocprofv3 in KiB; they are converted to bytes.
Dev tool: not part of the product.
"""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

B, N, K = 8, 20000, 5
STAGES = [(128, 32), (256, 16), (256, 8)]
OPS = ["avg_voxelize_fwd", "avg_voxelize_bwd", "trilinear_devoxelize_fwd",
       "trilinear_devoxelize_bwd", "conv3d_fwd", "conv3d_bwd_data", "conv3d_wgrad"]


def run():
    import torch
    from pcfm import ops

    def marker():
        torch.cumsum(torch.ones(3, device="cuda"), 0)

    g = torch.Generator(device="cuda").manual_seed(0)
    for c, r in STAGES:
        x = torch.randn(B, 3, N, device="cuda", generator=g)
        x = x - x.mean(2, keepdim=True)
        x = x / (x.norm(dim=1, keepdim=True).max(dim=2, keepdim=True).values * 2.0 + 1e-6) + 0.5
        nc = torch.clamp(x * r, 0, r - 1)
        vc = torch.round(nc).to(torch.int32)
        feat = torch.randn(B, c, N, device="cuda", generator=g)
        grid = torch.randn(B, c, r ** 3, device="cuda", generator=g)
        _, ind, cnt = ops.avg_voxelize_forward(feat, vc, r)
        _, inds, wgts = ops.trilinear_devoxelize_forward(r, True, nc, grid)
        vg = torch.randn(B, c, r, r, r, device="cuda", generator=g)
        wt = torch.randn(c, c, 3, 3, 3, device="cuda", generator=g) * (1.0 / (27 * c) ** 0.5)
        xs, gys = ops.conv3d_split(vg), ops.conv3d_split(vg * 0.5)
        img_f, img_b = ops.conv3d_prep_weight(wt, False), ops.conv3d_prep_weight(wt, True)
        calls = {
            "conv3d_fwd": lambda: ops.conv3d_igemm_split(xs, img_f, None, B, c, c, r, "f"),
            "conv3d_bwd_data": lambda: ops.conv3d_igemm_split(gys, img_b, None, B, c, c, r, "b"),
            "conv3d_wgrad": lambda: ops.conv3d_wgrad_split(xs, gys, B, c, c, r),
            "avg_voxelize_fwd": lambda: ops.avg_voxelize_forward(feat, vc, r),
            "avg_voxelize_bwd": lambda: ops.avg_voxelize_backward(grid, ind, cnt),
            "trilinear_devoxelize_fwd": lambda: ops.trilinear_devoxelize_forward(r, True, nc, grid),
            "trilinear_devoxelize_bwd": lambda: ops.trilinear_devoxelize_backward(feat, inds, wgts,
                                                                                  r),
        }
        for name in OPS:
            calls[name]()
            torch.cuda.synchronize()
            marker()
            for _ in range(K):
                calls[name]()
            marker()
            torch.cuda.synchronize()


def _rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))))
    out = []
    for r in rows:  # FETCH_SIZE / WRITE_SIZE are reported in KiB
        out.append((r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0, r["Counter_Name"]))
    return out


def _segments(rows):
    """Split the dispatch list at marker kernels; return the K-call segments in order."""
    segs, cur, inside = [], [], False
    for name, val, _ in rows:
        if "scan" in name.lower() and "pcfm" not in name:
            if inside:
                segs.append(cur)
            cur, inside = [], not inside
            continue
        if inside:
            cur.append((name, val))
    return segs


def summarize(dfetch, dwrite):
    fetch, write = _segments(_rows(dfetch)), _segments(_rows(dwrite))
    # calibration: seg_rows (the channels-last copy of the segment sum) reads the
    # (B, C, N) input once: B*C*N*4 bytes per launch (+ small rank/key arrays)
    labels = [(c, r, op) for c, r in STAGES for op in OPS]
    res, calib = {}, []
    for (c, r, op), fs, ws in zip(labels, fetch, write):
        for name, val in fs:
            if "seg_rows" in name:
                calib.append(B * c * N * 4 / val)
    corr = sum(calib) / len(calib) if calib else 2.0
    for (c, r, op), fs, ws in zip(labels, fetch, write):
        fb = sum(v for _, v in fs) / K * corr
        wb = sum(v for _, v in ws) / K
        res[f"{op}@C{c}R{r}"] = {"fetch_bytes": fb, "write_bytes": wb, "traffic_bytes": fb + wb}
    return {"batch": B, "points": N,
            "fetch_correction": corr, "calibration": "seg_rows reads B*C*N*4 bytes",
            "shapes": f"B={B} N={N} randn coords through Voxelization normalisation",
            "ops": res}


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        print(json.dumps(summarize(sys.argv[2], sys.argv[3]), indent=1))
