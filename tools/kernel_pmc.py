"""Matrix-core / VALU / LDS counters of the dominant kernels (rocprofv3 --pmc),
north_star's "MFMA-busy counters against gfx950 peak" and SURVEY.md 8d
"Counters".

    python tools/kernel_pmc.py run          # the workload (each op K times)
    rocprofv3 --kernel-trace --pmc <counters> --output-format csv -d OUT/<pass> -o t \
        -- python tools/kernel_pmc.py run   # one pass per counter set (tools/kernel_pmc.sh)
    python tools/kernel_pmc.py summarize OUT/<pass> ... > profiles/rNN_kernel_pmc.json

Workload (B = 8, N = 20000 where it applies -- the C2 train step's shapes):
  conv3d fwd / bwd-data / wgrad at C128 R32, C256 R16 and C256 R8 (split
  operands, as the step runs them), the devoxelization forward, the pointwise
  GEMMs, the EMD forward, Chamfer forward at C2 (8 x 20000 x 20000), ball query at C5
  (4 x 100000 points, 4096 centers, U = 32).
Derived per kernel: MFMA-pipe busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (1024
SIMDs x GRBM_GUI_ACTIVE / 8) (GRBM_GUI_ACTIVE is summed over the 8 XCDs;
MI355X_MICROARCH.md), and the same cycles divided by 32 per
v_mfma_f32_32x32x16_bf16 against the kernel's algorithmic MFMA count.
Dev tool: not part of the product.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

K = 3
SIMDS = 1024


def run():
    import torch
    from pcfm import ops
    g = torch.Generator(device="cuda").manual_seed(0)
    b = 8
    for c, r in ((128, 32), (256, 16), (256, 8)):
        x = torch.randn(b, c, r, r, r, device="cuda", generator=g)
        w = torch.randn(c, c, 3, 3, 3, device="cuda", generator=g) * (1.0 / (27 * c) ** 0.5)
        xs, gys = ops.conv3d_split(x), ops.conv3d_split(x * 0.5)
        img_f, img_b = ops.conv3d_prep_weight(w, False), ops.conv3d_prep_weight(w, True)
        for _ in range(K):
            ops.conv3d_igemm_split(xs, img_f, None, b, c, c, r, "f")
            ops.conv3d_igemm_split(gys, img_b, None, b, c, c, r, "b")
            ops.conv3d_wgrad_split(xs, gys, b, c, c, r)
        torch.cuda.synchronize()
    for c, r in ((128, 32), (256, 16)):  # devoxelization forward (SE scale + point add)
        x = torch.rand(b, 3, 20000, device="cuda", generator=g) * (r - 1)
        grid = torch.randn(b, c, r ** 3, device="cuda", generator=g)
        sc = torch.rand(b, c, device="cuda", generator=g)
        pf = torch.randn(b, c, 20000, device="cuda", generator=g)
        for _ in range(K):
            ops.trilinear_devoxelize_scale_add(r, True, x, grid, sc, pf)
        torch.cuda.synchronize()
    for ci, co in ((256, 256), (128, 256)):  # SharedMLP 1x1 convs, fwd / bwd-data / wgrad
        x = torch.randn(b, ci, 20000, device="cuda", generator=g)
        w = torch.randn(co, ci, 1, device="cuda", generator=g) * ci ** -0.5
        dy = torch.randn(b, co, 20000, device="cuda", generator=g)
        for _ in range(K):
            ops.pointwise_forward(x, w, None)
            ops.pointwise_backward_data(dy, w)
            ops.pointwise_backward_weight(x, dy)
        torch.cuda.synchronize()
    e1 = torch.rand(8, 2048, 3, device="cuda", generator=g)
    e2 = torch.rand(8, 2048, 3, device="cuda", generator=g)
    for _ in range(K):  # EMD forward at the bench size (exp-bound VALU)
        ops.approxmatch_cost_forward(e1, e2)
    torch.cuda.synchronize()
    a = torch.randn(8, 20000, 3, device="cuda", generator=g)
    p = torch.randn(8, 20000, 3, device="cuda", generator=g)
    d1, d2 = torch.empty(8, 20000, device="cuda"), torch.empty(8, 20000, device="cuda")
    i1 = torch.empty(8, 20000, dtype=torch.int32, device="cuda")
    i2 = torch.empty(8, 20000, dtype=torch.int32, device="cuda")
    for _ in range(K):
        ops.chamfer_3D.forward(a, p, d1, d2, i1, i2)
    torch.cuda.synchronize()
    pts = torch.rand(4, 3, 100000, device="cuda", generator=g)
    ctr = torch.rand(4, 3, 4096, device="cuda", generator=g)
    for _ in range(K):
        ops.ball_query(ctr, pts, 0.05, 32)
    torch.cuda.synchronize()


def _load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def summarize(dirs):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    for d in dirs:
        disp = defaultdict(dict)
        for r in _load(d):
            key = (r["Kernel_Name"], r.get("Dispatch_Id", r.get("Correlation_Id")))
            disp[key][r["Counter_Name"]] = disp[key].get(r["Counter_Name"], 0.0) + float(
                r["Counter_Value"])
        for (name, _), cs in disp.items():
            for cn, v in cs.items():
                per[name][cn].append(v)
    out = {}
    for name, cs in per.items():
        short = name.replace("(anonymous namespace)::", "").split("(")[0][-90:]
        avg = {cn: sum(v) / len(v) for cn, v in cs.items()}
        entry = {"dispatches": max(len(v) for v in cs.values()), "mean_per_dispatch": avg}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and avg.get("GRBM_GUI_ACTIVE"):
            entry["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (
                SIMDS * avg["GRBM_GUI_ACTIVE"] / 8.0)
            entry["mfma_32x32x16_equiv"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / 32.0
        if "SQ_LDS_BANK_CONFLICT" in avg and avg.get("SQ_LDS_IDX_ACTIVE"):
            entry["lds_conflict_frac"] = avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"]
        out[short] = entry
    return {"workload": "tools/kernel_pmc.py run (conv3d C128R32/C256R16/C256R8 B=8 split "
                        "operands; devox fwd C128R32/C256R16; pointwise 256->256 / 128->256 at "
                        "B=8 N=20000; EMD fwd B=8 N=2048; Chamfer fwd 8x20000x20000; ball query "
                        "4x100000, M=4096, U=32)",
            "derivation": "mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 * GRBM_GUI_ACTIVE / 8)",
            "kernels": out}


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        print(json.dumps(summarize(sys.argv[2:]), indent=1))
