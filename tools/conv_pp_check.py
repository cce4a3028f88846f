"""Dev check: the voxel-conv GEMM outputs at the PVConv stage shapes (forward,
backward-data, occupancy-masked) saved to argv[1] (torch.save), and per-shape
timings; run once with PCFM_CONV_PP=0 and once with 1, then compare the files
(`python tools/conv_pp_check.py --compare a.pt b.pt`)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import torch  # noqa: E402


def run(path):
    from pcfm import _lib, ops
    _lib.load()
    out = {}
    for (b, cin, cout, r) in ((8, 128, 128, 32), (8, 256, 256, 16), (8, 128, 256, 16),
                              (2, 128, 128, 32), (8, 256, 256, 8)):
        g = torch.Generator(device="cuda").manual_seed(b + cin + r)
        x = torch.randn(b, cin, r, r, r, device="cuda", generator=g)
        x[:, :, : r // 2] = 0.0  # empty half: masks skip taps / tiles
        xs = ops.conv3d_split(x)
        w = torch.randn(cout, cin, 3, 3, 3, device="cuda", generator=g) * 0.05
        bias = torch.randn(cout, device="cuda", generator=g)
        img = ops.conv3d_prep_weight(w, False)
        cnt = (x.abs().sum(1) > 0).int().view(b, -1).contiguous()
        occ = ops.conv3d_occupancy(cnt, r)
        key = f"b{b}_c{cin}x{cout}_r{r}"

        def f():
            return ops.conv3d_igemm_split(xs, img, bias, b, cin, cout, r, "x")
        out[key + "_fwd"] = f().cpu()
        if occ is not None:
            out[key + "_fwd_occ"] = ops.conv3d_igemm_split(xs, img, bias, b, cin, cout, r, "x",
                                                           occ=occ, occ_mode=1).cpu()
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        flops = 2.0 * b * r ** 3 * 27 * cin * cout
        print(json.dumps({"shape": key, "ms": ms, "tflops_fp32eq": flops / ms / 1e9,
                          "frac_of_833": flops / ms / 1e9 / 833.3}), flush=True)
        if cin % 128 == 0:
            dy = torch.randn(b, cout, r, r, r, device="cuda", generator=g)
            gys = ops.conv3d_split(dy)
            imgt = ops.conv3d_prep_weight(w, True)
            out[key + "_bwd"] = ops.conv3d_igemm_split(gys, imgt, None, b, cout, cin, r, "x").cpu()
    torch.save(out, path)


def compare(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    res = {k: float((A[k].double() - B[k].double()).abs().max() / A[k].double().pow(2).mean().sqrt())
           for k in A}
    print(json.dumps({"all_equal": all(v == 0.0 for v in res.values()),
                      "max_rel_to_rms": max(res.values()), "cases": res}))
    return max(res.values()) < 1e-5


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    run(sys.argv[1])
