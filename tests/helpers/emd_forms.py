"""Subprocess of tests/test_gpu_ops.py::test_emd_rowpass_form_matches_split_form: runs
approxmatch on a fixed set of shapes under the PCFM_EMD_FORM the parent set,
saves the match matrices to argv[1] (.npz) and
the mean launch time at B=8, N=M=2048 (the metric's EMD size) to argv[2]."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

CASES = [("f32", 8, 2048, 2048), ("f32", 3, 1000, 333), ("f32", 2, 77, 300),
         ("f64", 2, 500, 500), ("f32", 1, 5000, 4999), ("f32", 4, 1, 64)]


def main():
    from pcfm import _lib, ops
    _lib.load()
    out = {}
    for k, (dt, b, n, m) in enumerate(CASES):
        g = torch.Generator(device="cuda").manual_seed(k)
        dtype = torch.float32 if dt == "f32" else torch.float64
        a = torch.rand(b, n, 3, device="cuda", generator=g, dtype=dtype)
        c = torch.rand(b, m, 3, device="cuda", generator=g, dtype=dtype)
        out[f"case{k}"] = ops.approxmatch_forward(a, c).cpu().numpy()
    np.savez(sys.argv[1], **out)
    g = torch.Generator(device="cuda").manual_seed(0)
    a = torch.rand(8, 2048, 3, device="cuda", generator=g)
    c = torch.rand(8, 2048, 3, device="cuda", generator=g)
    for _ in range(3):
        ops.approxmatch_forward(a, c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        ops.approxmatch_forward(a, c)
    e1.record()
    torch.cuda.synchronize()
    json.dump({"approxmatch_ms_b8_n2048": e0.elapsed_time(e1) / reps,
               "form": os.environ.get("PCFM_EMD_FORM", "rowpass")}, open(sys.argv[2], "w"))


if __name__ == "__main__":
    main()
