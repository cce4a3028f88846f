"""A/B timing of the voxel-conv GEMMs at the C2 stage shapes (dev tool).

    PCFM_LIB=<variant .so> python tools/conv_ab.py [tag]   -> one JSON line

Times conv3d fwd (split operands), bwd-data and wgrad at C128 R32 and C256 R16
(B = 8) with HIP events over 20 launches each, after 3 warm-ups."""
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


res = {"tag": sys.argv[1] if len(sys.argv) > 1 else os.environ.get("PCFM_LIB", "main")}
OUT = {}
g = torch.Generator(device="cuda").manual_seed(0)
b = 8
for c, r in ((128, 32), (256, 16), (256, 8)):
    x = torch.randn(b, c, r, r, r, device="cuda", generator=g)
    w = torch.randn(c, c, 3, 3, 3, device="cuda", generator=g) * (1.0 / (27 * c) ** 0.5)
    xs, gys = ops.conv3d_split(x), ops.conv3d_split(x * 0.5)
    img_f, img_b = ops.conv3d_prep_weight(w, False), ops.conv3d_prep_weight(w, True)
    flops = 2.0 * b * r ** 3 * 27 * c * c
    tf = timeit(lambda: ops.conv3d_igemm_split(xs, img_f, None, b, c, c, r, "f"))
    tw = timeit(lambda: ops.conv3d_wgrad_split(xs, gys, b, c, c, r))
    # correctness guard: the variant must agree with the exact fp32 conv
    y = ops.conv3d_igemm_split(xs, img_f, None, b, c, c, r, "f")
    ref = torch.nn.functional.conv3d(x, w, padding=1)
    err = float((y - ref).abs().max() / ref.abs().max())
    # the weight gradient (small) and a 1/64 sample of the forward output
    OUT[f"C{c}R{r}"] = (y.flatten()[::64].cpu(), ops.conv3d_wgrad_split(xs, gys, b, c, c, r).cpu())
    res[f"C{c}R{r}"] = {"fwd_ms": tf, "wgrad_ms": tw, "fwd_TF_fp32eq": flops / tf / 1e9,
                        "wgrad_TF_fp32eq": flops / tw / 1e9, "fwd_rel_err": err}
save = os.environ.get("CONV_SAVE")  # outputs for a bitwise comparison across variants
if save:
    if os.path.exists(save):
        ref = torch.load(save, weights_only=True)
        res["bit_equal_to_saved"] = all(torch.equal(a, c) for k in OUT for a, c in zip(OUT[k], ref[k]))
    else:
        torch.save(OUT, save)
print(json.dumps(res), flush=True)
