"""Probe: Conv3d 3x3x3 fp32 fwd+bwd time per backend/layout at the PVConv shapes
(B=8; C=128@32^3, C=256@16^3, C=256@8^3).  Dev tool, not part of the product.

    python tools/conv3d_probe.py [variant ...]
variants: default, cl3d (channels_last_3d), bench (cudnn.benchmark), nocudnn
(PyTorch's native vol2col + GEMM path); a "+bf16" suffix runs the same in bf16
and "+cl3d" adds channels_last_3d to any variant.
"""
import sys
import time

import torch

SHAPES = [(8, 128, 32), (8, 256, 16), (8, 256, 8)]


def run(variant, iters=5):
    base = variant.split("+")[0]
    dt = torch.bfloat16 if "+bf16" in variant else torch.float32
    cl = base == "cl3d" or "+cl3d" in variant
    torch.backends.cudnn.enabled = base != "nocudnn"
    torch.backends.cudnn.benchmark = base == "bench"
    torch.backends.cudnn.allow_tf32 = False
    res = {}
    for b, c, r in SHAPES:
        conv = torch.nn.Conv3d(c, c, 3, padding=1).cuda().to(dt)
        x = torch.randn(b, c, r, r, r, device="cuda", dtype=dt, requires_grad=True)
        if cl:
            conv = conv.to(memory_format=torch.channels_last_3d)
            x = x.detach().to(memory_format=torch.channels_last_3d).requires_grad_(True)
        gy = torch.randn(b, c, r, r, r, device="cuda", dtype=dt)
        if cl:
            gy = gy.to(memory_format=torch.channels_last_3d)
        t = {}
        for phase in ("fwd", "fwd_bwd"):
            for i in range(iters + 2):
                if i == 2:
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                y = conv(x)
                if phase == "fwd_bwd":
                    y.backward(gy)
            torch.cuda.synchronize()
            t[phase] = (time.perf_counter() - t0) * 1e3 / iters
        flop = 2 * b * r ** 3 * c * c * 27
        t["fwd_TF"] = flop / (t["fwd"] * 1e-3) / 1e12
        t["fwd_bwd_TF"] = 3 * flop / (t["fwd_bwd"] * 1e-3) / 1e12
        res[f"C{c}R{r}"] = {k: round(v, 3) for k, v in t.items()}
        print(variant, f"C{c}R{r}", res[f"C{c}R{r}"], flush=True)
    return res


if __name__ == "__main__":
    for v in (sys.argv[1:] or ["default", "cl3d", "nocudnn", "bench"]):
        t0 = time.perf_counter()
        run(v)
        print(v, "total probe time", round(time.perf_counter() - t0, 1), "s", flush=True)
