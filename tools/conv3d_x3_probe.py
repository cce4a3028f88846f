"""Probe: bf16x3 voxel conv vs MIOpen fp32 at the PVConv shapes: accuracy
against an fp64 reference and time.  Dev tool."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm import ops  # noqa: E402

torch.backends.cudnn.benchmark = True
torch.backends.cudnn.allow_tf32 = False


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / iters


for b, c, r in [(8, 128, 32), (8, 256, 16), (8, 256, 8)]:
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(b, c, r, r, r, device="cuda", generator=g)
    w = torch.randn(c, c, 3, 3, 3, device="cuda", generator=g) * (1.0 / (27 * c) ** 0.5)
    bias = torch.randn(c, device="cuda", generator=g)
    gy = torch.randn(b, c, r, r, r, device="cuda", generator=g)
    y = ops.conv3d_forward(x, w, bias)
    dx = ops.conv3d_backward_data(gy, w)
    dw = ops.conv3d_backward_weight(x, gy)
    dw32 = torch.nn.grad.conv3d_weight(x, w.shape, gy, padding=1)
    y32 = torch.nn.functional.conv3d(x, w, bias, padding=1)
    dx32 = torch.nn.grad.conv3d_input(x.shape, w, gy, padding=1)
    # fp64 reference on 2 samples
    x64, w64 = x[:2].double().cpu(), w.double().cpu()
    y64 = torch.nn.functional.conv3d(x64, w64, bias.double().cpu(), padding=1)
    dx64 = torch.nn.grad.conv3d_input(x64.shape, w64, gy[:2].double().cpu(), padding=1)
    dw64 = torch.nn.grad.conv3d_weight(x64, w64.shape, gy[:2].double().cpu(), padding=1)
    dw2 = ops.conv3d_backward_weight(x[:2].contiguous(), gy[:2].contiguous())
    dw2_32 = torch.nn.grad.conv3d_weight(x[:2], w.shape, gy[:2], padding=1)

    def rel(a, ref):
        a = a.double().cpu()
        return ((a - ref).abs().max() / ref.pow(2).mean().sqrt()).item()

    flop = 2 * b * r ** 3 * c * c * 27
    t_x3 = timeit(lambda: ops.conv3d_forward(x, w, bias))
    t_bd = timeit(lambda: ops.conv3d_backward_data(gy, w))
    t_32 = timeit(lambda: torch.nn.functional.conv3d(x, w, bias, padding=1))
    t_wg_old = timeit(lambda: ops.conv3d_backward_weight(x, gy))
    xs_, gys_ = ops.conv3d_split(x), ops.conv3d_split(gy)
    t_wg = timeit(lambda: ops.conv3d_wgrad_split(xs_, gys_, b, c, c, r))
    t_split = timeit(lambda: ops.conv3d_split(gy))
    print(f"   split {t_split:.3f} ms; wgrad (split operands) {t_wg:.3f} ms vs on-the-fly "
          f"{t_wg_old:.3f} ms")
    t_wg32 = timeit(lambda: torch.nn.grad.conv3d_weight(x, w.shape, gy, padding=1))
    t_bd32 = timeit(lambda: torch.nn.grad.conv3d_input(x.shape, w, gy, padding=1))
    print(f"C{c}R{r}: fwd x3 {t_x3:.3f} ms ({flop / t_x3 / 1e9:.0f} TF)  bwd-data x3 {t_bd:.3f} ms"
          f" ({flop / t_bd / 1e9:.0f} TF)  MIOpen fp32 fwd {t_32:.3f} ms ({flop / t_32 / 1e9:.0f} TF)"
          f" | max err/rms vs fp64: x3 fwd {rel(y[:2], y64):.2e} bwd {rel(dx[:2], dx64):.2e}"
          f"  fp32 fwd {rel(y32[:2], y64):.2e} bwd {rel(dx32[:2], dx64):.2e}", flush=True)
    print(f"   wgrad x3 {t_wg:.3f} ms ({flop / t_wg / 1e9:.0f} TF) MIOpen fp32 wgrad {t_wg32:.3f} ms "
          f"bwd-data {t_bd32:.3f} ms | wgrad err/rms vs fp64: x3 {rel(dw2, dw64):.2e} "
          f"fp32 {rel(dw2_32, dw64):.2e}; full-batch x3 vs fp32 {rel(dw, dw32.double().cpu()):.2e}",
          flush=True)
