"""Where does the GPU path's gradient leave the CPU path's?  (dev diagnostic)

MODE=sensitivity (CPU only): the same comparison between two CPU runs whose
rgb inputs differ by 1e-6 relative (coordinates untouched, so no voxel moves):
how far the model's own backward moves when its forward moves by ~1e-6 -- the
floor of any elementwise gradient comparison (profiles/r05_grad_sensitivity.json).

Runs the perturbed C1 hybrid golden (tests/golden/model_hybrid_c1_perturbed.npz)
once on cuda:0 in exact-fp32 mode and once on the CPU (pcfm.cpu_ops backend),
same weights and inputs, and compares the gradient arriving at every
submodule's output (max |g_gpu - g_cpu| / max |g_cpu|), in backward order, plus
the parameter gradients per module.  Prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd"), os.path.join(REPO, "tests")]

from golden_util import perturb_zero_init_  # noqa: E402
from pcfm.models import HybridMLP  # noqa: E402
from pcfm.precision import exact_fp32  # noqa: E402


def run(dev, g, rgb_eps=0.0):
    torch.manual_seed(int(g["seed"]))
    pf = HybridMLP(cond_dim=129, point_dim=6)
    perturb_zero_init_(pf, int(g["perturb_seed"]))
    pf = pf.to(dev).train()
    grads, order = {}, []

    def hook(name):
        def fwd(mod, inp, out):
            t = out[0] if isinstance(out, (tuple, list)) else out
            if torch.is_tensor(t) and t.requires_grad:
                def cap(gr, name=name):
                    grads[name] = gr.detach().double().cpu()
                    order.append(name)
                t.register_hook(cap)
        return fwd

    for n, m in pf.named_modules():
        if n and n.count(".") <= 5:
            m.register_forward_hook(hook(n))
    x = torch.from_numpy(g["x"]).clone()
    if rgb_eps:
        gen = torch.Generator().manual_seed(5)
        x[..., 3:] *= 1 + rgb_eps * torch.randn(x[..., 3:].shape, generator=gen)
    x = x.to(dev)
    v = pf(x, torch.from_numpy(g["t"]).to(dev), torch.from_numpy(g["cond"]).to(dev),
           cond_drop_mask=torch.from_numpy(g["mask"]).to(dev))
    loss = torch.nn.functional.mse_loss(v, torch.from_numpy(g["target"]).to(dev))
    loss.backward()
    pg = {n: p.grad.detach().double().cpu() for n, p in pf.named_parameters() if p.grad is not None}
    return grads, order, pg


def main():
    g = np.load(os.path.join(REPO, "tests", "golden", "model_hybrid_c1_perturbed.npz"))
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cudnn.benchmark = False
    mode = os.environ.get("MODE", "exact")
    rel = lambda a, b: float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))  # noqa: E731
    if mode == "sensitivity":
        torch.set_num_threads(8)
        a, order, pa = run("cpu", g)
        b, _, pb = run("cpu", g, rgb_eps=1e-6)
        print(json.dumps({"mode": mode, "rgb_rel_perturbation": 1e-6,
                          "outputs": [(n, rel(b[n], a[n])) for n in order],
                          "params": sorted(((n, rel(pb[n], pa[n])) for n in pa),
                                           key=lambda kv: -kv[1])[:40]}))
        return
    if "bmm64" in mode:  # the exact-fp32 1x1 convs' GEMMs in float64 (isolates hipBLASLt fp32)
        from modules import shared_mlp as SM
        orig = SM.PointwiseConv1d.forward

        def fwd64(self, x):
            if self.x3_ok(x) or not self._is_1x1() or x.dim() != 3 or not x.is_cuda:
                return orig(self, x)
            w = self.weight[:, :, 0].double().unsqueeze(0).expand(x.shape[0], -1, -1)
            y = torch.bmm(w, x.double())
            if self.bias is not None:
                y = y + self.bias.double()[None, :, None]
            return y.float()
        SM.PointwiseConv1d.forward = fwd64
    if "torchbn" in mode:  # torch's BatchNorm + activation instead of the fused kernels
        from modules import norm_act as NA
        NA._fusable = lambda *a, **k: False
    if mode.startswith("exact"):
        with exact_fp32(True):
            gg, order, gp = run("cuda", g)
    else:
        gg, order, gp = run("cuda", g)
    torch.set_num_threads(8)
    cg, _, cp = run("cpu", g)
    out = {"mode": mode, "outputs": [(n, rel(gg[n], cg[n])) for n in order if n in cg],
           "params": sorted(((n, rel(gp[n], cp[n])) for n in gp if n in cp),
                            key=lambda kv: -kv[1])[:40]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
