"""Run-to-run reproducibility of the HybridMLP (C1, perturbed golden) forward +
backward on the HIP path (dev tool): the same inputs and weights N times in one
process, exact-fp32 mode; per parameter, how many distinct gradient bit
patterns came out, and the gradient-norm deviation from the golden per
iteration.  One JSON line per finding, then a summary line."""
import hashlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd"), os.path.join(REPO, "tests")]


def main():
    from golden_util import perturb_zero_init_
    from pcfm import _lib
    from pcfm.models import HybridMLP
    from pcfm.precision import exact_fp32
    _lib.load()
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    g = np.load(os.path.join(REPO, "tests", "golden", "model_hybrid_c1_perturbed.npz"))
    torch.manual_seed(int(g["seed"]))
    pf = HybridMLP(cond_dim=129, point_dim=6)
    perturb_zero_init_(pf, int(g["perturb_seed"]))
    pf = pf.to("cuda").train()
    names = [n for n, _ in pf.named_parameters()]
    x = torch.from_numpy(g["x"]).cuda()
    t = torch.from_numpy(g["t"]).cuda()
    cond = torch.from_numpy(g["cond"]).cuda()
    mask = torch.from_numpy(g["mask"]).cuda()
    target = torch.from_numpy(g["target"]).cuda()
    hashes = [set() for _ in names]
    vh = set()
    devs = []
    for _ in range(reps):
        pf.zero_grad(set_to_none=True)
        with exact_fp32(True):
            v = pf(x, t, cond, cond_drop_mask=mask)
            loss = torch.nn.functional.mse_loss(v, target)
            loss.backward()
        torch.cuda.synchronize()
        vh.add(hashlib.sha1(v.detach().cpu().numpy().tobytes()).hexdigest())
        norms = []
        for i, p in enumerate(pf.parameters()):
            if p.grad is None:
                norms.append(0.0)
                continue
            hashes[i].add(hashlib.sha1(p.grad.cpu().numpy().tobytes()).hexdigest())
            norms.append(p.grad.double().norm().item())
        gd = np.abs(np.array(norms) - g["grad_norms"]) / np.maximum(g["grad_norms"], 1e-30)
        live = np.array([not n.endswith(".bias") or gd[i] < 1 for i, n in enumerate(names)])
        devs.append(float(gd[live].max()))
    varying = [(names[i], len(h)) for i, h in enumerate(hashes) if len(h) > 1]
    for n, k in varying:
        print(json.dumps({"param": n, "distinct_grads": k}))
    print(json.dumps({"reps": reps, "distinct_v": len(vh), "params_varying": len(varying),
                      "grad_norm_dev_per_rep": devs}))


if __name__ == "__main__":
    main()
