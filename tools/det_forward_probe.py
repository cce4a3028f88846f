"""Dev probe: is the hybrid point flow's forward bitwise reproducible?  Runs
pf.forward twice on identical inputs (train mode, the production path) with a
forward hook on every submodule and reports, in execution order, the modules
whose outputs differ between the two runs (the first one is the culprit; the
rest inherit it).  Also repeats single ops at the C2 shapes.  JSON lines."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import torch  # noqa: E402

from pcfm.train import TrainConfig, Trainer  # noqa: E402


def run(tr, x, t, cond, mask):
    outs = []
    hooks = []
    for name, mod in tr.pf.named_modules():
        def hook(m, i, o, name=name):
            o = o[0] if isinstance(o, tuple) else o
            if isinstance(o, torch.Tensor):
                outs.append((name, o.detach().clone()))
        hooks.append(mod.register_forward_hook(hook))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        v = tr.pf(x, t, cond, cond_drop_mask=mask)
    for h in hooks:
        h.remove()
    torch.cuda.synchronize()
    return v.detach().clone(), outs


def main():
    dev = torch.device("cuda", 0)
    b, n = int(os.environ.get("B", "8")), int(os.environ.get("N", "4096"))
    cfg = TrainConfig(batch_size=b, num_points=n, tunableop=False, miopen_find=False)
    tr = Trainer(cfg, dev)
    tr.train_mode()
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(b, n, 6, device=dev, generator=g)
    t = torch.rand(b, device=dev, generator=g)
    cond = torch.randn(b, cfg.latent_dim + cfg.cond_dim, device=dev, generator=g)
    res = [run(tr, x, t, cond, None) for _ in range(3)]
    for k in (1, 2):
        diff = [name for (name, a), (_, c) in zip(res[0][1], res[k][1])
                if a.shape != c.shape or not torch.equal(a, c)]
        print(json.dumps({"run": k, "v_equal": bool(torch.equal(res[0][0], res[k][0])),
                          "n_hooked": len(res[0][1]), "n_differ": len(diff),
                          "first_differ": diff[:12]}), flush=True)


if __name__ == "__main__":
    main()
