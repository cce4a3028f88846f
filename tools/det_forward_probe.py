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
            if i and isinstance(i[0], torch.Tensor):
                outs.append((name + ".in", i[0].detach().clone()))
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
    runs = int(os.environ.get("RUNS", "3"))
    res = [run(tr, x, t, cond, None) for _ in range(runs)]
    for k in range(1, runs):
        diff = [name for (name, a), (_, c) in zip(res[0][1], res[k][1])
                if a.shape != c.shape or not torch.equal(a, c)]
        print(json.dumps({"run": k, "v_equal": bool(torch.equal(res[0][0], res[k][0])),
                          "n_hooked": len(res[0][1]), "n_differ": len(diff),
                          "first_differ": diff[:12]}), flush=True)


if __name__ == "__main__" and not os.environ.get("BWD"):
    main()


def backward_probe():
    """head_out's saved input vs its input at call time (an in-place overwrite
    by a later kernel would show here), and head_out.weight.grad over two
    identical forward_backward calls."""
    dev = torch.device("cuda", 0)
    b, n = int(os.environ.get("B", "8")), int(os.environ.get("N", "4096"))
    cfg = TrainConfig(batch_size=b, num_points=n, tunableop=False, miopen_find=False)
    tr = Trainer(cfg, dev)
    tr.train_mode()
    ho = tr.pf.ctx_net.head_out
    seen = {}

    def hook(m, i, o):
        seen["in"] = i[0].detach().clone()
        seen["out"] = o
    h = ho.register_forward_hook(hook)
    from pcfm.train import synthetic_batch
    batch = synthetic_batch(cfg, dev, generator=torch.Generator(device=dev).manual_seed(3))
    grads = []
    for k in range(3):
        tr.opt.zero_grad(set_to_none=True)
        torch.manual_seed(5)
        orig = tr.scaler.scale

        def scale_hook(loss, orig=orig):
            saved = seen["out"].grad_fn.saved_tensors[0]
            seen["saved_equal"] = bool(torch.equal(saved, seen["in"]))
            seen["saved_maxdiff"] = float((saved - seen["in"]).abs().max())
            return orig(loss)
        tr.scaler.scale = scale_hook
        tr.forward_backward(batch, 201)
        tr.scaler.scale = orig
        grads.append(ho.weight.grad.detach().clone())
        print(json.dumps({"call": k, "saved_input_unchanged": seen["saved_equal"],
                          "saved_maxdiff": seen["saved_maxdiff"],
                          "wgrad_equal_to_first": bool(torch.equal(grads[0], grads[-1]))}),
              flush=True)
    h.remove()


if __name__ == "__main__" and os.environ.get("BWD"):
    backward_probe()
