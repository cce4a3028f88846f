"""Dev probe: which part of PVConv's forward is not reproducible under GPU
contention?  Records, per PVConv call, the voxelized grid, the conv pair's
output and the SE-devox output (clones only there, to disturb timing little),
runs the point flow several times on identical inputs and reports the first
(call, stage) that differs.  Run two copies at once.  JSON lines."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import torch  # noqa: E402

import modules.pvconv as pv  # noqa: E402
import modules.norm_act as na  # noqa: E402
from pcfm.train import TrainConfig, Trainer  # noqa: E402

REC = []


def main():
    orig_tee = pv.Voxelization.forward_tee
    orig_pair = pv.conv_bn_act_pair
    orig_se = pv._SEDevoxAdd.apply

    def tee(self, f, c):
        out = orig_tee(self, f, c)
        REC.append(("grid", out[0].detach().clone()))
        return out

    def pair(*a, **k):
        out = orig_pair(*a, **k)
        REC.append(("pair", out.detach().clone()))
        return out

    def se(*a):
        ins = [x.detach().clone() if isinstance(x, torch.Tensor) else x for x in a]
        out = orig_se(*a)
        REC.append(("se_devox", out.detach().clone()))
        again = orig_se(*ins)  # same inputs, right away: an in-kernel race shows here
        REC.append(("se_devox_again_equal", torch.tensor(bool(torch.equal(out, again)))))
        for k, x in enumerate(ins):
            if isinstance(x, torch.Tensor):
                REC.append((f"se_in{k}", x))
        return out
    pv.Voxelization.forward_tee = tee
    pv.conv_bn_act_pair = pair
    pv._SEDevoxAdd.apply = se
    dev = torch.device("cuda", 0)
    b, n = int(os.environ.get("B", "8")), int(os.environ.get("N", "4096"))
    cfg = TrainConfig(batch_size=b, num_points=n, tunableop=False, miopen_find=False)
    tr = Trainer(cfg, dev)
    tr.train_mode()
    if os.environ.get("FREEZE", "1") == "1":
        for m in tr.pf.modules():
            if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
                m.momentum = 0.0
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(b, n, 6, device=dev, generator=g)
    t = torch.rand(b, device=dev, generator=g)
    cond = torch.randn(b, cfg.latent_dim + cfg.cond_dim, device=dev, generator=g)
    runs = []
    for _ in range(int(os.environ.get("RUNS", "10"))):
        REC.clear()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            tr.pf(x, t, cond, cond_drop_mask=None)
        torch.cuda.synchronize()
        runs.append(list(REC))
    for k in range(1, len(runs)):
        first = None
        for i, ((n0, a), (_, c)) in enumerate(zip(runs[0], runs[k])):
            if n0 == "se_devox_again_equal":
                if not bool(c):
                    first = {"record": i, "what": "se_devox not reproducible on its own inputs"}
                    break
                continue
            if not torch.equal(a, c):
                first = {"record": i, "what": n0,
                         "max_abs_diff": float((a - c).abs().max()),
                         "n_diff": int((a != c).sum())}
                break
        print(json.dumps({"run": k, "first": first}), flush=True)


if __name__ == "__main__":
    main()
