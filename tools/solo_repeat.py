"""Dev probe: one process, no second GPU user -- the DDP gradient-mean test's
reference step (Trainer.forward_backward on one B=8 shard) repeated RUNS times
on identical inputs; reports every run whose head_out.weight gradient or
devoxelization outputs differ from run 0's (element detail as in
tests/helpers/ddp_grad_rank.py).  JSON lines."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd"),
                os.path.join(REPO, "tests", "helpers")]

import torch  # noqa: E402

import ddp_grad_rank as H  # noqa: E402
from pcfm.train import TrainConfig, Trainer  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    cfg = TrainConfig(batch_size=H.B, num_points=H.N, steps_per_epoch=4, epochs=1,
                      tunableop=False, miopen_find=False)
    tr = Trainer(cfg, dev)
    tr.train_mode()
    H._trace_ops()
    batch, draws = H.shard(cfg, 0, dev)
    ref, ref_keep = None, None
    bad = 0
    for k in range(int(os.environ.get("RUNS", "40"))):
        tr.opt.zero_grad(set_to_none=True)
        H.TRACE = []
        H.KEEP.clear()
        tr.forward_backward(batch, H.EPOCH, draws)
        g = tr.pf.ctx_net.head_out.weight.grad.detach().clone()
        keep = list(H.KEEP)
        torch.cuda.synchronize()
        if ref is None:
            ref, ref_keep = g, keep
            continue
        if not torch.equal(g, ref):
            bad += 1
            rep = None
            for ci, (ta, tb) in enumerate(zip(ref_keep, keep)):
                for ti, (u, v) in enumerate(zip(ta, tb)):
                    if u.shape == v.shape and not torch.equal(u, v):
                        d = u != v
                        rep = {"call": ci, "tensor": ti, "n_diff": int(d.sum()),
                               "first_idx": d.nonzero()[:4].tolist()}
                        break
                if rep:
                    break
            print(json.dumps({"run": k, "head_out_grad_differs": True, "devox": rep}), flush=True)
    print(json.dumps({"runs": int(os.environ.get("RUNS", "40")), "differing": bad}), flush=True)


if __name__ == "__main__":
    main()
