"""The N>1 path on the CPU: two ranks, gloo, the same DDP wiring bench.py uses
over RCCL (one process per device, batch sharded, gradient all-reduce).

* PVConv under DDP: each rank's gradient after backward equals the mean of the
  per-shard gradients computed in one process (the all-reduce is the only
  exchange step).
* Trainer.step under DDP: after one full step (backward, clip, AdamW) the
  parameters are identical on both ranks.
"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "point-cloud-flow-matching_amd")
WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup(rank, port):
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from oracle.oracle import TorchBackend
    import modules.functional.backend as be
    be._backend = TorchBackend()
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=WORLD)


def _pvconv_batch():
    g = torch.Generator().manual_seed(7)
    feats = torch.randn(2 * WORLD, 8, 256, generator=g)
    coords = torch.randn(2 * WORLD, 3, 256, generator=g)
    return feats, coords


def _pvconv_model():
    from modules import PVConv
    torch.manual_seed(3)
    return PVConv(8, 8, 3, resolution=4, with_se=True)


def _rank_pvconv(rank, port, out_dir):
    _setup(rank, port)
    from torch.nn.parallel import DistributedDataParallel as DDP
    model = DDP(_pvconv_model())
    feats, coords = _pvconv_batch()
    sl = slice(2 * rank, 2 * rank + 2)
    y, _ = model((feats[sl], coords[sl]))
    y.square().mean().backward()
    grads = {k: p.grad.clone() for k, p in model.module.named_parameters()}
    torch.save(grads, os.path.join(out_dir, f"pv{rank}.pt"))
    dist.destroy_process_group()


def _rank_train(rank, port, out_dir):
    _setup(rank, port)
    from pcfm.train import TrainConfig, Trainer, synthetic_batch
    cfg = TrainConfig(batch_size=2, num_points=256, ctx_stage_channels=[16, 32, 32],
                      ctx_stage_res=[4, 4, 2], pf_width=32, lf_width=32, enc_width=16,
                      latent_dim=8, steps_per_epoch=4, epochs=1)
    tr = Trainer(cfg, "cpu", rank=rank, world_size=WORLD, ddp=True)
    tr.train_mode()
    g = torch.Generator().manual_seed(100 + rank)  # a different shard per rank
    tr.step(synthetic_batch(cfg, "cpu", generator=g), epoch=201)
    params = {f"{name}.{k}": v.detach().clone()
              for name, m in (("enc", tr.enc), ("pf", tr.pf), ("lf", tr.lf))
              for k, v in m.state_dict().items()}
    torch.save(params, os.path.join(out_dir, f"tr{rank}.pt"))
    dist.destroy_process_group()


def _spawn(fn, tmp_path):
    mp.start_processes(fn, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True,
                       start_method="spawn")


def test_ddp_pvconv_grads_are_shard_mean(tmp_path, oracle_backend):
    _spawn(_rank_pvconv, tmp_path)
    g0 = torch.load(tmp_path / "pv0.pt", weights_only=True)
    g1 = torch.load(tmp_path / "pv1.pt", weights_only=True)
    # single-process reference: per-shard grads, averaged
    model = _pvconv_model()
    feats, coords = _pvconv_batch()
    per = []
    for r in range(WORLD):
        model.zero_grad()
        sl = slice(2 * r, 2 * r + 2)
        y, _ = model((feats[sl], coords[sl]))
        y.square().mean().backward()
        per.append({k: p.grad.clone() for k, p in model.named_parameters()})
    for k in g0:
        want = (per[0][k] + per[1][k]) / WORLD
        torch.testing.assert_close(g0[k], g1[k], rtol=0, atol=0)
        torch.testing.assert_close(g0[k], want, rtol=1e-5, atol=1e-6)


def test_ddp_train_step_keeps_ranks_in_sync(tmp_path):
    _spawn(_rank_train, tmp_path)
    p0 = torch.load(tmp_path / "tr0.pt", weights_only=True)
    p1 = torch.load(tmp_path / "tr1.pt", weights_only=True)
    assert p0.keys() == p1.keys()
    for k in p0:
        if "running_" in k or "num_batches" in k:
            continue  # BatchNorm statistics are per rank (no SyncBN), as in the reference
        torch.testing.assert_close(p0[k], p1[k], rtol=0, atol=0, msg=k)
