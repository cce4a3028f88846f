"""One rank of tests/test_gpu_ddp.py: two Trainer steps under DDP (gloo, the
ranks sharing the box's GPU), then every rank's parameter / EMA checksums and
the step's losses are gathered and written by rank 0 to argv[1]."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pcfm.train import TrainConfig, Trainer, init_distributed, synthetic_batch  # noqa: E402


def main():
    _, rank, world, local = init_distributed("gloo")
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    cfg = TrainConfig(batch_size=2, num_points=2048, steps_per_epoch=4, epochs=1,
                      tunableop=False, miopen_find=False)
    tr = Trainer(cfg, dev, rank=rank, world_size=world, ddp=True)
    tr.train_mode()
    batch = synthetic_batch(cfg, dev, generator=torch.Generator(device=dev).manual_seed(7 + rank))
    out = None
    for _ in range(2):
        out = tr.step(batch, epoch=201)
    torch.cuda.synchronize(dev)
    # the parameters (DDP broadcasts rank 0's at wrap time; the EMA shadows are
    # taken before the wrap from each rank's own seed + rank init, as the
    # reference does, train.py:182, 232, 242-244, so they are rank-specific)
    sums = torch.tensor([p.detach().double().sum().item() for p in tr._clip_params],
                        dtype=torch.float64)
    gathered = [torch.zeros_like(sums) for _ in range(world)]
    dist.all_gather(gathered, sums)
    losses = torch.tensor([float(out["loss_point"]), float(out["loss_latent"])],
                          dtype=torch.float64)
    lg = [torch.zeros_like(losses) for _ in range(world)]
    dist.all_gather(lg, losses)
    if rank == 0:
        json.dump({"world": world, "sums": [g.tolist() for g in gathered],
                   "losses": [g.tolist() for g in lg],
                   "backend": dist.get_backend()}, open(sys.argv[1], "w"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
