import sys, os, torch
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "point-cloud-flow-matching_amd")]
from pcfm.train import TrainConfig, Trainer, synthetic_batch
DEV = torch.device("cuda", 0)
cfg = dict(batch_size=2, num_points=1024, steps_per_epoch=4, epochs=1, tunableop=False, miopen_find=False, device_rng=False)
res = []
for fused in (True, True, False, False):
    tr = Trainer(TrainConfig(fused_step=fused, **cfg), DEV)
    tr.train_mode()
    batch = synthetic_batch(tr.cfg, DEV, generator=torch.Generator(device=DEV).manual_seed(3))
    torch.manual_seed(5)
    for _ in range(2):
        tr.step(batch, epoch=201)
    res.append([p.detach().double().sum().item() for p in tr._clip_params])
import numpy as np
a, b, c, d = map(np.array, res)
print("fused vs fused max diff", np.abs(a - b).max(), "torch vs torch", np.abs(c - d).max(), "fused vs torch", np.abs(a - c).max())
i = int(np.argmax(np.abs(a - c))); print("worst param index", i, a[i], c[i])
