"""Elementwise parameter-gradient fixtures from the REFERENCE's own modules.

    python tests/golden/make_grad_golden.py /root/reference

Run in the build container (the reference tree is mounted read-only there);
nothing under tests/ reads the reference at test time -- only the .npz files.
Same setup as make_golden.py (reference Python imported by path, the native
`_pvcnn_backend` replaced by this build's C oracle, CPU, one thread), same
seeds and inputs as pvconv_r8.npz and model_hybrid_c1_perturbed.npz:

  * pvconv_r8_grads.npz -- every parameter gradient of the reference PVConv
    block (R=8, SE), in full (15 k values).
  * model_hybrid_c1_perturbed_grads.npz -- the reference HybridMLP at C1 size
    with its zero-initialised parameters perturbed (so every branch reaches v):
    for each parameter, the gradient at up to 64 seeded positions (the whole
    20.8 M-value gradient would be an 83 MB fixture) plus the parameter's max
    |gradient| over ALL its elements, the normaliser of the elementwise test.

tests/test_gpu_model.py::test_*_elementwise_grads compare the HIP path with
these per element."""
from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402

SAMPLES = 64


def sample_positions(numel: int, k: int, seed: int) -> np.ndarray:
    """Seeded sorted flat positions; tests/golden_util.py restates this."""
    if numel <= k:
        return np.arange(numel, dtype=np.int64)
    g = torch.Generator().manual_seed(seed)
    return np.sort(torch.randperm(numel, generator=g)[:k].numpy()).astype(np.int64)


def pvconv_grads(ref: str) -> None:
    from modules.pvconv import PVConv  # reference
    torch.manual_seed(7)
    blk = PVConv(16, 16, kernel_size=3, resolution=8, with_se=True, normalize=True, eps=1e-6)
    d = np.load(os.path.join(HERE, "pvconv_r8.npz"))
    feats = torch.from_numpy(d["feats"]).requires_grad_(True)
    coords = torch.from_numpy(d["coords"])
    out, _ = blk((feats, coords))
    assert np.array_equal(out.detach().numpy(), d["out"])  # the pinned forward, unchanged
    loss = (out * torch.linspace(-1, 1, out.numel()).view_as(out)).sum()
    loss.backward()
    arrs = {f"grad/{n}": p.grad.numpy() for n, p in blk.named_parameters()}
    np.savez_compressed(os.path.join(HERE, "pvconv_r8_grads.npz"), **arrs)


def hybrid_perturbed_grads(ref: str) -> None:
    import models  # reference
    d = np.load(os.path.join(HERE, "model_hybrid_c1_perturbed.npz"))
    torch.manual_seed(int(d["seed"]))
    pf = models.HybridMLP(cond_dim=129, point_dim=6)
    MG.perturb_zero_init_(pf, int(d["perturb_seed"]))
    pf.train()
    v = pf(torch.from_numpy(d["x"]), torch.from_numpy(d["t"]), torch.from_numpy(d["cond"]),
           cond_drop_mask=torch.from_numpy(d["mask"]))
    assert np.array_equal(v.detach().numpy(), d["v"])
    loss = torch.nn.functional.mse_loss(v, torch.from_numpy(d["target"]))
    loss.backward()
    names, pos, vals, absmax, param_of = [], [], [], [], []
    for i, (n, p) in enumerate(pf.named_parameters()):
        names.append(n)
        g = p.grad.reshape(-1).numpy() if p.grad is not None else np.zeros(p.numel(), np.float32)
        idx = sample_positions(g.size, SAMPLES, 1000 + i)
        pos.append(idx)
        vals.append(g[idx])
        param_of.append(np.full(idx.size, i, np.int32))
        absmax.append(float(np.abs(g).max()))
    np.savez_compressed(
        os.path.join(HERE, "model_hybrid_c1_perturbed_grads.npz"), param_names=np.array(names),
        param_of=np.concatenate(param_of), flat_pos=np.concatenate(pos),
        grad=np.concatenate(vals).astype(np.float32), grad_absmax=np.array(absmax, np.float64))


def main() -> None:
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    torch.set_num_threads(1)
    MG._install_oracle_backend()
    sys.path.insert(0, os.path.join(ref, "third_party", "pvcnn"))
    sys.path.insert(0, ref)
    pvconv_grads(ref)
    hybrid_perturbed_grads(ref)
    print("wrote pvconv_r8_grads.npz, model_hybrid_c1_perturbed_grads.npz")


if __name__ == "__main__":
    main()
