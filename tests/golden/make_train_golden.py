"""Generate tests/golden/train_step_c1.npz by running the REFERENCE's train.main()
(/root/reference/train.py:86-715) for two steps on the CPU.

Run in the build container, where the reference tree is mounted read-only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_train_golden.py /root/reference

Nothing is copied out of the reference: the script imports it, runs it, and
records numbers.  Stand-ins, all outside the step being pinned:
  * `datasets` (h5py is not in the image): a synthetic
    dataset in the PartNet-H5 item schema (datasets.py:574-621:
    train_points / test_points (N, 3), train_rgb / test_rgb in [0, 1], cond (J,));
  * `modules.functional.backend` (its CUDA JIT build cannot run here): the C
    oracle's `_pvcnn_backend` surface (oracle/oracle.py TorchBackend).
The reference's own argparse defaults are used except for the flags below
(C1 size, two steps, RGB on from epoch 1, a CFG dropout that is not ~0).

Recorded per step (class-level wrappers around the reference's own objects,
so train.py:553-673 runs as written):
  * the batch (the encoder input = cat[train_points, train_rgb]; cond from the
    last columns of the point-flow condition);
  * every random draw in step order: torch.randn / torch.rand / torch.randn_like
    and Beta.sample -> z_pts (xyz randn, rgb rand), t_pts, the CFG-drop uniforms,
    eps_z, t_z;
  * the point-flow velocity, loss_point (= mse_xyz + lambda_color * mse_rgb) and
    loss_latent (the F.mse_loss values);
  * the pre-clip gradients (norm and sum per parameter, the first 8 values) and
    the total norm returned by clip_grad_norm_;
  * the parameters after AdamW.step (sum per parameter, the first 8 values) and
    the EMA shadows after each EMA.update.
The initial parameter sums are recorded too, so a reimplementation can check
that the same seed gives the same initial weights before anything else.
After the epoch the reference samples with its EMA weights (train.py:282-429,
Heun, --sample_steps 2): recorded are the prior draws, every velocity
evaluation (t, condition, v) of the point and latent flows, and the final
point clouds handed to chamfer_l2.

On the CPU the reference's CUDA autocast / GradScaler are inert (GradScaler
disables itself without CUDA), so the step is plain fp32.
"""
from __future__ import annotations

import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

B, N, J, LATENT = 2, 1024, 1, 128
N_ITEMS = 4  # -> 2 steps of B=2 (drop_last)
SEED = 123

ARGS = ["--data_dir", "unused", "--pf_backbone", "hybrid", "--batch_size", str(B),
        "--num_workers", "0", "--tr_max_sample_points", str(N), "--te_max_sample_points",
        str(N), "--latent_dim", str(LATENT), "--epochs", "1", "--save_every", "1",
        "--geom_warmup_epochs", "0", "--color_prior", "uniform", "--cfg_drop_p", "0.5",
        "--cfg_drop_warmup_epochs", "1", "--sample_steps", "2", "--vis_count", "1",
        "--seed", str(SEED)]


class _SynthDS(torch.utils.data.Dataset):
    """PartNet-H5 item schema (datasets.py:574-621) from a fixed numpy seed
    (no torch RNG is consumed, so the reference's seed_all stream is untouched)."""

    def __init__(self, seed):
        g = np.random.default_rng(seed)
        self.pts = g.standard_normal((N_ITEMS, N, 3)).astype(np.float32)
        self.rgb = g.random((N_ITEMS, N, 3)).astype(np.float32)
        self.cond = g.random((N_ITEMS, J)).astype(np.float32)
        self.cond_dim, self.has_rgb = J, True

    def __len__(self):
        return N_ITEMS

    def __getitem__(self, i):
        return {"idx": i, "train_points": torch.from_numpy(self.pts[i]),
                "test_points": torch.from_numpy(self.pts[i]),
                "train_rgb": torch.from_numpy(self.rgb[i]),
                "test_rgb": torch.from_numpy(self.rgb[i]),
                "cond": torch.from_numpy(self.cond[i])}


def _install_stubs():
    sys.path.insert(0, REPO)
    from oracle.oracle import TorchBackend
    be = types.ModuleType("modules.functional.backend")
    be._backend = TorchBackend()
    sys.modules["modules.functional.backend"] = be

    ds = types.ModuleType("datasets")

    def get_datasets(args):
        args.cond_dim, args.has_rgb = J, True
        return _SynthDS(1), _SynthDS(2)

    def init_np_seed(worker_id):
        np.random.seed(torch.initial_seed() % 4294967296)

    ds.get_datasets, ds.init_np_seed = get_datasets, init_np_seed
    sys.modules["datasets"] = ds


class _Recorder:
    def __init__(self):
        self.on = True
        self.sampling = False  # after the epoch: save_val_recon / save_val_samples
        self.steps = []  # one dict per training step
        self.events = []  # sampling-phase events in order
        self.names = {}

    @property
    def cur(self):
        return self.steps[-1]

    def draw(self, kind, t):
        if self.on and self.steps:
            self.cur.setdefault("draws", []).append((kind, t.detach().clone()))
        elif self.sampling:
            self.events.append(("draw", kind, t.detach().clone()))


def _first(t, k=8):
    return t.detach().reshape(-1)[:k].double().numpy()


def main() -> None:
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    torch.set_num_threads(1)
    _install_stubs()
    sys.path.insert(0, ref)
    import importlib.util
    import models  # reference models.py (puts third_party/pvcnn on sys.path itself)
    import util  # reference util.py
    # reference train.py by path (third_party/pvcnn, now on sys.path, has a train.py too)
    spec = importlib.util.spec_from_file_location("ref_train", os.path.join(ref, "train.py"))
    train = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(train)

    rec = _Recorder()
    F = torch.nn.functional

    def wrap_fn(owner, name, kind):
        orig = getattr(owner, name)

        def f(*a, **kw):
            out = orig(*a, **kw)
            rec.draw(kind, out)
            return out
        setattr(owner, name, f)

    wrap_fn(torch, "randn", "randn")
    wrap_fn(torch, "rand", "rand")
    wrap_fn(torch, "randn_like", "randn_like")
    beta_sample = torch.distributions.Beta.sample

    def beta(self, *a, **kw):
        out = beta_sample(self, *a, **kw)
        rec.draw("beta", out)
        return out
    torch.distributions.Beta.sample = beta

    enc_fwd = models.ShapeEncoder.forward

    def enc_forward(self, x):
        if rec.on:
            rec.steps.append({"enc_in": x.detach().clone()})
            rec.names.setdefault("enc", [n for n, _ in self.named_parameters()])
        return enc_fwd(self, x)
    models.ShapeEncoder.forward = enc_forward

    pf_fwd = models.HybridMLP.forward

    def pf_forward(self, x, t, cond, cond_drop_mask=None):
        out = pf_fwd(self, x, t, cond, cond_drop_mask=cond_drop_mask)
        if rec.on:
            rec.names.setdefault("pf", [n for n, _ in self.named_parameters()])
            rec.cur.update(x_t=x.detach().clone(), t_pts=t.detach().clone(),
                           cond_full=cond.detach().clone(), v=out.detach().clone(),
                           mask=(cond_drop_mask.detach().clone() if cond_drop_mask is not None
                                 else torch.zeros(x.shape[0], 1)))
        elif rec.sampling:
            rec.events.append(("pf", t.detach().clone(), cond.detach().clone(),
                               out.detach().clone()))
        return out
    models.HybridMLP.forward = pf_forward

    lf_fwd = models.ConditionalLatentVelocityNet.forward

    def lf_forward(self, y, t, cond, *a, **kw):
        out = lf_fwd(self, y, t, cond, *a, **kw)
        if rec.on:
            rec.names.setdefault("lf", [n for n, _ in self.named_parameters()])
            rec.cur.update(y_t=y.detach().clone(), v_z=out.detach().clone())
        elif rec.sampling:
            rec.events.append(("lf", t.detach().clone(), out.detach().clone()))
        return out
    models.ConditionalLatentVelocityNet.forward = lf_forward

    mse = F.mse_loss

    def mse_loss(a, b, *x, **kw):
        out = mse(a, b, *x, **kw)
        if rec.on and rec.steps:
            rec.cur.setdefault("mse", []).append(float(out.item()))
        return out
    F.mse_loss = mse_loss

    clip = torch.nn.utils.clip_grad_norm_

    def clip_grad_norm_(params, *a, **kw):
        params = list(params)
        if rec.on:
            rec.cur.update(
                pre_param_sums=np.array([p.detach().double().sum().item() for p in params]),
                grad_norms=np.array([p.grad.double().norm().item() if p.grad is not None else 0.0
                                     for p in params]),
                grad_sums=np.array([p.grad.double().sum().item() if p.grad is not None else 0.0
                                    for p in params]),
                grad_first=np.stack([_first(p.grad) if p.grad is not None and p.grad.numel() >= 8
                                     else np.zeros(8) for p in params]),
                numel=np.array([p.numel() for p in params]))
        total = clip(params, *a, **kw)
        if rec.on:
            rec.cur["total_norm"] = float(total)
        return total
    torch.nn.utils.clip_grad_norm_ = clip_grad_norm_

    adam_step = torch.optim.AdamW.step

    def step(self, *a, **kw):
        out = adam_step(self, *a, **kw)
        if rec.on:
            ps = [p for g in self.param_groups for p in g["params"]]
            rec.cur.update(
                post_param_sums=np.array([p.detach().double().sum().item() for p in ps]),
                post_param_first=np.stack([_first(p) if p.numel() >= 8 else np.zeros(8)
                                           for p in ps]),
                lrs=np.array([g["lr"] for g in self.param_groups]))
        return out
    torch.optim.AdamW.step = step

    ema_update = util.EMA.update

    def ema_upd(self, model):
        ema_update(self, model)
        if rec.on:
            key = "ema_pf" if "ctx_net.t_proj.weight" in self.shadow else "ema_lf"
            rec.cur[key] = np.array([v.double().sum().item() for v in self.shadow.values()
                                     if v.dtype.is_floating_point])
    util.EMA.update = ema_upd
    train.EMA.update = ema_upd

    save = torch.save

    def torch_save(*a, **kw):  # end of the epoch: the steps are done, sampling follows
        rec.on, rec.sampling = False, True
        return save(*a, **kw)
    torch.save = torch_save

    cd = train.chamfer_l2

    def chamfer_l2(pred, target):
        if rec.sampling:
            rec.events.append(("chamfer", pred.detach().clone(), target.detach().clone()))
        return cd(pred, target)
    train.chamfer_l2 = chamfer_l2

    with tempfile.TemporaryDirectory() as out_dir:
        sys.argv = ["train.py"] + ARGS + ["--out_dir", out_dir]
        train.main()

    out = {"args": np.array(ARGS), "n_steps": len(rec.steps)}
    for k, v in rec.names.items():
        out[f"names_{k}"] = np.array(v)
    for i, st in enumerate(rec.steps):
        p = f"s{i}_"
        enc_in = st["enc_in"].numpy()
        out[p + "train_points"] = enc_in[..., :3]
        out[p + "train_rgb"] = enc_in[..., 3:]
        out[p + "cond"] = st["cond_full"][:, LATENT:].numpy()
        kinds = [k for k, _ in st["draws"]]
        # train.py:271-276 (uniform colour prior), :604-605, :617, :637, :639-640
        assert kinds == ["randn", "rand", "beta", "rand", "randn_like", "beta"], kinds
        d = [t for _, t in st["draws"]]
        out[p + "z_pts"] = torch.cat([d[0], d[1]], dim=-1).numpy()
        out[p + "t_pts"] = d[2].numpy()
        out[p + "drop_u"] = d[3].numpy()
        out[p + "eps_z"] = d[4].numpy()
        out[p + "t_z"] = d[5].numpy()
        for k in ("x_t", "v", "mask", "y_t", "v_z"):
            out[p + k] = st[k].numpy()
        mses = st["mse"]
        assert len(mses) == 3, mses  # xyz, rgb, latent
        out[p + "mse"] = np.array(mses)
        for k in ("pre_param_sums", "grad_norms", "grad_sums", "grad_first", "numel",
                  "post_param_sums", "post_param_first", "lrs", "ema_pf", "ema_lf",
                  "total_norm"):
            out[p + k] = np.asarray(st[k])
    # sampling (train.py:282-429, EMA weights, Heun with --sample_steps 2):
    # save_val_recon (encoder z, point Heun), then save_val_samples (latent Heun
    # from randn z, point Heun); each ends in a chamfer_l2 call
    ev = rec.events
    cuts = [i for i, e in enumerate(ev) if e[0] == "chamfer"]
    assert len(cuts) == 2, [e[0] for e in ev]
    for tag, part in (("recon", ev[:cuts[0] + 1]), ("samples", ev[cuts[0] + 1:cuts[1] + 1])):
        draws = [e for e in part if e[0] == "draw"]
        pfs = [e for e in part if e[0] == "pf"]
        lfs = [e for e in part if e[0] == "lf"]
        if tag == "samples":
            assert [d[1] for d in draws] == ["randn", "randn", "rand"], [d[1] for d in draws]
            out["samples_z0"] = draws[0][2].numpy()
            out["samples_lf_t"] = np.stack([e[1].numpy() for e in lfs])
            out["samples_lf_v"] = np.stack([e[2].numpy() for e in lfs])
            draws = draws[1:]
        else:
            assert [d[1] for d in draws] == ["randn", "rand"], [d[1] for d in draws]
        out[f"{tag}_x0"] = torch.cat([draws[0][2], draws[1][2]], -1).numpy()
        out[f"{tag}_cond"] = pfs[0][2].numpy()
        out[f"{tag}_pf_t"] = np.stack([e[1].numpy() for e in pfs])
        out[f"{tag}_pf_v"] = np.stack([e[3].numpy() for e in pfs])
        out[f"{tag}_final_xyz"] = part[-1][1].numpy()
        out[f"{tag}_target"] = part[-1][2].numpy()
    np.savez_compressed(os.path.join(HERE, "train_step_c1.npz"), **out)
    print("wrote train_step_c1.npz:", len(rec.steps), "steps; losses",
          [s["mse"] for s in rec.steps])


if __name__ == "__main__":
    main()
