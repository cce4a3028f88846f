"""Trainer checkpoint / resume (the reference's checkpoint dict, train.py:681-699,
and auto-resume, :470-520) on the CPU: a resumed trainer continues exactly
where the saved one would have."""
import torch

from pcfm.train import TrainConfig, Trainer, synthetic_batch


def _cfg(seed):
    return TrainConfig(batch_size=2, num_points=256, ctx_stage_channels=[16, 32, 32],
                       ctx_stage_res=[4, 4, 2], pf_width=32, lf_width=32, enc_width=16,
                       latent_dim=8, steps_per_epoch=4, epochs=1, seed=seed, amp=False)


def _state(tr):
    out = {}
    for name, m in (("enc", tr.enc), ("pf", tr.pf), ("lf", tr.lf)):
        out.update({f"{name}.{k}": v.detach().clone() for k, v in m.state_dict().items()})
    out.update({f"ema_pf.{k}": v.clone() for k, v in tr.ema_pf.shadow.items()})
    return out


def test_resume_continues_bit_exact(tmp_path, oracle_backend):
    batch = synthetic_batch(_cfg(0), "cpu", generator=torch.Generator().manual_seed(7))
    a = Trainer(_cfg(0), "cpu")
    a.train_mode()
    for _ in range(2):
        a.step(batch, epoch=201)
    path = tmp_path / "hybrid_ep0001.pt"
    torch.save(a.checkpoint(epoch=1), path)
    ck = torch.load(path, map_location="cpu", weights_only=True)
    assert set(ck) >= {"epoch", "encoder", "pf", "lf", "ema_pf", "ema_lf", "args", "cond_dim",
                       "opt", "scaler", "global_step"}

    b = Trainer(_cfg(123), "cpu")  # different initial weights
    b.train_mode()
    assert b.load_checkpoint(ck) == 2
    sa, sb = _state(a), _state(b)
    assert all(torch.equal(sa[k], sb[k]) for k in sa)

    for tr in (a, b):
        torch.manual_seed(99)  # the step's draws
        tr.step(batch, epoch=201)
    sa, sb = _state(a), _state(b)
    bad = [k for k in sa if not torch.equal(sa[k], sb[k])]
    assert not bad, bad[:5]


def test_load_checkpoint_rejects_wrong_ema_shape(oracle_backend):
    a = Trainer(_cfg(0), "cpu")
    ck = a.checkpoint(epoch=3)
    k = next(iter(ck["ema_pf"]))
    ck["ema_pf"][k] = torch.zeros(3, 3, 3)
    try:
        Trainer(_cfg(0), "cpu").load_checkpoint(ck)
    except ValueError as e:
        assert "shape" in str(e)
    else:
        raise AssertionError("a wrong-shape EMA entry was accepted")


def test_unfitting_optimizer_state_warns_and_resumes(oracle_backend, capsys):
    """An optimizer / scaler state that does not load (here: one parameter group
    missing) is reported and skipped; weights, EMA and epoch still resume
    (reference train.py:498-516)."""
    a = Trainer(_cfg(0), "cpu")
    ck = a.checkpoint(epoch=6)
    ck["opt"]["param_groups"] = ck["opt"]["param_groups"][:2]
    ck["scaler"] = {"scale": "not a number"}
    b = Trainer(_cfg(123), "cpu")
    assert b.load_checkpoint(ck) == 7
    assert "opt state load failed" in capsys.readouterr().out
    sa, sb = _state(a), _state(b)
    assert all(torch.equal(sa[k], sb[k]) for k in sa)


@__import__("pytest").mark.gpu
def test_resume_fused_step_gpu(tmp_path):
    """Same on the GPU path: fused AdamW + EMA update (pcfm.optim), bf16 autocast
    head, AMP scaler state; the resumed trainer's next step is bit-identical."""
    def cfg(seed):
        c = _cfg(seed)
        c.amp, c.miopen_find, c.tunableop = True, False, False
        return c
    dev = torch.device("cuda", 0)
    batch = synthetic_batch(cfg(0), dev, generator=torch.Generator(device=dev).manual_seed(7))
    a = Trainer(cfg(0), dev)
    assert a.fused_step
    a.train_mode()
    for _ in range(2):
        a.step(batch, epoch=201)
    path = tmp_path / "ck.pt"
    torch.save(a.checkpoint(epoch=4), path)
    b = Trainer(cfg(5), dev)
    b.train_mode()
    assert b.load_checkpoint(torch.load(path, map_location="cpu", weights_only=True)) == 5
    for tr in (a, b):
        torch.manual_seed(99)
        torch.cuda.manual_seed(99)
        tr.step(batch, epoch=201)
    torch.cuda.synchronize(dev)
    sa, sb = _state(a), _state(b)
    bad = [k for k in sa if not torch.equal(sa[k], sb[k])]
    assert not bad, bad[:5]
