"""Generation on the HIP path (pcfm/sample.py): runs, is finite, and the GPU
Chamfer metric equals the reference's cdist formula (train.py:80-84)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_chamfer_l2_gpu_matches_cdist():
    from pcfm.sample import chamfer_l2
    g = torch.Generator(device="cuda").manual_seed(0)
    a = torch.randn(3, 1000, 3, device="cuda", generator=g)
    b = torch.randn(3, 800, 3, device="cuda", generator=g)
    d2 = torch.cdist(a.double(), b.double()).pow(2)
    exp = d2.min(2).values.mean(1) + d2.min(1).values.mean(1)
    torch.testing.assert_close(chamfer_l2(a, b).double(), exp, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("method,amp", [("heun", False), ("dopri5_fixed", True)])
def test_generate_gpu(method, amp):
    from pcfm.sample import generate
    from pcfm.train import TrainConfig, build_models
    torch.manual_seed(0)
    cfg = TrainConfig(batch_size=2, num_points=2000)
    _, pf, lf = build_models(cfg, "cuda")
    pf.eval()
    lf.eval()
    cond = torch.rand(2, cfg.cond_dim, device="cuda")
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        x, nfe = generate(pf, lf, 2, 2000, point_dim=6, latent_dim=cfg.latent_dim, cond=cond,
                          steps=3, method=method, guidance_scale=1.0)
    assert x.shape == (2, 2000, 6) and torch.isfinite(x).all()
    assert nfe == (6 if method == "heun" else 1 + 3 * 6)
