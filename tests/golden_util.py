"""Helpers shared by the golden-fixture tests."""
import torch


def perturb_zero_init_(module, seed: int = 5, std: float = 0.05) -> None:
    """Same as tests/golden/make_golden.py:perturb_zero_init_ -- every all-zero
    parameter gets seeded N(0, std^2) values, in named_parameters order (at the
    reference's initialisation ContextNet.head_out is zero, so v would not see
    the PVConv pyramid)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for _, p in module.named_parameters():
            if not bool(p.detach().abs().sum()):
                p.copy_(torch.randn(p.shape, generator=g) * std)


def grid_sample_devox(grid, pts, r):
    """trilinear_devox.cu:21-80 as F.grid_sample(align_corners=True): the grid
    index is x*r*r + y*r + z, i.e. (D, H, W) = (x, y, z), and grid_sample's last
    coordinate axis is (W, H, D) = (z, y, x), normalised from [0, r-1] to [-1, 1]."""
    import torch
    import torch.nn.functional as TF
    b, c = grid.shape[:2]
    g = grid.reshape(b, c, r, r, r)
    p = pts.permute(0, 2, 1).flip(-1) * (2.0 / (r - 1)) - 1.0      # (b, n, 3) as (z, y, x)
    out = TF.grid_sample(g, p.reshape(b, 1, 1, -1, 3), mode="bilinear",
                         padding_mode="border", align_corners=True)
    return out.reshape(b, c, -1)
