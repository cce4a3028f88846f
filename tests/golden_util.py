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
