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


# biases of convolutions that feed a BatchNorm: analytically zero gradient, so
# what the reference stores for them is rounding noise (|g| ~ 1e-9)
NOISE_BIAS = ("layers.0.bias", "voxel_layers.0.bias", "voxel_layers.3.bias")


def grad_errors_full(module, fixture):
    """pvconv_r8_grads.npz: {param: max |g - g_ref| / max |g_ref|} over every element."""
    import numpy as np
    out = {}
    for n, p in module.named_parameters():
        ref = fixture[f"grad/{n}"]
        got = p.grad.detach().cpu().numpy()
        out[n] = float(np.abs(got - ref).max() / max(float(np.abs(ref).max()), 1e-30))
    return out


def grad_errors_sampled(module, fixture, elements=False):
    """model_hybrid_c1_perturbed_grads.npz: {param: max |g - g_ref| / max |g_ref|}
    over the fixture's seeded positions, normalised by the parameter's max
    |gradient| over all its elements (stored beside the samples).  With
    `elements`, also the array of every sampled element's normalised error."""
    import numpy as np
    names = list(fixture["param_names"])
    params = dict(module.named_parameters())
    assert names == list(params), "parameter order differs from the reference's"
    of, pos, ref, amax = (fixture["param_of"], fixture["flat_pos"], fixture["grad"],
                          fixture["grad_absmax"])
    out, el = {}, []
    for i, n in enumerate(names):
        sel = of == i
        g = params[n].grad
        flat = (g.detach().reshape(-1).cpu().numpy() if g is not None
                else np.zeros(int(params[n].numel()), np.float32))
        e = np.abs(flat[pos[sel]] - ref[sel]) / max(float(amax[i]), 1e-30)
        out[n] = float(e.max())
        if not n.endswith(NOISE_BIAS):
            el.append(e)
    return (out, np.concatenate(el)) if elements else out


def worst(errs, skip=NOISE_BIAS):
    """(max error, its parameter) over the live parameters."""
    live = {k: v for k, v in errs.items() if not k.endswith(skip)}
    k = max(live, key=live.get)
    return live[k], k
