"""GPU: the per-points plan caches (pcfm.plans) give exactly what recomputing
gives -- here the voxel-grid coordinates, whose resolution-independent [0, 1]
part is shared by the stages' voxelizations of the same points."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    from pcfm import _lib, ops
    _lib.load()
    return ops


@pytest.mark.parametrize("normalize,eps", [(True, 0.0), (True, 1e-6), (False, 0.0)])
def test_grid_coords_shared_across_resolutions_bit_identical(ops, normalize, eps):
    from modules.voxelization import Voxelization
    from pcfm import plans
    g = torch.Generator(device="cuda").manual_seed(7)
    coords = torch.randn(4, 3, 5000, device="cuda", generator=g) * 0.7
    for r in (32, 16, 8):
        vox = Voxelization(r, normalize=normalize, eps=eps)
        norm, vc = plans.grid_coords(vox, coords)
        # the reference's sequence of torch ops, recomputed (voxelization.py:18-28)
        c = coords - coords.mean(2, keepdim=True)
        if normalize:
            u = c / (c.norm(dim=1, keepdim=True).max(dim=2, keepdim=True).values * 2.0 + eps) + 0.5
        else:
            u = (c + 1) / 2.0
        ref = torch.clamp(u * r, 0, r - 1)
        assert torch.equal(norm, ref)
        assert torch.equal(vc, torch.round(ref).to(torch.int32))
        assert plans.grid_coords(vox, coords)[0] is norm  # cached per resolution
