"""Run the voxel-conv kernels at the bench's R32/C128 shape a few times (for a
rocprofv3 --pmc pass).  Dev tool: python tools/conv_pmc.py [iters]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "point-cloud-flow-matching_amd")]
from pcfm import ops  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 3
b, c, r = 8, 128, 32
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(b, c, r, r, r, device="cuda", generator=g)
w = torch.randn(c, c, 3, 3, 3, device="cuda", generator=g) * (1.0 / (27 * c) ** 0.5)
gy = torch.randn(b, c, r, r, r, device="cuda", generator=g)
xs, gys = ops.conv3d_split(x), ops.conv3d_split(gy)
img = ops.conv3d_prep_weight(w, False)
for _ in range(it):
    ops.conv3d_igemm_split(xs, img, None, b, c, c, r, "fwd")
    ops.conv3d_wgrad_split(xs, gys, b, c, c, r)
torch.cuda.synchronize()
