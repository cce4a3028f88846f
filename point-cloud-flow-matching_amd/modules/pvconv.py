"""PVConv: point-voxel convolution block.

Reference: third_party/pvcnn/modules/pvconv.py:11-39.  Voxelize (gfx950 scatter
kernel) -> two Conv3d/BN3d/LeakyReLU(0.1) stages (+ SE; the 3x3x3 convs run on
the bf16x3 matrix-core kernels of modules/voxel_conv.py) -> trilinear
devoxelize (gfx950 gather kernel) -> + pointwise SharedMLP branch.  Modules are
created in the reference's order, so a given torch seed yields the same
initial weights, and the state_dict keys (voxel_layers.{0,1,3,4,6.fc.*},
point_features.layers.*) are the reference's.
"""
import torch.nn as nn

import modules.functional as F
from modules.norm_act import conv_bn_act
from modules.se import SE3d
from modules.shared_mlp import SharedMLP
from modules.voxel_conv import VoxelConv3d
from modules.voxelization import Voxelization

__all__ = ["PVConv"]


def _conv_bn_lrelu(cin, cout, kernel_size):
    return [
        VoxelConv3d(cin, cout, kernel_size, stride=1, padding=kernel_size // 2),
        nn.BatchNorm3d(cout, eps=1e-4),
        nn.LeakyReLU(0.1, True),
    ]


class PVConv(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, resolution, with_se=False,
                 normalize=True, eps=0):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = kernel_size
        self.resolution = resolution
        self.voxelization = Voxelization(resolution, normalize=normalize, eps=eps)
        stages = _conv_bn_lrelu(in_channels, out_channels, kernel_size)
        stages += _conv_bn_lrelu(out_channels, out_channels, kernel_size)
        if with_se:
            stages.append(SE3d(out_channels))
        self.voxel_layers = nn.Sequential(*stages)
        self.point_features = SharedMLP(in_channels, out_channels)

    def forward(self, inputs):
        features, coords = inputs
        grid, grid_coords = self.voxelization(features, coords)
        layers = self.voxel_layers  # Conv3d, BN3d, LeakyReLU, Conv3d, BN3d, LeakyReLU[, SE3d]
        grid = conv_bn_act(layers[0], layers[1], grid, layers[2].negative_slope)
        grid = conv_bn_act(layers[3], layers[4], grid, layers[5].negative_slope)
        if len(layers) > 6:
            grid = layers[6](grid)
        voxel_branch = F.trilinear_devoxelize(grid, grid_coords, self.resolution, self.training)
        return voxel_branch + self.point_features(features), coords
