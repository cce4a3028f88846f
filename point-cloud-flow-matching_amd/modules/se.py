"""Squeeze-and-excitation over a voxel grid.  Reference:
third_party/pvcnn/modules/se.py:6-17 (parameter names fc.0 / fc.2 kept)."""
import torch.nn as nn

__all__ = ["SE3d"]


class SE3d(nn.Module):
    def __init__(self, channel, reduction=8):
        super().__init__()
        hidden = channel // reduction
        self.fc = nn.Sequential(
            nn.Linear(channel, hidden, bias=False),
            nn.ReLU(inplace=True),
            nn.Linear(hidden, channel, bias=False),
            nn.Sigmoid(),
        )

    def forward(self, inputs):
        b, c = inputs.shape[0], inputs.shape[1]
        pooled = inputs.mean(-1).mean(-1).mean(-1)  # same reduction order as the reference
        return inputs * self.fc(pooled).view(b, c, 1, 1, 1)
