"""SharedMLP: a stack of pointwise (1x1) conv + BatchNorm + ReLU.

Reference: third_party/pvcnn/modules/shared_mlp.py:6-33.  Parameter names
(layers.{3k}, layers.{3k+1}) match, so reference checkpoints load unchanged.
"""
import torch.nn as nn

__all__ = ["SharedMLP"]

_KINDS = {1: (nn.Conv1d, nn.BatchNorm1d), 2: (nn.Conv2d, nn.BatchNorm2d)}


class SharedMLP(nn.Module):
    def __init__(self, in_channels, out_channels, dim=1):
        super().__init__()
        if dim not in _KINDS:
            raise ValueError(f"SharedMLP: dim must be 1 or 2, got {dim}")
        conv, norm = _KINDS[dim]
        widths = list(out_channels) if isinstance(out_channels, (list, tuple)) else [out_channels]
        stack = []
        prev = in_channels
        for w in widths:
            stack += [conv(prev, w, 1), norm(w), nn.ReLU(True)]
            prev = w
        self.layers = nn.Sequential(*stack)

    def forward(self, inputs):
        # (features, coords, ...) tuples pass the trailing items through untouched
        if isinstance(inputs, (list, tuple)):
            return (self.layers(inputs[0]), *inputs[1:])
        return self.layers(inputs)
