"""HIP-backed drop-in for the reference's models/fc_layer.py (FcLayer, :6-12)."""
import torch.nn as nn

from jmt.nn import Linear

__all__ = ['FcLayer']


class FcLayer(nn.Module):
    """One linear projection, used as (512+768)->512, 768->512 and 1024->512 (main.py:318,360,379)."""

    def __init__(self, input_dim, output_dim):
        super(FcLayer, self).__init__()
        self.fc_layer = Linear(input_dim, output_dim)

    def forward(self, x):
        return self.fc_layer(x)
