"""HIP-backed drop-in for the reference's models/intra_modal_transformer_fusion.py."""
from __future__ import annotations

import torch.nn as nn

from jmt import functional as F
from jmt.nn import Linear, MultiheadAttention

from .mm_multi_transformers import (Attention, SequentialEncoder, TransformerEncoderBlock,
                                    TransformerEncoderLayer)

__all__ = ["Attention", "SequentialEncoder", "TransformerEncoderBlock",
           "TransformerEncoderLayer", "Intra_modal_transformer_fusion"]


class Intra_modal_transformer_fusion(nn.Module):
    """intra_modal_transformer_fusion.py:74-111: optional shared fc 768->512 on each input,
    stack the two backbones as a length-2 sequence per (b, t), encoder block, MHA, keep the last
    token.  Only the last query row of the final attention is computed (the only one kept,
    :108)."""

    def __init__(self, feat_dim, num_heads, hidden_dim, num_layers, reduce_dim_for_audio=False):
        super().__init__()
        self.final_visual_encoder = TransformerEncoderBlock(feat_dim, num_heads, hidden_dim,
                                                            num_layers)
        self.final_self_attention = MultiheadAttention(512, num_heads)
        self.fc = Linear(768, 512)

    def forward(self, features_a, features_b):
        if features_a.shape[-1] == 768:
            features_a = self.fc(features_a)
        if features_b.shape[-1] == 768:
            features_b = self.fc(features_b)
        B, T, E = features_a.shape
        st = F.stack_seq((features_a, features_b), seq_first_in=False)    # (2, B*T, E)
        enc = self.final_visual_encoder(st)
        last = enc[-1:]
        fa, _ = self.final_self_attention(last, enc, enc)
        return fa[0].reshape(B, T, E)
