"""HIP-backed drop-in for the reference's models/mm_transformers.py (no comet_ml / torchvision /
matplotlib imports: they are unused there, mm_transformers.py:2-18)."""
from __future__ import annotations

import torch.nn as nn

from jmt import functional as F
from jmt import grouped
from jmt import streams
from jmt import taps
from jmt.nn import Linear

from .mm_multi_transformers import (Attention, SequentialEncoder, TransformerEncoderBlock,
                                    TransformerEncoderLayer)
from .mm_multi_transformers import MultiheadAttention

__all__ = ["Attention", "SequentialEncoder", "TransformerEncoderBlock",
           "TransformerEncoderLayer", "MultimodalTransformer_wo_JR"]


class MultimodalTransformer_wo_JR(nn.Module):
    """JMT without joint representation, mm_transformers.py:87-146.

    The encoders receive (B, T, D) directly, i.e. self-attention runs over the BATCH axis
    (seq = B, batch = T) exactly as in the reference (:120-122); the cross-attentions permute to
    (T, B, D) (:125-135).  `gated_attention` is constructed and unused (:103)."""

    def __init__(self, visual_dim, audio_dim, num_heads, hidden_dim, num_layers,
                 output_format: str):
        super().__init__()
        assert output_format in ['FC'], output_format
        self.output_format = output_format
        self.visual_encoder = TransformerEncoderBlock(visual_dim, num_heads, hidden_dim,
                                                      num_layers)
        self.physiological_encoder = TransformerEncoderBlock(audio_dim, num_heads, hidden_dim,
                                                             num_layers)
        self.cross_attention_v = MultiheadAttention(visual_dim, num_heads)
        self.cross_attention_p = MultiheadAttention(audio_dim, num_heads)
        self.gated_attention = Linear(visual_dim + audio_dim, 1)
        self.final_layer = Linear(1024, 512)

    def forward(self, visual_features, physiological_features):
        if grouped.enabled() and visual_features.shape == physiological_features.shape:
            return self._forward_grouped(visual_features, physiological_features)
        dev = visual_features.device
        v, p = streams.run_parallel([lambda: self.visual_encoder(visual_features),
                                     lambda: self.physiological_encoder(physiological_features)],
                                    dev)
        taps.record("enc.visual_encoder", v)
        taps.record("enc.physiological_encoder", p)
        vt, pt = v.permute(1, 0, 2), p.permute(1, 0, 2)
        ov, op = streams.run_parallel([lambda: self.cross_attention_v(vt, pt, pt)[0],
                                       lambda: self.cross_attention_p(pt, vt, vt)[0]], dev)
        ov, op = ov.permute(1, 0, 2), op.permute(1, 0, 2)
        taps.record("ca.0", ov)
        taps.record("ca.1", op)
        assert self.output_format == 'FC', self.output_format
        return F.linear((ov, op), self.final_layer.weight, self.final_layer.bias)

    def _forward_grouped(self, visual_features, physiological_features):
        """Same math as forward(), the two branches batched (jmt/grouped.py): the encoders of
        both streams as one grouped layer sequence on a stacked (2, B, T, E) buffer (their
        self-attention over the batch axis, :120-122), the two cross-attentions over T as one
        grouped block (:125-135), final_layer on the concatenation as one K-concatenated GEMM
        (:139-144)."""
        X = grouped.stack_groups(visual_features, physiological_features)
        for lv, lp in zip(self.visual_encoder.layers, self.physiological_encoder.layers):
            X = grouped.encoder_group(X, [lv, lp], lv.attention.num_heads, batch_axis=True)
        taps.record_stacked(["enc.visual_encoder", "enc.physiological_encoder"], X)
        O2 = grouped.cross_attention6(X, [self.cross_attention_v, self.cross_attention_p],
                                      self.cross_attention_v.num_heads,
                                      pairs=grouped.CROSS_PAIRS_WO_JR)
        taps.record_stacked(["ca.0", "ca.1"], O2)
        return grouped.concat_linear(O2, self.final_layer.weight, self.final_layer.bias)
