"""HIP-backed drop-in for the reference's models/mm_multi_transformers.py.

Same class names, constructor signatures, submodule names (hence state_dict keys) and forward
semantics as the reference (file:line cited per class); every op runs on libjmt_hip.so kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from jmt import functional as F
from jmt import grouped
from jmt import streams
from jmt import taps
from jmt.nn import Linear, LayerNorm, MLP, MultiheadAttention

__all__ = ["Attention", "SequentialEncoder", "TransformerEncoderBlock",
           "TransformerEncoderLayer", "MultimodalTransformer_w_JR", "FeatureConcatFC"]


class Attention(nn.Module):
    """Unused by the reference's models (mm_multi_transformers.py:7-26); kept for API parity."""

    def __init__(self, input_dim):
        super().__init__()
        self.W = Linear(input_dim, input_dim)
        self.V = Linear(input_dim, input_dim, bias=False)
        self.tanh = nn.Tanh()
        self.fc = Linear(input_dim, 2)
        self.out_layer1 = Linear(512, 256)
        self.out_layer2 = Linear(256, 64)
        self.out_layer3 = Linear(64, 2)

    def forward(self, x):
        # mm_multi_transformers.py:19-26: additive attention weights over dim 1, then the
        # 512 -> 256 -> 64 -> 2 projection chain (the linears on the HIP GEMM; tanh / softmax /
        # the weighting are torch elementwise ops on this never-called path)
        q = self.W(x)
        attn_weights = torch.softmax(self.V(torch.tanh(q)), dim=1)
        attended_x = attn_weights * x
        return self.out_layer3(self.out_layer2(self.out_layer1(attended_x)))


class SequentialEncoder(nn.Sequential):
    """mm_multi_transformers.py:29-33."""

    def forward(self, x):
        for module in self._modules.values():
            x = module(x)
        return x


class TransformerEncoderLayer(nn.Module):
    """Post-LN encoder layer, mm_multi_transformers.py:48-70:
    x = LN1(x + MHA(x, x, x)); x = LN2(x + W2 relu(W1 x + b1) + b2)."""

    def __init__(self, input_dim, num_heads, hidden_dim):
        super().__init__()
        self.attention = MultiheadAttention(input_dim, num_heads)
        self.feed_forward = MLP(input_dim, hidden_dim, input_dim)
        self.layer_norm1 = LayerNorm(input_dim)
        self.layer_norm2 = LayerNorm(input_dim)

    def forward(self, x):
        if grouped.enabled() and x.dim() == 3 and x.dtype == F.compute_dtype() and \
                x.permute(1, 0, 2).is_contiguous():
            # seq-first view of a (N, L, E) buffer (the SELF_ATTEN head's token stack, the
            # ungrouped encoders): the grouped layer with one group — its backward accumulates
            # the residual and projection input gradients in place (no autograd gradient sums)
            Y = grouped.encoder_group(x.permute(1, 0, 2).unsqueeze(0), [self],
                                      self.attention.num_heads)
            return Y.squeeze(0).permute(1, 0, 2)
        attn_output, _ = self.attention(x, x, x)
        x = self.layer_norm1(x, attn_output)
        ff_output = self.feed_forward(x)
        return self.layer_norm2(x, ff_output)


class TransformerEncoderBlock(nn.Module):
    """mm_multi_transformers.py:36-45."""

    def __init__(self, input_dim, num_heads, hidden_dim, num_layers):
        super().__init__()
        self.layers = SequentialEncoder(
            *[TransformerEncoderLayer(input_dim, num_heads, hidden_dim) for _ in range(num_layers)])

    def forward(self, x):
        return self.layers(x)


class MultimodalTransformer_w_JR(nn.Module):
    """JMT with joint representation, mm_multi_transformers.py:73-214.

    forward(visual (B,T,512), physiological (B,T,512)):
      FC head         -> (T, B, 1024) seq-first (the reference's layout quirk, kept)
      SELF_ATTEN head -> (B, T, 512)
    `final_encoder` (E=3072) is constructed and never called, as in the reference (:92-93)."""

    def __init__(self, visual_dim, audio_dim, num_heads, hidden_dim, num_layers,
                 output_format: str):
        super().__init__()
        assert output_format in ["FC", "SELF_ATTEN"], output_format
        self.output_format = output_format
        self.num_heads = num_heads
        self.visual_encoder = TransformerEncoderBlock(visual_dim, num_heads, hidden_dim,
                                                      num_layers)
        self.physiological_encoder = TransformerEncoderBlock(audio_dim, num_heads, hidden_dim,
                                                             num_layers)
        self.joint_representation_encoder = TransformerEncoderBlock(audio_dim, num_heads,
                                                                    hidden_dim, num_layers)
        self.final_encoder = TransformerEncoderBlock(3072, num_heads, hidden_dim, num_layers)
        self.cross_attention_v = MultiheadAttention(visual_dim, num_heads)
        self.cross_attention_p = MultiheadAttention(audio_dim, num_heads)
        self.cross_attention_pv = MultiheadAttention(512, num_heads)
        self.out_layer_pv = Linear(1024, 512)
        if output_format == "FC":
            self.out_layer1 = Linear(3072, 1024)
        elif output_format == "SELF_ATTEN":
            self.final_visual_encoder = TransformerEncoderBlock(visual_dim, num_heads, hidden_dim,
                                                                num_layers)
            self.final_self_attention = MultiheadAttention(512, num_heads)
        else:
            raise NotImplementedError(output_format)

    def forward(self, visual_features, physiological_features):
        if grouped.enabled() and visual_features.shape == physiological_features.shape:
            return self._forward_grouped(visual_features, physiological_features)
        # cat + out_layer_pv as ONE K-concatenated GEMM (:120-124)
        joint_representation = F.linear((visual_features, physiological_features),
                                        self.out_layer_pv.weight, self.out_layer_pv.bias)
        v = visual_features.permute(1, 0, 2)          # free: a strided view (:127-129)
        p = physiological_features.permute(1, 0, 2)
        j = joint_representation.permute(1, 0, 2)
        dev = visual_features.device
        # the three encoders are independent: concurrent streams (:132-136)
        v, p, j = streams.run_parallel([lambda: self.visual_encoder(v),
                                        lambda: self.physiological_encoder(p),
                                        lambda: self.joint_representation_encoder(j)], dev)
        taps.record("enc.visual_encoder", v, True)
        taps.record("enc.physiological_encoder", p, True)
        taps.record("enc.joint_representation_encoder", j, True)

        # six cross-attentions (:142-167, key is value in every call); each module is applied
        # to the same query twice, so its query projection is computed once
        def ca(mod, query, keys):
            return F.multihead_attention_shared_query(
                query, keys, mod.in_proj_weight, mod.in_proj_bias, mod.out_proj.weight,
                mod.out_proj.bias, mod.num_heads)

        r_v, r_p, r_pv = streams.run_parallel(
            [lambda: ca(self.cross_attention_v, v, (p, j)),
             lambda: ca(self.cross_attention_p, p, (v, j)),
             lambda: ca(self.cross_attention_pv, j, (v, p))], dev)
        outs = [r_v[0],      # CA_v(v, p)
                r_p[0],      # CA_p(p, v)
                r_pv[0],     # CA_pv(j, v)
                r_v[1],      # CA_v(v, j)
                r_pv[1],     # CA_pv(j, p)
                r_p[1]]      # CA_p(p, j)
        for i, o in enumerate(outs):
            taps.record(f"ca.{i}", o, True)
        if self.output_format == "SELF_ATTEN":
            return self._self_atten_head(outs)
        # FC head (:201-211): torch.cat of the 6 outputs never materialised (K-concat GEMM)
        return F.linear(tuple(outs), self.out_layer1.weight, self.out_layer1.bias)

    def _forward_grouped(self, visual_features, physiological_features):
        """Same math, batched across the parallel branches (jmt/grouped.py): the three streams
        in one stacked (3, B, T, E) buffer — out_layer_pv's K-concatenated GEMM (:120-124)
        writing the joint representation into its third slot — each encoder layer of the three
        encoders as one grouped launch sequence, the six cross-attentions as one (:132-167)."""
        X = grouped.stack_joint(visual_features, physiological_features,
                                self.out_layer_pv.weight, self.out_layer_pv.bias)
        for lv, lp, lj in zip(self.visual_encoder.layers, self.physiological_encoder.layers,
                              self.joint_representation_encoder.layers):
            X = grouped.encoder_group(X, [lv, lp, lj], self.num_heads)
        taps.record_stacked(["enc.visual_encoder", "enc.physiological_encoder",
                             "enc.joint_representation_encoder"], X)
        O6 = grouped.cross_attention6(X, [self.cross_attention_v, self.cross_attention_p,
                                          self.cross_attention_pv], self.num_heads)
        taps.record_stacked([f"ca.{i}" for i in range(O6.shape[0])], O6)
        if self.output_format == "SELF_ATTEN":
            S, B, T, E = O6.shape
            enc = self.final_visual_encoder(grouped.stack_tokens(O6))
            return grouped.last_query_mha(enc, self.final_self_attention).reshape(B, T, E)
        # FC head (:201-211): seq-first (T, B, 1024), as the reference returns it
        return grouped.concat_linear(O6, self.out_layer1.weight,
                                     self.out_layer1.bias).permute(1, 0, 2)

    def _self_atten_head(self, outs):
        # :169-199 — stack to (6, B*T, 512), encoder over the 6-token sequences, MHA, keep
        # token 5.  Only the last query row of the final attention is computed: it is the
        # only one the reference keeps ([:, :, -1, :], :193).
        T, B, E = outs[0].shape
        st = F.stack_seq(outs, seq_first_in=True)
        enc = self.final_visual_encoder(st)
        return grouped.last_query_mha(enc, self.final_self_attention).reshape(B, T, E)


class FeatureConcatFC(nn.Module):
    """mm_multi_transformers.py:217-224: fc(cat(v, a))."""

    def __init__(self, visual_dim, audio_dim):
        super().__init__()
        self.fc = Linear(visual_dim + audio_dim, 512)

    def forward(self, visual_features, audio_features):
        return F.linear((visual_features, audio_features), self.fc.weight, self.fc.bias)
