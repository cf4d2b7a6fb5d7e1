"""nn.Module building blocks with the parameter names / shapes / init of their torch
counterparts (so state_dicts round-trip with the reference's `fusion_w.pt`, main.py:105-177),
whose forward runs the HIP kernels of jmt.functional."""
from __future__ import annotations

import math

import torch
from torch import nn

from . import functional as F


class Linear(nn.Module):
    """Drop-in for nn.Linear (weight (out, in), bias (out,), kaiming-uniform init)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.empty(out_features)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1 / math.sqrt(self.in_features) if self.in_features > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x, out_dtype=None):
        return F.linear(x, self.weight, self.bias, out_dtype=out_dtype)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}"


class LayerNorm(nn.Module):
    """Drop-in for nn.LayerNorm(D) (weight, bias, eps=1e-5).  Used fused with the residual add:
    `norm(x, residual)` = LayerNorm(x + residual)."""

    def __init__(self, normalized_shape: int, eps: float = 1e-5):
        super().__init__()
        self.normalized_shape = (normalized_shape,)
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(normalized_shape))
        self.bias = nn.Parameter(torch.zeros(normalized_shape))

    def forward(self, x, residual=None):
        return F.add_layer_norm(x, residual, self.weight, self.bias, self.eps)


class _OutProj(Linear):
    pass


class MultiheadAttention(nn.Module):
    """Drop-in for nn.MultiheadAttention(embed_dim, num_heads) with dropout 0, seq-first inputs
    and the packed `in_proj_weight` / `in_proj_bias` + `out_proj` parameters.  forward returns
    (attn_output, None): the head-averaged weights torch also returns are discarded by every
    reference call site and are not materialised."""

    def __init__(self, embed_dim: int, num_heads: int, dropout: float = 0.0, bias: bool = True):
        super().__init__()
        assert embed_dim % num_heads == 0, "embed_dim must be divisible by num_heads"
        if dropout != 0.0:
            raise NotImplementedError("attention dropout is not on the JMT path (p=0)")
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.head_dim = embed_dim // num_heads
        self.batch_first = False
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * embed_dim))
        self.out_proj = _OutProj(embed_dim, embed_dim, bias=bias)
        self._reset_parameters()

    def _reset_parameters(self):
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.constant_(self.in_proj_bias, 0.0)
        nn.init.constant_(self.out_proj.bias, 0.0)

    def forward(self, query, key, value, key_padding_mask=None, need_weights=True,
                attn_mask=None, average_attn_weights=True, is_causal=False):
        if key_padding_mask is not None or attn_mask is not None or is_causal:
            raise NotImplementedError("masks are not used on the JMT path")
        out = F.multihead_attention(query, key, value, self.in_proj_weight, self.in_proj_bias,
                                    self.out_proj.weight, self.out_proj.bias, self.num_heads)
        return out, None


class MLP(nn.Sequential):
    """Linear-ReLU-[Dropout]-Linear with nn.Sequential indexing (so keys read
    `feed_forward.0.weight` / `vregressor.3.weight`), executed as one fused MLP function."""

    def __init__(self, d_in: int, d_hidden: int, d_out: int, dropout=None):
        mods = [Linear(d_in, d_hidden), nn.ReLU()]
        if dropout is not None:
            mods.append(nn.Dropout(dropout))
        mods.append(Linear(d_hidden, d_out))
        super().__init__(*mods)
        self._p = dropout

    def forward(self, x, out_dtype=None):
        l1, l2 = self[0], self[len(self) - 1]
        if self._p and self.training:
            # dropout p > 0 is off the benchmarked path (config_file.json:69-70 use 0.0)
            h = torch.nn.functional.dropout(l1(x).relu(), self._p, True)
            return l2(h, out_dtype=out_dtype)
        return F.mlp(x, l1.weight, l1.bias, l2.weight, l2.bias, out_dtype=out_dtype)
