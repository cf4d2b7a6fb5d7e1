"""HIP-backed drop-in for the reference's models/two_transformers.py."""
from __future__ import annotations

from typing import Tuple

import torch
from torch import nn

from jmt import functional as F
from jmt import taps
from jmt.nn import Linear, MLP

from .mm_multi_transformers import MultimodalTransformer_w_JR
from .mm_multi_transformers import FeatureConcatFC
from .mm_transformers import MultimodalTransformer_wo_JR

__all__ = ['Two_transformers', 'SingleBackbonePretrainer']


class Two_transformers(nn.Module):
    """two_transformers.py:17-128.  forward(f1_norm=audio, f2_norm=video) -> (vouts, aouts),
    (T, B) for TRANSFORMER/FC and (B, T) otherwise — the reference's layouts, reproduced."""

    def __init__(self, v_dropout: float, a_dropout: float, num_heads: int, num_layers: int,
                 joint_modalities: str, output_format: str = 'FC', vision_in_ft: int = 512,
                 digitize_num: int = 1):
        super(Two_transformers, self).__init__()
        assert isinstance(v_dropout, float), type(v_dropout)
        assert 0.0 <= v_dropout < 1., v_dropout
        self.v_dropout = v_dropout
        assert isinstance(a_dropout, float), type(a_dropout)
        assert 0.0 <= a_dropout < 1., a_dropout
        self.a_dropout = a_dropout
        assert isinstance(num_heads, int), type(num_heads)
        assert num_heads > 0, num_heads
        self.num_heads = num_heads
        assert isinstance(num_layers, int), type(num_layers)
        assert num_layers > 0, num_layers
        self.num_layers = num_layers
        assert isinstance(joint_modalities, str), type(joint_modalities)
        assert joint_modalities in ['NONE', 'TRANSFORMER', 'FC'], joint_modalities
        self.joint_modalities = joint_modalities
        assert isinstance(vision_in_ft, int), type(vision_in_ft)
        assert vision_in_ft > 0, vision_in_ft
        self.vision_in_ft = vision_in_ft

        self.linear = None
        if vision_in_ft != 512:
            self.linear = Linear(vision_in_ft, 512)

        assert output_format in ['FC', 'SELF_ATTEN'], output_format
        self.output_format = output_format

        if joint_modalities == 'TRANSFORMER':
            self.mm_transformer = MultimodalTransformer_w_JR(
                visual_dim=512, audio_dim=512, num_heads=num_heads, hidden_dim=512,
                num_layers=num_layers, output_format=output_format)
            dim = 1024 if output_format == 'FC' else 512
        elif joint_modalities == 'FC':
            self.mm_transformer = FeatureConcatFC(512, 512)
            dim = 512
        elif joint_modalities == 'NONE':
            assert output_format in ['FC'], output_format
            self.mm_transformer = MultimodalTransformer_wo_JR(
                visual_dim=512, audio_dim=512, num_heads=num_heads, hidden_dim=512,
                num_layers=num_layers, output_format=output_format)
            dim = 512
        else:
            raise NotImplementedError(joint_modalities)

        # digitize_num = 1: the reference's V/A regressors (two_transformers.py:104-114).
        # digitize_num = k > 1 (an extra keyword, default off): the same MLPs emit k bin logits
        # per clip — the expression-style head SURVEY.md §8d maps configs[4] to, trained with
        # losses.loss.CCCLoss(digitize_num=k) (loss.py:14-22) on the (N, k) rows
        assert isinstance(digitize_num, int) and 1 <= digitize_num <= 64, digitize_num
        self.digitize_num = digitize_num
        self.vregressor = MLP(dim, 128, digitize_num, dropout=v_dropout)
        self.aregressor = MLP(dim, 128, digitize_num, dropout=a_dropout)

    def forward(self, f1_norm, f2_norm):
        video = F.l2_normalize(f2_norm)          # :118
        audio = F.l2_normalize(f1_norm)          # :119
        if self.linear is not None:
            video = self.linear(video)           # :120-121
        av = self.mm_transformer(video, audio)
        taps.record("head", av, self.joint_modalities == 'TRANSFORMER' and
                    self.output_format == 'FC')
        # regressors in fp32 out (predictions feed the fp32 CCC statistics)
        vr, ar = self.vregressor, self.aregressor
        if (F.pair_mlps_enabled() and not ((vr._p or ar._p) and self.training)
                and vr[0].weight.shape == ar[0].weight.shape):
            # both regressors read av: one MLP-pair function (fewer launches, same arithmetic
            # per output element as the two MLP calls below)
            vouts, aouts = F.mlp_pair(av, vr, ar, out_dtype=torch.float32)
            vouts, aouts = vouts.squeeze(2), aouts.squeeze(2)
        else:
            vouts = vr(av, out_dtype=torch.float32).squeeze(2)
            aouts = ar(av, out_dtype=torch.float32).squeeze(2)
        if vouts.dim() == 2 and not vouts.is_contiguous():   # seq-first (T,B) -> contiguous
            vouts = F.TransposeCopyFn.apply(vouts)
            aouts = F.TransposeCopyFn.apply(aouts)
        return vouts, aouts


class SingleBackbonePretrainer(nn.Module):
    """two_transformers.py:131-162 (PRETRAINING goal only)."""

    def __init__(self, v_dropout: float, a_dropout: float):
        super(SingleBackbonePretrainer, self).__init__()
        assert isinstance(v_dropout, float), type(v_dropout)
        assert 0.0 <= v_dropout < 1., v_dropout
        self.v_dropout = v_dropout
        assert isinstance(a_dropout, float), type(a_dropout)
        assert 0.0 <= a_dropout < 1., a_dropout
        self.a_dropout = a_dropout
        self.regressor = MLP(512, 128, 2, dropout=a_dropout)

    def forward(self, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        assert x.ndim == 3, x.ndim
        out = self.regressor(x, out_dtype=torch.float32)
        return out[:, :, 0], out[:, :, 1]
