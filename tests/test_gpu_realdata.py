"""The real-data shape path: T = 16 clips per window (config_file.json:14-15,
512/32), intra-modal fusion 'encoder_plus_self_attention' for vision (R2D1 + I3D, 512 each) and
audio (ResNet18 512 + wavLM 768 through the shared 768->512 fc; train.py:193-198, 250-255), then
Two_transformers(TRANSFORMER, FC, vision_in_ft=512) + 2x CCCLoss — HIP modules vs the CPU oracle
(oracle/jmt_ref.py, pinned by the reference goldens).  fp32: 1e-4 on predictions / losses, 1e-3 on
gradients; bf16: the 16-bit error model of tests/parity.py (min(5 %, K_STRICT x the error of the oracle with
bf16 storage emulated, floor u x the prediction spread)."""
import pytest
import torch

from jmt import functional as JF
from oracle import jmt_ref as R
from oracle.hashinit import init_module_

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _build():
    from models.intra_modal_transformer_fusion import Intra_modal_transformer_fusion
    from models.two_transformers import Two_transformers
    vis = Intra_modal_transformer_fusion(512, 1, 512, 1)
    aud = Intra_modal_transformer_fusion(512, 1, 512, 1, reduce_dim_for_audio=True)
    tt = Two_transformers(0.0, 0.0, 1, 1, "TRANSFORMER", "FC", 512)
    init_module_(vis, "vis.")
    init_module_(aud, "aud.")
    init_module_(tt, "rd.")
    return vis.to(DEV), aud.to(DEV), tt.to(DEV)


def _inputs(B=4, T=16):
    g = torch.Generator().manual_seed(16)
    r2d1, i3d, res18 = (torch.randn(B, T, 512, generator=g) for _ in range(3))
    wavlm = torch.randn(B, T, 768, generator=g)
    lv = torch.rand(B, T, generator=g) * 2 - 1
    la = torch.rand(B, T, generator=g) * 2 - 1
    return r2d1, i3d, res18, wavlm, lv, la


def _oracle(vis, aud, tt, xs):
    r2d1, i3d, res18, wavlm, lv, la = xs
    pv = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in vis.state_dict().items()}
    pa = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in aud.state_dict().items()}
    pt = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in tt.state_dict().items()}
    B, T = lv.shape
    visual = R.intra_modal_forward(r2d1, i3d, pv, "", 1, 1)
    audio = R.intra_modal_forward(res18, wavlm, pa, "", 1, 1)
    vo, ao = R.two_transformers_forward(audio, visual, pt, 1, 1, "TRANSFORMER", "FC", 512)
    loss = R.ccc_loss(vo.reshape(1, -1), lv.reshape(1, -1)) + \
        R.ccc_loss(ao.reshape(1, -1), la.reshape(1, -1))
    loss.backward()
    return vo.detach(), ao.detach(), float(loss), pv, pt


@pytest.mark.parametrize("cd", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_realdata_shape_path_vs_oracle(cd):
    from losses.loss import CCCLoss
    vis, aud, tt = _build()
    xs = _inputs()
    r2d1, i3d, res18, wavlm, lv, la = xs
    B, T = lv.shape
    crit = CCCLoss(1)
    with JF.compute_mode(cd):
        visual = vis(r2d1.to(DEV), i3d.to(DEV))
        audio = aud(res18.to(DEV), wavlm.to(DEV))
        vo, ao = tt(audio, visual)
        loss = crit(vo.view(-1, B * T), lv.to(DEV).view(-1, B * T)) + \
            crit(ao.view(-1, B * T), la.to(DEV).view(-1, B * T))
        loss.backward()
    rvo, rao, rloss, pv, pt = _oracle(vis, aud, tt, xs)
    assert vo.shape == rvo.shape == (T, B)
    if cd == torch.float32:
        scale = max(1.0, float(rvo.abs().max()))
        assert float((vo.cpu() - rvo).abs().max()) <= 1e-4 * scale
        assert float((ao.cpu() - rao).abs().max()) <= 1e-4 * scale
        assert abs(float(loss) - rloss) <= 1e-4
        for name, mod, ref in (("final_visual_encoder.layers.0.attention.in_proj_weight", vis, pv),
                               ("fc.weight", vis, pv),
                               ("mm_transformer.out_layer1.weight", tt, pt),
                               ("mm_transformer.cross_attention_pv.in_proj_weight", tt, pt)):
            g = dict(mod.named_parameters())[name].grad
            r = ref[name].grad
            if r is None:
                assert g is None or float(g.abs().max()) == 0.0
                continue
            err = float((g.cpu() - r).abs().max())
            assert err <= 1e-3 * max(1e-6, float(r.abs().max())) + 1e-7, (name, err)
    else:
        # strict 16-bit bound (tests/parity.py): errors relative to the largest |prediction|
        # (loss: to the loss), within min(5 %, K_STRICT x the rounding-emulating oracle's)
        from tests.parity import CEIL, K_STRICT, UNIT
        with R.emulate_storage(cd):
            evo, eao, eloss, _, _ = _oracle(vis, aud, tt, xs)
        bnd = lambda e: min(CEIL[cd]["out"], K_STRICT * max(e, 2 * UNIT[cd]))
        mx = float(max(rvo.abs().max(), rao.abs().max()))
        for got, emu, ref in ((vo, evo, rvo), (ao, eao, rao)):
            e_gpu = float((got.float().cpu() - ref).abs().max()) / mx
            e_emu = float((emu - ref).abs().max()) / mx
            assert e_gpu <= bnd(e_emu), (e_gpu, e_emu)
        e_gpu, e_emu = abs(float(loss) - rloss) / abs(rloss), abs(eloss - rloss) / abs(rloss)
        assert e_gpu <= bnd(e_emu), (float(loss), rloss, eloss)
