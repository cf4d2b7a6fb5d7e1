"""Host-side logic of the drop-in modules that needs no GPU: module/class identity, constructor
signatures, state_dict keys and shapes identical to the reference, layout bookkeeping."""
import inspect
import os

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

import pytest
import torch

from jmt import functional as F
from jmt import dist as jdist
from oracle import jmt_ref as R


def _keys_shapes(m):
    return {k: tuple(v.shape) for k, v in m.state_dict().items()}


@pytest.mark.parametrize("jm,fmt,vin,L", [("TRANSFORMER", "FC", 2048, 1),
                                          ("TRANSFORMER", "SELF_ATTEN", 2048, 2),
                                          ("NONE", "FC", 2048, 1), ("FC", "FC", 512, 1)])
def test_two_transformers_state_dict_matches_reference(jm, fmt, vin, L):
    from models.two_transformers import Two_transformers
    m = Two_transformers(0.0, 0.0, 1, L, jm, fmt, vin)
    assert _keys_shapes(m) == R.two_transformers_shapes(L, jm, fmt, vin)


def test_golden_key_sets_cover_our_params(golden):
    from models.two_transformers import Two_transformers
    m = Two_transformers(0.0, 0.0, 8, 2, "TRANSFORMER", "FC", 2048)
    gkeys = {k.split("/", 1)[1].rsplit(":", 1)[0] for k in golden
             if k.startswith("tr_fc_h8l2/") and k.endswith(":norm")}
    ours = set(m.state_dict())
    assert ours <= gkeys


def test_intra_modal_state_dict():
    from models.intra_modal_transformer_fusion import Intra_modal_transformer_fusion
    m = Intra_modal_transformer_fusion(512, 1, 512, 1)
    assert _keys_shapes(m) == R.intra_modal_shapes(512, 1)


def test_constructor_signatures_match_reference():
    from models.two_transformers import Two_transformers
    from models.mm_multi_transformers import MultimodalTransformer_w_JR, FeatureConcatFC
    from models.mm_transformers import MultimodalTransformer_wo_JR
    from models.intra_modal_transformer_fusion import Intra_modal_transformer_fusion
    from models.fc_layer import FcLayer
    from losses.loss import CCCLoss, CELoss, CCC_CE_Loss
    from losses.CCCLoss import CCCLoss as CCCLossIgnore
    sig = lambda c: list(inspect.signature(c.__init__).parameters)[1:]
    # the reference's positional parameters in order; the one extra (digitize_num: configs[4]'s
    # expression-style head) comes after them with a default that keeps the reference behaviour
    assert sig(Two_transformers) == ["v_dropout", "a_dropout", "num_heads", "num_layers",
                                     "joint_modalities", "output_format", "vision_in_ft",
                                     "digitize_num"]
    assert inspect.signature(Two_transformers.__init__).parameters["digitize_num"].default == 1
    assert sig(MultimodalTransformer_w_JR) == ["visual_dim", "audio_dim", "num_heads",
                                               "hidden_dim", "num_layers", "output_format"]
    assert sig(MultimodalTransformer_wo_JR) == sig(MultimodalTransformer_w_JR)
    assert sig(FeatureConcatFC) == ["visual_dim", "audio_dim"]
    assert sig(Intra_modal_transformer_fusion) == ["feat_dim", "num_heads", "hidden_dim",
                                                   "num_layers", "reduce_dim_for_audio"]
    assert sig(FcLayer) == ["input_dim", "output_dim"]
    assert sig(CCCLoss) == ["digitize_num", "range", "eps"]
    assert sig(CELoss) == ["digitize_num", "range", "weights"]
    assert sig(CCC_CE_Loss) == ["digitize_num", "range", "alpha", "beta"]
    assert sig(CCCLossIgnore) == ["ignore"]


def test_constructor_asserts_like_reference():
    from models.two_transformers import Two_transformers
    with pytest.raises(AssertionError):
        Two_transformers(0, 0.0, 1, 1, "TRANSFORMER")        # v_dropout must be a float
    with pytest.raises(AssertionError):
        Two_transformers(0.0, 0.0, 1, 1, "BOGUS")
    with pytest.raises(AssertionError):
        Two_transformers(0.0, 0.0, 1, 1, "NONE", "SELF_ATTEN")


def test_hash_init_applies_to_our_modules():
    from models.two_transformers import Two_transformers
    from oracle.hashinit import init_module_, param_value
    m = Two_transformers(0.0, 0.0, 1, 1, "TRANSFORMER", "FC", 2048)
    init_module_(m, "")
    w = m.mm_transformer.out_layer1.weight.detach().numpy()
    assert (w == param_value("mm_transformer.out_layer1.weight", w.shape)).all()


def test_rows_layout_of_permuted_views():
    x = torch.zeros(4, 7, 16)          # (B, T, E) memory
    v = x.permute(1, 0, 2)             # (T, B, E) seq-first view
    L = F.Rows(v)
    assert L.rows == 28 and L.ld == 16 and L.perm == [1, 0] and L.t.data_ptr() == x.data_ptr()
    y = L.like(8, torch.float32)
    assert y.shape == (7, 4, 8) and y.permute(1, 0, 2).is_contiguous()
    # (S, B*T, E) view of a (B*T, S, E) buffer (the SELF_ATTEN stack) and its last-token slice
    buf = torch.zeros(6, 3, 16)
    s = buf.permute(1, 0, 2)
    last = s[-1:]
    Ll = F.Rows(last)
    assert Ll.rows == 6 and Ll.ld == 48
    # a non-collapsible view falls back to a copy
    assert F.Rows(torch.zeros(4, 6, 16)[:, ::2]).ld == 32   # uniform row stride: no copy
    nc = torch.zeros(4, 6, 16)[:, :3]
    Ln = F.Rows(nc)
    assert Ln.ld == 16 and Ln.t.is_contiguous()


def test_shard_range_matches_dataparallel_scatter():
    # torch.nn.DataParallel scatters dim 0 in chunks of ceil(B / g)
    for B, g in [(64, 8), (64, 3), (10, 4)]:
        chunks = torch.arange(B).chunk(g)
        for r in range(g):
            lo, hi = jdist.shard_range(B, r, g)
            ref = chunks[r] if r < len(chunks) else torch.arange(0)
            assert list(range(lo, hi)) == ref.tolist()


def test_compute_dtype_policy():
    assert F.compute_dtype() == torch.float32
    with F.compute_mode(torch.bfloat16):
        assert F.compute_dtype() == torch.bfloat16
    assert F.compute_dtype() == torch.float32


def test_bench_synthetic_batches_identical_across_world_sizes():
    """bench.py's per-global-window generators: 2 ranks x 3 windows == 1 rank x 6 windows."""
    import importlib
    import sys
    sys.path.insert(0, REPO_ROOT)
    bench = importlib.import_module("bench")
    one = bench.synthetic_batch(6, 5, 8, 16, 0, "cpu")
    two = [bench.synthetic_batch(3, 5, 8, 16, r, "cpu") for r in range(2)]
    for k in range(2):                                    # audio, video
        assert torch.equal(one[k], torch.cat([two[0][k], two[1][k]], 0))
    for k in range(2, 4):                                 # labels (1, B*T)
        assert torch.equal(one[k].view(6, 5), torch.cat([t[k].view(3, 5) for t in two], 0))
