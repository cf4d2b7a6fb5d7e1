"""HBM feature-store gather (csrc/gather.hip) vs the numpy gather of the same table rows and vs
the restatement of train.py:150-171: exact for float32 tables, conversion-exact to bf16/f16."""
import numpy as np
import pytest
import torch

from jmt.featstore import FeatureStore, FeatureStoreWriter
from oracle import featstore_ref as FR
from tests.test_featstore import DIM, batches, make_tree

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("table_dtype", ["float32", "float16"])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_gather_matches_reference(tmp_path, table_dtype, out_dtype):
    root = str(tmp_path / "npy")
    lengths = make_tree(root, seed=1)
    sd = str(tmp_path / "store")
    FeatureStoreWriter.from_npy_tree(sd, root, "wavlm", DIM, dtype=table_dtype, lengths=lengths)
    fs = FeatureStore(sd, device="cuda")
    state, last = {}, None
    for clips in batches():
        ref = FR.window_feats(root, clips, state, DIM)
        rows, last = fs.window_rows("wavlm", clips, last)
        got = fs.gather("wavlm", rows, out_dtype)
        torch.cuda.synchronize()
        exp = torch.from_numpy(ref)
        if table_dtype == "float16":
            exp = exp.half().float()
        exp = exp.to(out_dtype)
        assert torch.equal(got.cpu(), exp), float((got.float().cpu() - exp.float()).abs().max())


def test_gather_large_rows_bandwidth_shape():
    """A (64, 16, 768) bf16 window batch from a 50k-row table: exact copy of the selected rows."""
    g = torch.Generator().manual_seed(0)
    table = torch.randn(50000, 768, generator=g).bfloat16().cuda()
    idx = torch.randint(-1, 50000, (64, 16), generator=g)
    from jmt import _lib
    from jmt.ops import dt, stream
    out = torch.empty(64, 16, 768, dtype=torch.bfloat16, device="cuda")
    idx_d = idx.cuda()
    _lib.call("jmt_gather_rows", dt(table), dt(out), 64 * 16, 768, table.data_ptr(), 768,
              table.shape[0], idx_d.data_ptr(), out.data_ptr(), 768, stream())
    ref = torch.where(idx[..., None] >= 0, table.cpu()[idx.clamp(min=0)],
                      torch.zeros((), dtype=torch.bfloat16))
    assert torch.equal(out.cpu(), ref)
