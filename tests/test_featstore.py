"""Feature store host logic (jmt/featstore.py) vs the restatement of train.py:150-171
(oracle/featstore_ref.py) on a real <video>/<k>.npy tree with missing files and padding."""
import os

import numpy as np
import pytest

from jmt.featstore import FeatureStore, FeatureStoreWriter
from oracle import featstore_ref as FR

DIM = 40


def make_tree(tmp, seed=0):
    rng = np.random.default_rng(seed)
    lengths = {"vidA": 9, "vidB": 6, "vidC": 12}
    for v, n in lengths.items():
        os.makedirs(os.path.join(tmp, v), exist_ok=True)
        for k in range(1, n + 1):
            if (v, k) in {("vidA", 4), ("vidB", 1), ("vidC", 7), ("vidC", 8)}:
                continue                                   # missing feature files
            np.save(os.path.join(tmp, v, f"{k}.npy"), rng.normal(size=DIM).astype(np.float32))
    return lengths


def batches():
    return [
        [[("vidA", k) for k in range(1, 7)], [None, None] + [("vidB", k) for k in range(1, 5)]],
        [[("vidC", k) for k in range(4, 10)], [("vidA", k) for k in range(3, 9)]],
        [[("vidB", k) for k in range(1, 7)], [("vidC", k) for k in range(7, 13)]],
    ]


def test_store_window_rows_match_reference_loop(tmp_path):
    root = str(tmp_path / "npy")
    lengths = make_tree(root)
    store_dir = str(tmp_path / "store")
    FeatureStoreWriter.from_npy_tree(store_dir, root, "wavlm", DIM, dtype="float32",
                                     lengths=lengths)
    fs = FeatureStore(store_dir, device="cpu")
    table = fs.tables["wavlm"][:, :DIM].numpy()
    state, last = {}, None
    for clips in batches():
        ref = FR.window_feats(root, clips, state, DIM)
        rows, last = fs.window_rows("wavlm", clips, last)
        got = np.where(rows[..., None] >= 0, table[np.maximum(rows, 0)], 0.0)
        np.testing.assert_array_equal(got, ref)


def test_missing_first_clip_raises(tmp_path):
    root = str(tmp_path / "npy")
    lengths = make_tree(root)
    store_dir = str(tmp_path / "store")
    FeatureStoreWriter.from_npy_tree(store_dir, root, "wavlm", DIM, lengths=lengths)
    fs = FeatureStore(store_dir, device="cpu")
    with pytest.raises(KeyError):
        fs.window_rows("wavlm", [[("vidB", 1)]])
    with pytest.raises(KeyError):
        FR.window_feats(root, [[("vidB", 1)]], {}, DIM)


def test_default_store_is_fp32_exact(tmp_path):
    """The reference loads the wavLM features as fp32 np.load values (train.py:157-158): the
    default store keeps them bit-exact (fp16 storage is an explicit opt-in)."""
    root = str(tmp_path / "npy")
    lengths = make_tree(root)
    store_dir = str(tmp_path / "store")
    FeatureStoreWriter.from_npy_tree(store_dir, root, "wavlm", DIM, lengths=lengths)
    fs = FeatureStore(store_dir, device="cpu")
    table = fs.tables["wavlm"]
    assert table.dtype.is_floating_point and table.element_size() == 4
    rows, _ = fs.window_rows("wavlm", [[("vidA", k) for k in (1, 2, 3)]])
    for j, k in enumerate((1, 2, 3)):
        ref = np.load(os.path.join(root, "vidA", f"{k}.npy"))
        np.testing.assert_array_equal(table[int(rows[0, j]), :DIM].numpy(), ref)
