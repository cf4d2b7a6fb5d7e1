"""GPU validation post-processing (jmt/valpost.py, csrc/valpost.hip) vs the CPU restatement of
val.py:313-382 (oracle/valpost_ref.py) on synthetic validation batches: overlapping windows
(last writer wins), -5.0 labels, frames past a video's end, the seq-first (T, B) pairing quirk of
the TRANSFORMER/FC head.  Tolerance 1e-6 abs on CCC and smoothed predictions (float64 on the GPU;
the reference's arrays are float32 or float64 depending on whether a zero slot remains)."""
import numpy as np
import pytest
import torch

from jmt.valpost import VideoAccumulator
from oracle import valpost_ref as V

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _batches(seed, nbatch=6, B=4, T=64):
    rng = np.random.default_rng(seed)
    lengths = {f"vid{k}": int(rng.integers(150, 400)) for k in range(5)}
    names = list(lengths)
    started = set()
    out = []
    for _ in range(nbatch):
        fids = np.zeros((B, T), dtype=np.int64)
        vids = []
        lens = np.zeros((B, T), dtype=np.int64)
        for b in range(B):
            v = names[int(rng.integers(0, len(names)))]
            start = 1 if v not in started else int(rng.integers(1, lengths[v] - 20))
            started.add(v)
            fids[b] = start + np.arange(T)             # may run past the video's end
            vids.append([v] * T)
            lens[b] = lengths[v]
        lv = rng.uniform(-1, 1, (B, T)).astype(np.float32)
        la = rng.uniform(-1, 1, (B, T)).astype(np.float32)
        lv[rng.random((B, T)) < 0.05] = -5.0
        la[rng.random((B, T)) < 0.05] = -5.0
        pv = rng.normal(0, 0.7, (B, T)).astype(np.float32)
        pa = rng.normal(0, 0.7, (B, T)).astype(np.float32)
        out.append((pv, pa, lv, la, fids, vids, lens))
    return out


@pytest.mark.parametrize("seq_first", [False, True], ids=["BT", "TB_quirk"])
def test_video_accumulator_matches_oracle(seq_first):
    ref = V.ValState()
    acc = VideoAccumulator(DEV)
    for pv, pa, lv, la, fids, vids, lens in _batches(5 if seq_first else 4):
        if seq_first:                 # the FC head's (T, B) predictions paired with (B, T) labels
            pv, pa = pv.T.copy(), pa.T.copy()
        ref.update(pv, pa, lv, la, fids, vids, lens)
        acc.update(torch.from_numpy(pv).to(DEV), torch.from_numpy(pa).to(DEV),
                   torch.from_numpy(lv), torch.from_numpy(la), fids, vids, lens)
    av, aa, smooth = ref.finalize(20, 50)
    gv, ga, per = acc.finalize(20, 50, return_smoothed=True)
    assert abs(gv - av) < 1e-6 and abs(ga - aa) < 1e-6, (gv, av, ga, aa)
    assert list(per) == list(ref.pred_v)                      # same videos, same order
    for k, (sv, sa) in smooth.items():
        np.testing.assert_allclose(per[k]["pred_v"], sv, atol=1e-6)
        np.testing.assert_allclose(per[k]["pred_a"], sa, atol=1e-6)
        np.testing.assert_array_equal(per[k]["label_v"], np.asarray(ref.label_v[k], np.float64))
        np.testing.assert_array_equal(per[k]["label_a"], np.asarray(ref.label_a[k], np.float64))


def test_video_accumulator_hand_case():
    acc = VideoAccumulator(DEV)
    acc.update(torch.tensor([[0.1, 0.2, 0.3, 0.35, 0.4]], device=DEV),
               torch.tensor([[1.1, 1.2, 1.3, 1.35, 1.4]], device=DEV),
               torch.tensor([[0.5, -5.0, 0.7, 0.75, 0.8]]), torch.tensor([[0.6, 0.6, 0.6, 0.65, 0.6]]),
               [[1, 2, 3, 3, 4]], [["a"] * 5], [[6] * 5])
    acc.update(torch.tensor([[0.9, 0.8]], device=DEV), torch.tensor([[0.9, 0.8]], device=DEV),
               torch.tensor([[0.1, 0.2]]), torch.tensor([[0.1, 0.2]]), [[0, 9]], [["a", "a"]],
               [[6, 6]])
    pv = acc.buf[0, :6].cpu().numpy()
    np.testing.assert_array_equal(pv, np.array([0.1, 0, 0.35, 0.4, 0, 0.9], np.float32).astype(np.float64))
