"""Validation post-processing oracle (oracle/valpost_ref.py) pinned on CPU: ccc against the
reference's own EvaluationMetrics/cccmetric.py outputs (tests/golden/valpost.npz), the
uniform_filter1d window convention, and the scatter semantics of val.py:313-357 on hand cases."""
import os

import numpy as np
import pytest
from scipy.ndimage import uniform_filter1d

from oracle import valpost_ref as V

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "valpost.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


@pytest.mark.parametrize("tag", ["rand", "corr", "f32", "smallvar", "n2"])
def test_ccc_matches_reference(gold, tag):
    got = V.ccc(gold[tag + "/x"], gold[tag + "/y"])
    assert abs(got - float(gold[tag + "/ccc"])) <= 1e-12 * max(1.0, abs(got))


def test_ccc_identical_is_one_and_va(gold):
    x = np.linspace(-1, 1, 101)
    assert abs(V.ccc(x, x) - 1.0) < 1e-12          # cccmetric.py:81-89 self-check
    yt, yp = gold["va/true"], gold["va/pred"]
    cv, ca = V.ccc(yt[:, 0], yp[:, 0]), V.ccc(yt[:, 1], yp[:, 1])
    np.testing.assert_allclose([cv, ca, (cv + ca) / 2], gold["va/ccc"], rtol=1e-12)


@pytest.mark.parametrize("size", [20, 50, 7])
def test_uniform_filter_window_convention(size):
    """mode='constant', origin 0: window [i - size//2, i - size//2 + size) with zeros outside —
    the convention csrc/valpost.hip implements."""
    rng = np.random.default_rng(size)
    x = rng.uniform(-1.5, 1.5, 233)
    got = uniform_filter1d(np.clip(x, -1, 1), size=size, mode="constant")
    c = np.clip(x, -1, 1)
    ref = np.array([sum(c[t] for t in range(i - size // 2, i - size // 2 + size)
                        if 0 <= t < len(c)) / size for i in range(len(c))])
    np.testing.assert_allclose(got, ref, atol=1e-12)


def test_scatter_semantics_hand_case():
    st = V.ValState()
    # one window of video "a" (length 6): frame 1..4, frame 3 twice (last wins), frame 2 ignored
    st.update(vouts=[[0.1, 0.2, 0.3, 0.35, 0.4]], aouts=[[1.1, 1.2, 1.3, 1.35, 1.4]],
              labelsV=[[0.5, -5.0, 0.7, 0.75, 0.8]], labelsA=[[0.6, 0.6, 0.6, 0.65, 0.6]],
              frame_ids=[[1, 2, 3, 3, 4]], videos=[["a"] * 5], vid_lengths=[[6] * 5])
    assert st.pred_v["a"] == [0.1, 0, 0.35, 0.4, 0, 0]
    assert st.label_a["a"] == [0.6, 0, 0.65, 0.6, 0, 0]
    # frame id 0 -> Python index -1 (last element); frame id > length skipped
    st.update(vouts=[[0.9, 0.8]], aouts=[[0.9, 0.8]], labelsV=[[0.1, 0.2]], labelsA=[[0.1, 0.2]],
              frame_ids=[[0, 9]], videos=[["a", "a"]], vid_lengths=[[6, 6]])
    assert st.pred_v["a"][-1] == 0.9 and len(st.pred_v["a"]) == 6
    with pytest.raises(ValueError):
        st.update(vouts=[[0.1]], aouts=[[0.1]], labelsV=[[0.1]], labelsA=[[0.1]],
                  frame_ids=[[5]], videos=[["new"]], vid_lengths=[[9]])
