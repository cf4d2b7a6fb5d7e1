"""CPU restatement (oracle) of the reference's validation post-processing.  TEST INFRASTRUCTURE
ONLY (imported by tests/ as the checker; the product path is jmt/valpost.py + csrc/valpost.hip).

Restates, loop for loop, val.py:313-357 (per-video scatter of per-frame predictions and labels,
-5.0 labels skipped, Python list semantics), val.py:359-382 (np.clip, uniform_filter1d with
size 20 / 50 and mode='constant', concatenation in dict order, ccc) and
EvaluationMetrics/cccmetric.py:4-21 (ccc).  uniform_filter1d is scipy.ndimage's — the reference's
own dependency (val.py imports it), present in this image; its window convention is pinned by
tests/test_valpost.py.  Pinned: `ccc` against values produced by importing the reference's
EvaluationMetrics/cccmetric.py (tests/golden/make_golden_valpost.py -> tests/golden/valpost.npz).
"""
from __future__ import annotations

import numpy as np
from scipy.ndimage import uniform_filter1d

IGNORE = -5.0


def ccc(x, y):
    """cccmetric.py:4-21 (population std, no epsilon)."""
    if len(y) <= 1:
        raise ValueError("ccc needs at least 2 values (the reference calls sys.exit())")
    vx = x - np.mean(x)
    vy = y - np.mean(y)
    rho = np.sum(vx * vy) / (np.sqrt(np.sum(vx ** 2)) * np.sqrt(np.sum(vy ** 2)))
    x_m = np.mean(x)
    y_m = np.mean(y)
    x_s = np.std(x)
    y_s = np.std(y)
    return 2 * rho * x_s * y_s / ((x_s ** 2 + y_s ** 2 + (x_m - y_m) ** 2))


class ValState:
    """The four dicts of val.py:313-357 (insertion-ordered)."""

    def __init__(self):
        self.pred_v, self.pred_a, self.label_v, self.label_a = {}, {}, {}, {}

    def update(self, vouts, aouts, labelsV, labelsA, frame_ids, videos, vid_lengths):
        """val.py:313-357 with numpy inputs (the reference's .cpu().numpy() arrays)."""
        for voutputs, aoutputs, labelV, labelA, frameids, video, vid_length in zip(
                vouts, aouts, labelsV, labelsA, frame_ids, videos, vid_lengths):
            for voutput, aoutput, labV, labA, frameid, vid, length in zip(
                    voutputs, aoutputs, labelV, labelA, frameids, video, vid_length):
                if vid not in self.pred_a:
                    if frameid > 1:
                        raise ValueError("new video at frame id > 1 (reference exits)")
                    self.pred_a[vid] = [0] * length
                    self.pred_v[vid] = [0] * length
                    self.label_a[vid] = [0] * length
                    self.label_v[vid] = [0] * length
                    if labA == IGNORE or labV == IGNORE:
                        continue
                    self._put(vid, frameid, voutput, aoutput, labV, labA)
                else:
                    if frameid <= length:
                        if labA == IGNORE or labV == IGNORE:
                            continue
                        self._put(vid, frameid, voutput, aoutput, labV, labA)

    def _put(self, vid, frameid, voutput, aoutput, labV, labA):
        try:
            self.pred_a[vid][frameid - 1] = aoutput
            self.pred_v[vid][frameid - 1] = voutput
            self.label_a[vid][frameid - 1] = labA
            self.label_v[vid][frameid - 1] = labV
        except IndexError:      # the reference would raise; the GPU path skips the frame
            pass

    def finalize(self, size_v=20, size_a=50):
        """val.py:359-382: returns (accV, accA, per-video smoothed predictions)."""
        vout, aout, vtar, atar = [], [], [], []
        smooth = {}
        for key in self.pred_a.keys():
            sv = uniform_filter1d(np.clip(self.pred_v[key], -1.0, 1.0), size=size_v,
                                  mode='constant')
            sa = uniform_filter1d(np.clip(self.pred_a[key], -1.0, 1.0), size=size_a,
                                  mode='constant')
            smooth[key] = (sv, sa)
            for i in range(len(sa)):
                vout.append(sv[i])
                aout.append(sa[i])
                vtar.append(self.label_v[key][i])
                atar.append(self.label_a[key][i])
        return ccc(np.array(vout), np.array(vtar)), ccc(np.array(aout), np.array(atar)), smooth
