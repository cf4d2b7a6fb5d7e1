"""GPU validation post-processing: the per-video scatter, clipping,
uniform_filter1d smoothing and CCC of the reference's validate() (val.py:313-382,
EvaluationMetrics/cccmetric.py:4-21), without the per-frame Python loop and the per-batch
device-to-host copy of the predictions (val.py:307-311).

    acc = VideoAccumulator()
    for batch in loader:                        # the same arguments val.py zips over
        vouts, aouts = fusion_model(aud, vis)
        acc.update(vouts, aouts, labelsV, labelsA, frame_ids, videos, vid_lengths)
    accV, accA = acc.finalize()                 # sizes 20 (valence) / 50 (arousal), val.py:366-367

Reference semantics reproduced (val.py:313-357): the two nested zip()s over the first and second
axes of the seven arguments (so a seq-first (T, B) prediction is paired exactly as the reference
pairs it, truncated to the shorter axis); a video's arrays are created at its first appearance
with that entry's `vid_length` and zero-filled; frames whose valence or arousal label is -5.0 are
skipped; later hits of a (video, frame) overwrite earlier ones; frame ids index the arrays with
Python's list semantics (frame id 0 -> last element).  The reference aborts the process when a new
video starts at frame id > 1 (val.py:321-325); here that raises ValueError.

The host side only maps video names to segment offsets (one dict lookup per distinct name);
the per-frame work runs in libjmt_hip.so (csrc/valpost.hip).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .ops import stream


def _rows(x) -> List:
    """First-axis items of a tensor / array / nested sequence."""
    return [x[i] for i in range(len(x))]


def _as_tensor(x, dev) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.detach().to(dev, torch.float32)
    return torch.as_tensor(np.asarray(x, dtype=np.float32), device=dev)


class VideoAccumulator:
    def __init__(self, device=None, ignore: float = -5.0):
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.ignore = float(ignore)
        self.vids: Dict[object, int] = {}       # name -> id, in first-appearance order
        self.off: List[int] = []
        self.seglen: List[int] = []
        self.total = 0
        self.cap = 0
        self.buf: Optional[torch.Tensor] = None      # (4, cap) float64: pred_v, pred_a, lab_v, lab_a
        self.winner: Optional[torch.Tensor] = None   # (cap,) uint64 (int64 storage)
        self.seq = 0
        self._tabs = None

    # ---------------------------------------------------------------- segments
    def _grow(self, need: int):
        if need <= self.cap:
            return
        cap = max(need, 2 * self.cap, 1 << 14)
        buf = torch.zeros(4, cap, dtype=torch.float64, device=self.device)
        win = torch.zeros(cap, dtype=torch.int64, device=self.device)
        if self.buf is not None:
            buf[:, :self.cap].copy_(self.buf)
            win[:self.cap].copy_(self.winner)
        self.buf, self.winner, self.cap = buf, win, cap

    def _register(self, name, length: int, frameid: int):
        if frameid > 1:
            raise ValueError(f"video {name!r} starts at frame id {frameid} > 1 "
                             "(the reference exits here, val.py:321-325)")
        self.vids[name] = len(self.off)
        self.off.append(self.total)
        self.seglen.append(int(length))
        self.total += int(length)
        self._tabs = None

    def _tables(self):
        if self._tabs is None:
            self._tabs = (torch.tensor(self.off, dtype=torch.int64, device=self.device),
                          torch.tensor(self.seglen, dtype=torch.int32, device=self.device))
        return self._tabs

    # ---------------------------------------------------------------- update
    def update(self, vouts, aouts, labelsV, labelsA, frame_ids, videos, vid_lengths):
        """One validation batch, arguments exactly as zipped at val.py:313-315."""
        outer = [_rows(a) for a in (vouts, aouts, labelsV, labelsA, frame_ids, videos,
                                    vid_lengths)]
        n_outer = min(len(o) for o in outer)
        if n_outer == 0:
            return
        inner = [min(len(o[i]) for o in outer) for i in range(n_outer)]
        rect = all(n == inner[0] for n in inner)
        # host: names / frame ids / lengths of the zipped iteration, in its order
        names, fids, lens = [], [], []
        for i in range(n_outer):
            k = inner[i]
            names.extend(list(outer[5][i])[:k])
            fids.extend(np.asarray(outer[4][i]).reshape(-1)[:k].tolist())
            lens.extend(np.asarray(outer[6][i]).reshape(-1)[:k].tolist())
        n = len(names)
        if n == 0:
            return
        vid = np.empty(n, dtype=np.int32)
        for j, name in enumerate(names):      # one dict lookup per frame, new videos in order
            v = self.vids.get(name)
            if v is None:
                self._register(name, lens[j], int(fids[j]))
                v = self.vids[name]
            vid[j] = v
        self._grow(self.total)
        dev = self.device
        if rect:
            k = inner[0]
            vals = [_as_tensor(a, dev)[:n_outer, :k].reshape(-1).contiguous()
                    for a in (vouts, aouts, labelsV, labelsA)]
        else:
            vals = [torch.cat([_as_tensor(a[i], dev).reshape(-1)[:inner[i]]
                               for i in range(n_outer)]).contiguous()
                    for a in (vouts, aouts, labelsV, labelsA)]
        host = torch.from_numpy(np.stack([np.asarray(fids, dtype=np.int32),
                                          np.asarray(lens, dtype=np.int32), vid]))
        ints = host.to(dev, non_blocking=False)
        off_t, len_t = self._tables()
        b = self.buf
        _lib.call("jmt_vp_scatter", n, ints[0].data_ptr(), ints[1].data_ptr(),
                  ints[2].data_ptr(), off_t.data_ptr(), len_t.data_ptr(),
                  vals[0].data_ptr(), vals[1].data_ptr(), vals[2].data_ptr(), vals[3].data_ptr(),
                  self.ignore, self.seq, self.winner.data_ptr(), b[0].data_ptr(),
                  b[1].data_ptr(), b[2].data_ptr(), b[3].data_ptr(), stream())
        self.seq += n
        self._keep = (ints, vals)             # alive until the launches are ordered

    # ---------------------------------------------------------------- finalize
    def smoothed(self, size_v: int = 20, size_a: int = 50) -> torch.Tensor:
        """(2, total) float64: clipped + uniform_filter1d'd valence / arousal predictions."""
        off_t, len_t = self._tables()
        out = torch.empty(2, max(self.total, 1), dtype=torch.float64, device=self.device)
        for r, size in ((0, size_v), (1, size_a)):
            _lib.call("jmt_vp_smooth", self.total, len(self.off), off_t.data_ptr(),
                      len_t.data_ptr(), self.buf[r].data_ptr(), int(size), out[r].data_ptr(),
                      stream())
        return out

    def finalize(self, size_v: int = 20, size_a: int = 50, return_smoothed: bool = False):
        """(accV, accA) = ccc(smoothed predictions, labels) over all videos (val.py:359-382)."""
        if self.total <= 1:
            raise ValueError("ccc needs at least 2 frames (cccmetric.py:9-11 exits)")
        sm = self.smoothed(size_v, size_a)
        res = torch.empty(2, dtype=torch.float64, device=self.device)
        _lib.call("jmt_vp_ccc", self.total, sm[0].data_ptr(), self.buf[2].data_ptr(),
                  sm[1].data_ptr(), self.buf[3].data_ptr(), res.data_ptr(), stream())
        accV, accA = (float(v) for v in res.cpu())
        if not return_smoothed:
            return accV, accA
        smc = sm.cpu().numpy()
        lab = self.buf[2:4, :self.total].cpu().numpy()
        per = {}
        for name, v in self.vids.items():
            o, L = self.off[v], self.seglen[v]
            per[name] = {"pred_v": smc[0, o:o + L], "pred_a": smc[1, o:o + L],
                         "label_v": lab[0, o:o + L], "label_a": lab[1, o:o + L]}
        return accV, accA, per
