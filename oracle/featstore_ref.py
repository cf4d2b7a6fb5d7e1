"""CPU restatement (oracle) of the reference's in-loop wavLM feature assembly.  TEST
INFRASTRUCTURE ONLY (imported by tests/).

train.py:150-171: for each sample i and each clip of its window, the clip's feature file
<root>/<video>/<k>.npy (create_wavlm_audio_feat.py:7-33 layout) is np.load-ed if it exists;
otherwise the previously loaded vector is re-used (`feat_numpy` keeps its value across clips and
samples); the vectors are stacked into the window's (T, D) block.  `None` entries (padding clips,
padSequence.py:14-21) give zero rows here.  Parity unpinned by the reference's own tests (it has
none); pinned by this line-by-line restatement over real .npy files in tests/test_featstore.py."""
import os

import numpy as np


def window_feats(root, clips, state, dim):
    """clips[b][t] = (video, clip number) or None -> (B, T, dim) float32."""
    B = len(clips)
    T = max(len(r) for r in clips)
    out = np.zeros((B, T, dim), dtype=np.float32)
    for b, row in enumerate(clips):
        for t, c in enumerate(row):
            if c is None:
                continue
            p = os.path.join(root, c[0], f"{c[1]}.npy")
            if os.path.exists(p):
                state["feat_numpy"] = np.load(p)
            if "feat_numpy" not in state:
                raise KeyError("no feature loaded yet (NameError in the reference)")
            out[b, t] = state["feat_numpy"]
    return out
