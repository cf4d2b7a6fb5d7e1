"""HIP-backed drop-in for the reference's losses/CCCLoss.py (ignore-masked CCC)."""
import torch.nn as nn

from jmt import functional as F
from jmt import dist as jdist


class CCCLoss(nn.Module):
    """Lin's Concordance correlation coefficient with an ignore label (CCCLoss.py:4-43).

    Labels equal to `ignore` are masked (bit-exact compare on device); <= 1 surviving element
    gives a zero loss; note the reference's swapped std names and its division by the pre-mask
    y_pred.size(0) — both reproduced."""

    def __init__(self, ignore=-5.0):
        super(CCCLoss, self).__init__()
        self.ignore = ignore

    def forward(self, y_pred, y_true):
        return F.ccc_loss_ignore(y_pred, y_true, ignore=self.ignore, group=jdist.loss_group())
