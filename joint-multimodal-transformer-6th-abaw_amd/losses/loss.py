"""HIP-backed drop-in for the reference's losses/loss.py (CCCLoss is the training criterion,
main.py:24,794).  No .cuda() in the constructors: the statistics run on the device of the
predictions.  When jmt.dist has a loss group registered (one process per GPU), the CCC is the
global-batch statistic, as under the reference's DataParallel gather."""
import numpy as np
import torch
import torch.nn as nn

from jmt import functional as F
from jmt import dist as jdist


class CCCLoss(nn.Module):
    """loss.py:8-32: 1 - Lin's CCC of x (1,N) vs y (1,N); digitize_num>1: x is (N,k) logits,
    expected value over bins = linspace(range) first."""

    def __init__(self, digitize_num, range=[-1, 1], eps=1e-8):
        super(CCCLoss, self).__init__()
        self.digitize_num = digitize_num
        self.range = range
        self.eps = eps
        if self.digitize_num != 0:
            self.bins = torch.as_tensor(np.linspace(*self.range, num=self.digitize_num),
                                        dtype=torch.float32).view((1, -1))

    def forward(self, x, y):
        return F.ccc_loss(x, y, eps=self.eps, digitize_num=self.digitize_num, rng=self.range,
                          group=jdist.loss_group())

    def forward_add(self, x, y, prev):
        """prev + self(x, y) with the sum formed by the loss's own finish kernel (train.py:311's
        `v_loss + a_loss` as one expression: same value, one fp32 rounding, no add launch)."""
        return F.ccc_loss(x, y, eps=self.eps, digitize_num=self.digitize_num, rng=self.range,
                          group=jdist.loss_group(), add=prev)


class CELoss(nn.Module):
    """loss.py:34-51: cross entropy against labels digitized into `digitize_num` bins
    (np.digitize over linspace(range, digitize_num + 1), top bin clamped) — digitize, weighted
    log-softmax NLL and its gradient in HIP kernels (jmt_ce_*).  A label below range[0] makes the
    reference's F.cross_entropy raise IndexError (bin -1): the statistics kernel counts such
    labels and the call raises IndexError too — at once when eager (one host read, where the
    reference's host digitize synchronises), at the next eager call or
    jmt.functional.check_ce_labels() when the step was replayed from a hipGraph."""

    def __init__(self, digitize_num, range=[-1, 1], weights=None):
        super(CELoss, self).__init__()
        self.digitize_num = digitize_num
        self.range = range
        self.weights = torch.Tensor(weights) if weights is not None else None
        assert self.digitize_num != 1
        self.edges = np.linspace(*range, num=self.digitize_num + 1)

    def forward(self, x, y):
        if self.weights is not None and self.weights.device != x.device:
            self.weights = self.weights.to(x.device)      # once: later calls issue no copy
        return F.ce_loss(x, y.view(-1), self.digitize_num, rng=self.range, weights=self.weights,
                         group=jdist.loss_group())


class CCC_CE_Loss(nn.Module):
    """loss.py:53-66."""

    def __init__(self, digitize_num, range=[-1, 1], alpha=0.5, beta=0.5):
        super(CCC_CE_Loss, self).__init__()
        self.ccc_loss = CCCLoss(digitize_num, range=range)
        self.ce_loss = CELoss(digitize_num, range=range)
        self.alpha = alpha
        self.beta = beta

    def forward(self, x, y):
        cccl = self.ccc_loss(x, y)
        cel = self.ce_loss(x, y)
        return self.alpha * cccl + self.beta * cel
