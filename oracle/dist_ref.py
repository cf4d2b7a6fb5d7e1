"""CPU restatement of the data-parallel CCC of the HIP path (TEST INFRASTRUCTURE ONLY).

Mirrors, in torch fp64/fp32 CPU math, what jmt_ccc_stats / jmt_ccc_finish compute on the GPU:
rank-local sufficient statistics (n, mean_x, mean_y, M2x, M2y, Cxy), combined exactly in fixed
rank order with Chan et al.'s pairwise update, so that the loss over sharded ranks equals
losses/loss.py:18-32 evaluated on the DataParallel-gathered batch."""
from __future__ import annotations

import torch


def local_stats(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    x = x.reshape(-1).double()
    y = y.reshape(-1).double()
    n = x.numel()
    mx, my = x.mean(), y.mean()
    dx, dy = x - mx, y - my
    return torch.stack([torch.tensor(float(n), dtype=torch.float64), mx, my, (dx * dx).sum(),
                        (dy * dy).sum(), (dx * dy).sum()])


def chan_combine(stats: torch.Tensor) -> torch.Tensor:
    """stats: (world, 6) -> (6,) global (n, mean_x, mean_y, Sxx, Syy, Sxy)."""
    n, mx, my, sxx, syy, sxy = [stats[0, i] for i in range(6)]
    for r in range(1, stats.shape[0]):
        nb, mxb, myb, sxxb, syyb, sxyb = [stats[r, i] for i in range(6)]
        nt = n + nb
        dx, dy = mxb - mx, myb - my
        f = n * nb / nt
        sxx = sxx + sxxb + dx * dx * f
        syy = syy + syyb + dy * dy * f
        sxy = sxy + sxyb + dx * dy * f
        mx = mx + dx * nb / nt
        my = my + dy * nb / nt
        n = nt
    return torch.stack([n, mx, my, sxx, syy, sxy])


def ccc_loss_from_stats(g: torch.Tensor, eps: float = 1e-8) -> torch.Tensor:
    """losses/loss.py:23-32 from global statistics."""
    n, mx, my, sxx, syy, sxy = [g[i] for i in range(6)]
    rho = sxy / (torch.sqrt(sxx) * torch.sqrt(syy) + eps)
    xs = torch.sqrt(sxx / (n - 1))
    ys = torch.sqrt(syy / (n - 1))
    ccc = 2 * rho * xs * ys / (xs * xs + ys * ys + (mx - my) ** 2)
    return 1 - ccc


def global_ccc_loss_local(x_local: torch.Tensor, y_local: torch.Tensor,
                          all_stats: torch.Tensor, rank: int) -> torch.Tensor:
    """Differentiable in x_local: the global loss with this rank's statistics recomputed from
    x_local (so autograd gives exactly this rank's share of the global gradient) and the other
    ranks' statistics as constants."""
    mine = local_stats(x_local, y_local)
    rows = [mine if r == rank else all_stats[r].detach() for r in range(all_stats.shape[0])]
    return ccc_loss_from_stats(chan_combine(torch.stack(rows)))
