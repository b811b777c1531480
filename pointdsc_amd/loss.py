"""Drop-in ``SpectralMatchingLoss`` (libs/loss.py:115-139 of AmnonDrory/PointDSC),
forward only, on the gfx950 reduction kernels of ``libpdsc.so`` (fp64 sums).

Used by the reference's validation loop (libs/trainer.py:237) on the ``M`` that
``PointDSC.forward`` returns without the 'testing' key.  There is no autograd
through it (training proper is out of scope).
"""
from __future__ import annotations

import torch.nn as nn

from . import kernels


class SpectralMatchingLoss(nn.Module):
    """balanced=True: mean over pairs of 0.5 * sum gt (M-1)^2 / (relu(sum gt - 1) + 1)
    + 0.5 * sum (1-gt) M^2 / (relu(sum (1-gt) - 1) + 1); else MSE(M, gt);
    gt_ij = (l_i + l_j == 2) with a zero diagonal."""

    def __init__(self, balanced=True):
        super().__init__()
        self.balanced = balanced

    def forward(self, M, gt_labels):
        return kernels.spectral_matching_loss(M, gt_labels.float(), self.balanced)
