"""DiceCE loss of the reference trainer (3_train.py:72: DiceCELoss(to_onehot_y=True,
softmax=True)).

Restates MONAI's DiceCELoss with its defaults (monai/losses/dice.py:773-805 -> DiceLoss
:119-180, nn.CrossEntropyLoss): include_background, no sigmoid, squared_pred=False,
jaccard=False, smooth_nr = smooth_dr = 1e-5, batch=False, reduction 'mean', lambda_dice =
lambda_ce = 1.  It runs once per step on (B, 4, 128^3) logits -- outside the §8 hot path -- as
plain PyTorch GPU ops (autograd gives its backward).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class DiceCELoss(nn.Module):
    def __init__(self, to_onehot_y: bool = True, softmax: bool = True, smooth_nr: float = 1e-5,
                 smooth_dr: float = 1e-5, lambda_dice: float = 1.0, lambda_ce: float = 1.0):
        super().__init__()
        if not (to_onehot_y and softmax):
            raise NotImplementedError("only DiceCELoss(to_onehot_y=True, softmax=True)")
        self.smooth_nr, self.smooth_dr = smooth_nr, smooth_dr
        self.lambda_dice, self.lambda_ce = lambda_dice, lambda_ce

    def forward(self, logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        """logits (B, K, *S) float, target (B, 1, *S) integer class labels."""
        K = logits.shape[1]
        lab = target[:, 0].long()
        # Dice: softmax probabilities against the one-hot target, per (batch, class)
        p = torch.softmax(logits, dim=1)
        onehot = F.one_hot(lab, K).movedim(-1, 1).to(p.dtype)
        red = tuple(range(2, logits.dim()))
        inter = (p * onehot).sum(red)
        denom = onehot.sum(red) + p.sum(red)
        dice = 1.0 - (2.0 * inter + self.smooth_nr) / (denom + self.smooth_dr)
        # CE: class-index targets, mean over voxels and batch
        ce = F.cross_entropy(logits, lab)
        return self.lambda_dice * dice.mean() + self.lambda_ce * ce
