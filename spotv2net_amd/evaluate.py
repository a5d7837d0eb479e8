"""Evaluation path of the reference notebook:
6_results.ipynb cells 9-12 — model.eval(), per batch
``y_hat = model(data) * Std + Mean`` and ``y = data.y_x * Std + Mean``
(the 'Variance' scaler of 4_standardize_data.py), MSE = mean over batches of
the batch MSE (``test_loss / len(test_loader)``), and QLIKE
``y/ŷ - log(y/ŷ) - 1`` (cell 2 ``qlike``) elementwise, reported here also as
its mean.  Reference checkpoints (``*_weights_seed_*.pth``, written by
5_train_SpotV2Net.py:195 as a state_dict) load with ``load_checkpoint``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, Tuple

import torch


def qlike(y: torch.Tensor, yhat: torch.Tensor) -> torch.Tensor:
    r = y / yhat
    return r - torch.log(r) - 1


@dataclass
class EvalResult:
    mse: float
    qlike_mean: float
    qlike: torch.Tensor       # elementwise, as the notebook's qlike() returns
    predictions: torch.Tensor  # de-standardised, concatenated over batches
    actual: torch.Tensor


@torch.no_grad()
def evaluate(model: torch.nn.Module, batches: Iterable, variance_scaler: Tuple[float, float]
             ) -> EvalResult:
    mean, std = variance_scaler
    was_training = model.training
    model.eval()
    total, nb = 0.0, 0
    preds, actual = [], []
    for data in batches:
        yh = model(data) * std + mean
        y = data.y_x * std + mean
        total = total + torch.nn.functional.mse_loss(yh, y)
        nb += 1
        preds.append(yh)
        actual.append(y)
    model.train(was_training)
    if nb == 0:
        raise ValueError("no batches")
    p = torch.cat(preds)
    a = torch.cat(actual)
    q = qlike(a, p)
    return EvalResult(float(total / nb), float(q.mean()), q, p, a)


def load_checkpoint(model: torch.nn.Module, path: str) -> torch.nn.Module:
    """Load a reference state_dict checkpoint (weights only: no code runs)."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(sd)
    return model
