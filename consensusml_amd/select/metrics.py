"""Classification metrics of the reference (C27), on device tensors.

Definitions follow `composite_code/rnotebook/cml_targetaml_seanalysis.Rmd:818-848`
(TPR = TP/P, TNR = TN/N, FDR = 1 - TP/(TP+FP), FOR = 1 - TN/(TN+FN)), test error = mean(pred !=
truth) (`...seanalysis.Rmd:108`), precision / recall (`:178-186`) and log-loss
(`scripts/model_comp.py:24-27`). Unlike the reference (§4.3: stale ``pred1``/``pb1`` at
`:1203-1212`) every metric is computed from the predictions passed in.
"""
from __future__ import annotations

from typing import Dict

import torch


def confusion_matrix(y: torch.Tensor, p: torch.Tensor, k: int = 2) -> torch.Tensor:
    """[k, k] counts, rows = truth, cols = prediction."""
    y = y.long().view(-1)
    p = p.long().view(-1)
    return torch.bincount(y * k + p, minlength=k * k).view(k, k)


def binary_metrics(y: torch.Tensor, p: torch.Tensor) -> Dict[str, float]:
    cm = confusion_matrix(y, p, 2).double()
    tn, fp, fn, tp = cm[0, 0], cm[0, 1], cm[1, 0], cm[1, 1]

    def div(a, b):
        return float(a / b) if float(b) > 0 else float("nan")
    tpr = div(tp, tp + fn)
    tnr = div(tn, tn + fp)
    prec = div(tp, tp + fp)
    npv = div(tn, tn + fn)
    return {"tpr": tpr, "tnr": tnr, "fdr": 1.0 - prec if prec == prec else float("nan"),
            "for": 1.0 - npv if npv == npv else float("nan"), "precision": prec, "recall": tpr,
            "test_error": float((cm[0, 1] + cm[1, 0]) / cm.sum())}


def log_loss(y: torch.Tensor, prob1: torch.Tensor, eps: float = 1e-15) -> float:
    """Binary log-loss of P(y=1) (sklearn.metrics.log_loss semantics, clipped)."""
    p = prob1.double().clamp(eps, 1 - eps)
    y = y.double()
    return float(-(y * p.log() + (1 - y) * (1 - p).log()).mean())


def roc_curve(y: torch.Tensor, score: torch.Tensor):
    """(fpr, tpr, thresholds) like ROCR::performance(pred, "tpr", "fpr") (`...seanalysis.Rmd:176`)."""
    s, order = torch.sort(score.double().view(-1), descending=True)
    yy = y.view(-1)[order].double()
    tps = torch.cumsum(yy, 0)
    fps = torch.cumsum(1 - yy, 0)
    P = max(float(yy.sum()), 1.0)
    N = max(float((1 - yy).sum()), 1.0)
    z = torch.zeros(1, dtype=torch.float64)
    return torch.cat([z, fps / N]), torch.cat([z, tps / P]), torch.cat([s[:1] + 1, s])


def auc(y: torch.Tensor, score: torch.Tensor) -> float:
    fpr, tpr, _ = roc_curve(y.cpu(), score.cpu())
    return float(torch.trapz(tpr, fpr))
