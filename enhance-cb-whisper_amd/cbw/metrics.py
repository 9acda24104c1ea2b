"""Evaluation metrics of the reference's test loops (host-side, CPU; not on the GPU hot path).

* ``binary_precision_recall_curve`` — torchmetrics==1.2.0 ``PrecisionRecallCurve(task="binary")``
  (requirements.txt:19; constructed at efficient_kws/model.py:127 and model/model.py:76), absent
  here.  Restated: predictions outside [0, 1] go through a sigmoid; sort scores descending; at each
  distinct score s the cumulative TP/FP counts of "predict positive iff score >= s"; precision =
  TP / (TP + FP), recall = TP / P; both reversed (ascending threshold) and closed with
  (precision 1, recall 0); thresholds = the distinct scores ascending.  Cross-checked against
  scikit-learn's ``precision_recall_curve`` (the same published algorithm) in tests/test_scorer.py.
* ``operating_point`` — efficient_kws/model.py:806-839 (and model/model.py:373-405): the entry at
  index #(thresholds < threshold) of precision / recall, F1 = 2PR / (P + R) (0 if either is 0).
* ``evaluate_with_conf_int`` — confidence_intervals==0.0.3 (requirements.txt:1), absent here:
  metric on all samples, plus a percentile bootstrap CI (alpha %) over ``num_bootstraps`` resamples;
  with ``conditions`` the resampling draws whole conditions (speakers) with replacement, bootstrap b
  seeded with b.  CI values are "parity unpinned" (the library's RNG use is not available to check).
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence, Tuple

import numpy as np


def binary_precision_recall_curve(preds, target) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    p = np.asarray(preds, dtype=np.float64).reshape(-1)
    t = np.asarray(target).reshape(-1).astype(np.int64)
    if p.size and not np.all((p >= 0) & (p <= 1)):
        p = 1.0 / (1.0 + np.exp(-p))
    order = np.argsort(-p, kind="stable")
    p, t = p[order], t[order]
    ends = np.flatnonzero(np.diff(p)) if p.size > 1 else np.zeros(0, dtype=np.int64)
    ends = np.concatenate([ends, [p.size - 1]]).astype(np.int64) if p.size else ends
    tps = np.cumsum(t == 1)[ends].astype(np.float64)
    fps = (ends + 1) - tps
    with np.errstate(divide="ignore", invalid="ignore"):
        precision = tps / (tps + fps)
        recall = tps / tps[-1] if tps.size else tps
    precision = np.concatenate([precision[::-1], [1.0]])
    recall = np.concatenate([recall[::-1], [0.0]])
    return precision, recall, p[ends][::-1].copy()


def operating_point(precision: np.ndarray, recall: np.ndarray, thresholds: np.ndarray,
                    threshold: float) -> Tuple[float, float, float]:
    i = int(np.count_nonzero(np.asarray(thresholds) - threshold < 0))
    pr, rc = float(precision[i]), float(recall[i])
    f1 = 2 * pr * rc / (pr + rc) if (pr != 0 and rc != 0) else 0
    return pr, rc, f1


def _take(x, idx):
    if isinstance(x, np.ndarray):
        return x[idx]
    try:
        import torch
        if torch.is_tensor(x):
            return x[torch.as_tensor(idx, dtype=torch.long)]
    except ImportError:
        pass
    return [x[int(i)] for i in idx]


def bootstrap_indices(n: int, conditions: Optional[Sequence] = None, seed: Optional[int] = None) -> np.ndarray:
    rng = np.random.RandomState(seed)
    if conditions is None:
        return rng.choice(n, n, replace=True)
    cond = np.asarray(conditions)
    uniq = np.unique(cond)
    picked = rng.choice(uniq, len(uniq), replace=True)
    return np.concatenate([np.flatnonzero(cond == c) for c in picked])


def evaluate_with_conf_int(samples, metric: Callable, labels=None, conditions: Optional[Sequence] = None,
                           num_bootstraps: int = 1000, alpha: float = 5, samples2=None):
    def run(idx):
        s = samples if idx is None else _take(samples, idx)
        s2 = None if samples2 is None else (samples2 if idx is None else _take(samples2, idx))
        if labels is None:
            return metric(s, s2)
        return metric(labels if idx is None else _take(labels, idx), s, s2)

    center = run(None)
    if num_bootstraps <= 0:
        return center, (None, None)
    vals = [run(bootstrap_indices(len(samples), conditions, seed=b)) for b in range(num_bootstraps)]
    return center, (float(np.percentile(vals, alpha / 2)), float(np.percentile(vals, 100 - alpha / 2)))
