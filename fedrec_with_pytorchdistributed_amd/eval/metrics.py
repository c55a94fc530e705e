"""Ranking metrics: AUC, MRR, nDCG@k (reference ``evaluation_functions.py:5-31``).

Definitions match the reference:

* ``dcg_score``: gain ``2^y - 1``, discount ``log2(rank + 1)``, top ``k`` by score.
* ``ndcg_score``: ``dcg(y_true, y_score) / dcg(y_true, y_true)``.
* ``mrr_score``: ``sum(y / rank) / sum(y)`` in score order.
* ``roc_auc_score``: the Mann-Whitney statistic with average ranks for ties, i.e. what
  ``sklearn.metrics.roc_auc_score`` returns for binary labels (the reference imports
  sklearn's; this implementation removes the dependency and is checked against sklearn
  in the tests).

Sorting uses a stable descending order on ``-score`` so ties resolve like the reference's
``np.argsort(y_score)[::-1]`` (which reverses a stable ascending sort).

:func:`batch_metrics` evaluates many impressions at once (``[I, C]`` score matrix with the
positive in column 0, as in validation, ``client.py:160-165``) and returns the corpus
mean -- the fix for quirk Q9 (the reference returns only the last impression's numbers,
``client.py:171``), with the last impression's values kept for compat logging.
"""
from __future__ import annotations

from typing import Dict, Sequence

import numpy as np


def _order(y_score: np.ndarray) -> np.ndarray:
    return np.argsort(y_score, kind="stable")[::-1]


def dcg_score(y_true: Sequence[float], y_score: Sequence[float], k: int = 10) -> float:
    y_true = np.asarray(y_true, dtype=np.float64)
    order = _order(np.asarray(y_score))
    yt = np.take(y_true, order[:k])
    gains = 2.0 ** yt - 1.0
    disc = np.log2(np.arange(len(yt)) + 2.0)
    return float(np.sum(gains / disc))


def ndcg_score(y_true, y_score, k: int = 10) -> float:
    best = dcg_score(y_true, y_true, k)
    return dcg_score(y_true, y_score, k) / best


def mrr_score(y_true, y_score) -> float:
    y_true = np.asarray(y_true, dtype=np.float64)
    yt = np.take(y_true, _order(np.asarray(y_score)))
    rr = yt / (np.arange(len(yt)) + 1.0)
    return float(np.sum(rr) / np.sum(yt))


def _avg_ranks(x: np.ndarray) -> np.ndarray:
    order = np.argsort(x, kind="mergesort")
    xs = x[order]
    ranks = np.empty(len(x), dtype=np.float64)
    i = 0
    n = len(x)
    while i < n:
        j = i
        while j + 1 < n and xs[j + 1] == xs[i]:
            j += 1
        ranks[order[i:j + 1]] = 0.5 * (i + j) + 1.0
        i = j + 1
    return ranks


def roc_auc_score(y_true, y_score) -> float:
    y_true = np.asarray(y_true).astype(bool)
    y_score = np.asarray(y_score, dtype=np.float64)
    n_pos = int(y_true.sum())
    n_neg = len(y_true) - n_pos
    if n_pos == 0 or n_neg == 0:
        raise ValueError("Only one class present in y_true. ROC AUC score is not defined in that case.")
    r = _avg_ranks(y_score)
    return float((r[y_true].sum() - n_pos * (n_pos + 1) / 2.0) / (n_pos * n_neg))


def compute_amn(y_true, y_score):
    """AUC, MRR, nDCG@5, nDCG@10 of one impression (``evaluation_functions.py:26-31``)."""
    return (roc_auc_score(y_true, y_score), mrr_score(y_true, y_score),
            ndcg_score(y_true, y_score, 5), ndcg_score(y_true, y_score, 10))


def batch_metrics(scores: np.ndarray) -> Dict[str, float]:
    """Vectorised metrics for ``[I, C]`` scores whose positive is column 0.

    With exactly one positive per impression: AUC = fraction of negatives ranked below
    the positive (ties count 1/2); MRR = 1/rank; nDCG@k = 1/log2(rank+1) if rank <= k.
    ``rank`` breaks ties like the reference's reversed stable argsort: among equal
    scores the *later* column ranks first.
    """
    s = np.asarray(scores, dtype=np.float64)
    if s.ndim != 2 or s.shape[0] == 0:
        return {"auc": float("nan"), "mrr": float("nan"), "ndcg5": float("nan"), "ndcg10": float("nan"),
                "n": 0}
    p = s[:, :1]
    neg = s[:, 1:]
    C = s.shape[1]
    auc = ((neg < p).sum(1) + 0.5 * (neg == p).sum(1)) / (C - 1)
    # reversed stable argsort: all strictly-greater items, and equal items after column 0,
    # rank ahead of the positive
    rank = 1 + (neg > p).sum(1) + (neg == p).sum(1)
    mrr = 1.0 / rank
    nd5 = np.where(rank <= 5, 1.0 / np.log2(rank + 1.0), 0.0)
    nd10 = np.where(rank <= 10, 1.0 / np.log2(rank + 1.0), 0.0)
    out = {"auc": float(auc.mean()), "mrr": float(mrr.mean()), "ndcg5": float(nd5.mean()),
           "ndcg10": float(nd10.mean()), "n": int(s.shape[0])}
    out.update({"last_auc": float(auc[-1]), "last_mrr": float(mrr[-1]),
                "last_ndcg5": float(nd5[-1]), "last_ndcg10": float(nd10[-1])})
    return out


def metric_sums(scores: np.ndarray) -> np.ndarray:
    """Per-corpus sums ``[auc, mrr, ndcg5, ndcg10, count]`` (for an all-reduce of metrics)."""
    m = batch_metrics(scores)
    n = m["n"]
    if n == 0:
        return np.zeros(5)
    return np.array([m["auc"] * n, m["mrr"] * n, m["ndcg5"] * n, m["ndcg10"] * n, n], dtype=np.float64)
