"""Evaluation metrics of the reference harness (model/DeepFMs.py:22, 781-800).

Host-side (sklearn), as in the reference: AUC, PR-AUC, RCE, CTR, plus the
parameter census of print_size_of_model (:905-945).
"""
from __future__ import annotations

import numpy as np
from sklearn.metrics import auc, log_loss, precision_recall_curve, roc_auc_score  # noqa: F401


def prauc(gt, pred):
    prec, recall, _ = precision_recall_curve(gt, pred)
    return auc(recall, prec)


def ctr(gt):
    gt = np.asarray(gt)
    return float(np.sum(gt == 1)) / float(len(gt))


def rce(gt, pred):
    """Relative cross entropy vs predicting the data CTR everywhere (reference :796-800)."""
    ce = log_loss(gt, pred)
    c = ctr(gt)
    strawman = log_loss(gt, [c] * len(gt))
    return (1.0 - ce / strawman) * 100.0


def parameter_counts(model):
    out = dict(total=0, nonzero=0, emb1=0, emb2=0, dnn=0, r_nonzero=0)
    for name, p in model.named_parameters():
        out["total"] += int(np.prod(p.shape))
        out["nonzero"] += int((p != 0).sum().item())
        if "1st_embeddings" in name:
            out["emb1"] += int((p != 0).sum().item())
        if "2nd_embeddings" in name:
            out["emb2"] += int((p != 0).sum().item())
        if "linear_" in name:
            out["dnn"] += int((p != 0).sum().item())
        if name == "field_cov.weight":
            out["r_nonzero"] = int((0.5 * (p.data + p.data.t()) != 0).sum().item())
    return out
