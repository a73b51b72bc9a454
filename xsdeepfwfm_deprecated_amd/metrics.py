"""Evaluation metrics of the reference harness (model/DeepFMs.py:22, 781-800).

* ``DeviceMetrics``: AUC, PR-AUC, log-loss, RCE and CTR of a whole evaluation set on the device
  (C ABI ``dfwfm_eval_metrics``: a hand-written radix ranking + scans, sklearn 1.7 definitions, the same bits every call) -- what
  ``DeepFMs.eval_by_batch`` uses; a single 64-byte copy back per evaluation.
* ``roc_auc_score`` / ``prauc`` / ``rce`` / ``ctr``: the reference's host functions (sklearn), kept for
  the reference API (``eval_metric`` default, ``compute_prauc``, ``compute_rce``) on host arrays.
* ``parameter_counts``: the census of print_size_of_model (:905-945).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
from sklearn.metrics import auc, log_loss, precision_recall_curve, roc_auc_score  # noqa: F401

from . import _lib


class DeviceMetrics:
    """sklearn's roc_auc_score / precision_recall_curve+auc / log_loss / RCE on device tensors."""

    NAMES = ("auc", "prauc", "log_loss", "rce", "ctr", "positives", "n", "distinct_predictions")

    def __init__(self, device):
        self.device = torch.device(device)
        self.ws = torch.empty(0, dtype=torch.uint8, device=self.device)
        self.out = torch.zeros(8, dtype=torch.float64, device=self.device)

    def __call__(self, logits, labels, sync=True):
        """logits, labels: float32 device tensors [n] (labels 0/1).  Returns a dict of floats (or, with
        sync=False, the 8-double device tensor)."""
        n = int(logits.numel())
        logits = logits.reshape(-1).contiguous()
        labels = labels.reshape(-1).to(dtype=torch.float32).contiguous()
        if logits.dtype != torch.float32 or not logits.is_cuda or labels.numel() != n:
            raise RuntimeError("DeviceMetrics: float32 HIP logits and labels of equal length expected")
        L = _lib.lib()
        need = int(L.dfwfm_metrics_workspace_bytes(n))
        if self.ws.numel() < need:
            self.ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        out = torch.empty(8, dtype=torch.float64, device=self.device)
        st = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(L.dfwfm_eval_metrics(ctypes.c_void_p(logits.data_ptr()), ctypes.c_void_p(labels.data_ptr()), n,
                                        ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(self.ws.data_ptr()),
                                        self.ws.numel(), st), "dfwfm_eval_metrics")
        if not sync:
            return out
        return dict(zip(self.NAMES, out.cpu().tolist()))


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
