"""TEST INFRASTRUCTURE -- fp32 PyTorch-CPU port of the reference forward's op sequence.

Used as (1) the CPU baseline that bench.py times on the GPU box's host cores
(the reference itself cannot travel there), and (2) an fp32 cross-check of
the float64 oracle.  Never imported by the product package.

It deliberately keeps the reference's algorithmic shape so its CPU cost is
representative (reference model/DeepFMs.py:297-458):
  * one embedding lookup per field, numerical fields via a zero index and a
    scale by Xv (:297-299, :304, :334);
  * torch.stack of the 39 field embeddings -> [F, B, D] (:337);
  * the full outer product einsum('kij,lij->klij') -> [F, F, B, D] (:352),
    weighted by (R^T + R)/2 (:363-364), summed minus its diagonal, halved
    (:366-367);
  * fwlw einsums (:344-345), lw matmul (:450);
  * cat -> [B, F*D] and the addmm/ReLU MLP (:398-428);
  * total = sum(first) + sum(second) + sum(deep) + bias (:458).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _lookup(params, prefix, f, idx, qr_operation):
    k = f"{prefix}.{f}.weight"
    if k in params:
        return F.embedding(idx, params[k])
    wq, wr = params[f"{prefix}.{f}.weight_q"], params[f"{prefix}.{f}.weight_r"]
    c = wr.shape[0]
    eq = F.embedding(torch.div(idx, c, rounding_mode="floor"), wq)
    er = F.embedding(torch.remainder(idx, c), wr)
    return eq * er if qr_operation == "mult" else eq + er


def _field_embeddings(cfg, params, Xi, Xv, prefix):
    num = cfg["numerical"]
    zero = torch.zeros(Xi.shape[0], dtype=torch.long)
    out = []
    for f in range(cfg["field_size"]):
        if f < num:
            out.append(F.embedding(zero, params[f"{prefix}.{f}.weight"]) * Xv[:, f:f + 1])
        else:
            out.append(_lookup(params, prefix, f, Xi[:, f - num], cfg.get("qr_operation", "mult")))
    return out


@torch.no_grad()
def forward(cfg, params, Xi, Xv):
    """params: name -> float32 CPU tensor; Xi int64 [B, ncat]; Xv float32 [B, num]. Returns [B] fp32."""
    Xi = Xi.reshape(Xi.shape[0], -1)
    fwfm, fm = bool(cfg.get("use_fwfm")), bool(cfg.get("use_fm"))
    emb2 = _field_embeddings(cfg, params, Xi, Xv, "fm_2nd_embeddings") if (fwfm or fm or cfg.get("use_deep")) else None
    second = None
    if fwfm or fm:
        E = torch.stack(emb2)                                    # [F, B, D]
        if cfg.get("use_fwlw"):
            first = torch.einsum("ijk,ik->ijk", E, params["fwfm_linear.weight"])
            first = torch.einsum("ijk->ji", first)               # [B, F]
        else:
            first = torch.cat(_field_embeddings(cfg, params, Xi, Xv, "fm_1st_embeddings"), 1)
        outer = torch.einsum("kij,lij->klij", E, E)              # [F, F, B, D]
        if fwfm:
            W = params["field_cov.weight"]
            outer = torch.einsum("klij,kl->klij", outer, (W.t() + W) * 0.5)
        second = (outer.sum(0).sum(0) - torch.einsum("kkij->kij", outer).sum(0)) * 0.5   # [B, D]
        if cfg.get("use_lw"):
            first = torch.matmul(first, params["fm_1st.weight"].t())
    else:  # logistic regression
        first = torch.cat(_field_embeddings(cfg, params, Xi, Xv, "fm_1st_embeddings"), 1)
    total = first.sum(1)
    if second is not None:
        total = total + second.sum(1)
    if cfg.get("use_deep"):
        h = torch.cat(emb2, 1)
        for i in range(1, cfg["h_depth"] + 1):
            h = torch.relu(torch.addmm(params[f"net_1_linear_{i}.bias"], h, params[f"net_1_linear_{i}.weight"].t()))
        total = total + torch.mm(h, params["net_1_fc.weight"].t()).sum(1)
    return total + params["bias"]
