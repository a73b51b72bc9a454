"""TEST INFRASTRUCTURE -- CPU oracle for the DeepFwFM forward (float64 numpy).

This is the checker, never the product: only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import it.  The product path
(xsdeepfwfm_deprecated_amd) never calls into oracle/.

A float64 restatement of reference model/DeepFMs.py:285-469 (and
model/QREmbeddingBag.py:156-174 for QR tables), written from the algebra, not
from the reference's op sequence:

  E_f[b]   = v_f[0] * Xv[b, f]                       f <  numerical  (:297-299, :334)
           = v_f[Xi[b, f - numerical]]               plain / bag     (:334-335, :314)
           = Wq_f[i // c]  (*|+)  Wr_f[i % c]        QR              (QREmbeddingBag :157-172)
  fo[b, f] = w1_f[0] * Xv[b, f] | w1_f[Xi]           tables          (:300-305)
           = <E_f[b], Wfl[f]>                        fwlw            (:338-345)
  first[b] = fo[b] . w_lw  (lw, :445-450)  |  sum_f fo[b, f]         (:458, :463)
  second[b]= sum_{k<l} Rs[k,l] <E_k[b], E_l[b]>,  Rs = (R + R^T)/2   fwfm (:352-367)
           = sum_{k<l} <E_k[b], E_l[b]>                              fm   (:352-355)
  deep[b]  = fc . relu(W3 relu(W2 relu(W1 cat_f E_f[b] + b1) + b2) + b3)   (:398-428)
  logit[b] = first + second + deep + bias                            (:455-469)

Parity pinning: this restatement is checked against golden vectors produced by
importing the reference itself in the build container (tests/golden/,
generator tests/golden/gen_golden.py) and against the known-answer FwFM of the
reference's own C++ latency model (latency/criteo_latency.cpp:86-103,
tests/test_oracle.py).  See DESIGN.md "Oracle".
"""
from __future__ import annotations

import numpy as np


def _field_table(params, prefix, f):
    """(kind, tensors): kind 'plain' -> (W,), 'qr' -> (Wq, Wr)."""
    k = f"{prefix}.{f}.weight"
    if k in params:
        return "plain", (np.asarray(params[k], dtype=np.float64),)
    return "qr", (np.asarray(params[f"{prefix}.{f}.weight_q"], dtype=np.float64),
                  np.asarray(params[f"{prefix}.{f}.weight_r"], dtype=np.float64))


def _lookup(params, prefix, f, idx, qr_operation):
    kind, t = _field_table(params, prefix, f)
    if kind == "plain":
        return t[0][idx]
    wq, wr = t
    c = wr.shape[0]
    q, r = idx // c, idx % c
    return wq[q] * wr[r] if qr_operation == "mult" else wq[q] + wr[r]


def embeddings(cfg, params, Xi, Xv, prefix="fm_2nd_embeddings"):
    """E [B, F, dim] float64 for the given table family."""
    F, num = cfg["field_size"], cfg["numerical"]
    Xi = np.asarray(Xi).reshape(Xi.shape[0], -1).astype(np.int64)
    Xv = np.asarray(Xv, dtype=np.float64)
    cols = []
    for f in range(F):
        if f < num:
            v = np.asarray(params[f"{prefix}.{f}.weight"], dtype=np.float64)[0]
            cols.append(Xv[:, f:f + 1] * v[None, :])
        else:
            idx = Xi[:, f - num]
            kind, t = _field_table(params, prefix, f)
            # plain tables accept [0, n); a QR bag accepts any i with i // c inside weight_q
            limit = t[0].shape[0] if kind == "plain" else t[0].shape[0] * t[1].shape[0]
            if idx.size and (idx.min() < 0 or idx.max() >= limit):
                raise IndexError("index out of range in self")
            cols.append(_lookup(params, prefix, f, idx, cfg.get("qr_operation", "mult")))
    return np.stack(cols, axis=1)


def forward(cfg, params, Xi, Xv, return_parts=False):
    """logits float64 [B]."""
    F, D = cfg["field_size"], cfg["embedding_size"]
    second_kind = "fwfm" if cfg.get("use_fwfm") else ("fm" if cfg.get("use_fm") else None)
    B = np.asarray(Xi).shape[0]
    E = embeddings(cfg, params, Xi, Xv) if (second_kind or cfg.get("use_deep")) else None

    if cfg.get("use_fwlw"):
        wfl = np.asarray(params["fwfm_linear.weight"], dtype=np.float64)  # [F, D]
        fo = np.einsum("bfd,fd->bf", E, wfl)
    else:
        fo = embeddings(cfg, params, Xi, Xv, prefix="fm_1st_embeddings")[:, :, 0]
    if second_kind and cfg.get("use_lw"):
        first = fo @ np.asarray(params["fm_1st.weight"], dtype=np.float64)[0]
    else:
        first = fo.sum(axis=1)

    second = np.zeros(B)
    if second_kind:
        if second_kind == "fwfm":
            R = np.asarray(params["field_cov.weight"], dtype=np.float64)
            Rs = (R.T + R) * 0.5
        else:
            Rs = np.ones((F, F))
        G = np.einsum("bkd,bld->bkl", E, E)
        iu = np.triu_indices(F, k=1)
        second = (G[:, iu[0], iu[1]] * Rs[iu][None, :]).sum(axis=1)

    deep = np.zeros(B)
    if cfg.get("use_deep"):
        h = E.reshape(B, F * D)
        for i in range(1, cfg["h_depth"] + 1):
            W = np.asarray(params[f"net_1_linear_{i}.weight"], dtype=np.float64)
            bb = np.asarray(params[f"net_1_linear_{i}.bias"], dtype=np.float64)
            h = np.maximum(h @ W.T + bb, 0.0)
        deep = h @ np.asarray(params["net_1_fc.weight"], dtype=np.float64)[0]

    bias = float(np.asarray(params["bias"], dtype=np.float64)[0]) if "bias" in params else 0.0
    total = first + second + deep + bias
    if return_parts:
        return total, dict(first=first, second=second, deep=deep, E=E)
    return total


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-np.asarray(x, dtype=np.float64)))


def latency_fwfm_known_answer(Xi, Xv, field_sizes, emb=10):
    """Scalar restatement of the reference C++ latency model's FwFM (latency/criteo_latency.cpp:86-103)
    with its closed-form init_FM weights (:201-212: linear[i][j] = j*j*1.11, quadratic[i][j][k] = 1.2*j,
    corr = 1) and global_bias = 0 (`int global_bias = 0.3`, :236).  Returns the pre-loss sum."""
    Fn = len(field_sizes)
    f32 = np.float32
    s = f32(0.0)
    for i in range(Fn):
        s = f32(s + f32(f32(Xi[i] * Xi[i] * 1.11) * f32(Xv[i])))
    for i in range(Fn):
        for j in range(i + 1, Fn):
            for _ in range(emb):
                s = f32(s + f32(f32(f32(1.2 * Xi[i]) * f32(1.2 * Xi[j])) * f32(1.0)))
    return float(s)
