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

import numpy as np
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
    return forward_graph(cfg, params, Xi, Xv)


def forward_graph(cfg, params, Xi, Xv, masks=None, drop_p=0.0):
    """forward() with autograd; masks[h] ([B, width] bool, h = 0..H) are the deep tower's dropout keep
    masks (nn.Dropout: x * keep / (1 - p), reference :411, :417-426)."""
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
        scale = 1.0 / (1.0 - drop_p) if masks is not None else 1.0
        if masks is not None:
            h = h * (masks[0].to(h.dtype) * scale)
        for i in range(1, cfg["h_depth"] + 1):
            h = torch.relu(torch.addmm(params[f"net_1_linear_{i}.bias"], h, params[f"net_1_linear_{i}.weight"].t()))
            if masks is not None:
                h = h * (masks[i].to(h.dtype) * scale)
        total = total + torch.mm(h, params["net_1_fc.weight"].t()).sum(1)
    return total + params["bias"]


# ---- training step (reference model/DeepFMs.py:553-637) -------------------------------------------
def _mix32(x):
    """murmur3's 32-bit finaliser (csrc/dfwfm_device.h mix32)."""
    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x = (x * np.uint32(0x85EBCA6B)).astype(np.uint32)
    x ^= x >> np.uint32(13)
    x = (x * np.uint32(0xC2B2AE35)).astype(np.uint32)
    x ^= x >> np.uint32(16)
    return x


def dropout_masks(seed, p, B, widths, row0=0):
    """The HIP kernels' counter-hash dropout keep masks (csrc/dfwfm_device.h dropout_keep), restated:
    keep (layer, row, col) iff (mix32(seed ^ row*K1 ^ col*K2 ^ layer*K3) >> 8) / 2^24 >= p.
    widths[h] = columns of layer h's output."""
    out = []
    with np.errstate(over="ignore"):
        rows = (np.arange(B, dtype=np.int64) + row0).astype(np.uint32)[:, None]
        for layer, w in enumerate(widths):
            cols = np.arange(w, dtype=np.uint32)[None, :]
            key = (np.uint32(seed) ^ (rows * np.uint32(0x9E3779B9)) ^ (cols * np.uint32(0x7FEB352D))
                   ^ np.uint32((layer * 0x846CA68B) & 0xFFFFFFFF)).astype(np.uint32)
            h = _mix32(key)
            u = (h >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
            out.append(torch.from_numpy(u >= np.float32(p)))
    return out


def train_step(cfg, params, Xi, Xv, y, lr, l2, masks=None, drop_p=0.0):
    """One reference training step: BCE-with-logits mean, backward, torch.optim.Adam(lr, weight_decay=l2)
    on CPU.  Returns (logits, loss, grads, new_params) as numpy."""
    leaf = {k: torch.tensor(v, requires_grad=True) for k, v in params.items()}
    out = forward_graph(cfg, leaf, torch.as_tensor(Xi), torch.as_tensor(Xv), masks, drop_p)
    loss = F.binary_cross_entropy_with_logits(out, torch.as_tensor(y, dtype=torch.float32))
    loss.backward()
    grads = {k: (v.grad.numpy().copy() if v.grad is not None else np.zeros_like(params[k]))
             for k, v in leaf.items()}
    for v in leaf.values():
        if v.grad is None:
            v.grad = torch.zeros_like(v)
    opt = torch.optim.Adam(list(leaf.values()), lr=lr, weight_decay=l2)
    opt.step()
    return out.detach().numpy(), float(loss.item()), grads, {k: v.detach().numpy() for k, v in leaf.items()}


def step_seed(base, step):
    """Seed of a graph-replayed step (csrc/dfwfm_device.h step_seed): base ^ mix32(step * 0x9E3779B9 + 0x7F4A7C15),
    with `step` the device counter's value when the step's kernels run (0 for the first step)."""
    with np.errstate(over="ignore"):
        x = np.array([(step * 0x9E3779B9 + 0x7F4A7C15) & 0xFFFFFFFF], dtype=np.uint32)
        return int(np.uint32(base) ^ _mix32(x)[0])


def train_steps(cfg, params, batches, lr, l2, mask_fn=None, drop_p=0.0):
    """Several reference training steps with one persistent torch.optim.Adam (CPU).  batches: list of
    (Xi, Xv, y); mask_fn(k, B) -> dropout masks of step k (or None).  Returns (per-step logits, params)."""
    leaf = {k: torch.tensor(v, requires_grad=True) for k, v in params.items()}
    opt = torch.optim.Adam(list(leaf.values()), lr=lr, weight_decay=l2)
    outs = []
    for k, (Xi, Xv, y) in enumerate(batches):
        opt.zero_grad()
        masks = mask_fn(k, len(Xi)) if mask_fn else None
        out = forward_graph(cfg, leaf, torch.as_tensor(Xi), torch.as_tensor(Xv), masks, drop_p)
        loss = F.binary_cross_entropy_with_logits(out, torch.as_tensor(y, dtype=torch.float32))
        loss.backward()
        for v in leaf.values():
            if v.grad is None:
                v.grad = torch.zeros_like(v)
        opt.step()
        outs.append(out.detach().numpy())
    return outs, {k: v.detach().numpy() for k, v in leaf.items()}
