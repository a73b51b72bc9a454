"""Training path of DeepFMs (reference model/DeepFMs.py:497-748, 807-823).

The forward of a training step is the same fused HIP kernel; gradients come
from the HIP backward kernels (see csrc/).  Until those land, requesting a
gradient raises instead of silently falling back to PyTorch ops.
"""
from __future__ import annotations

import torch


class _FusedForward(torch.autograd.Function):
    @staticmethod
    def forward(ctx, eng, xi, xv, *params):
        return eng.forward(xi, xv)

    @staticmethod
    def backward(ctx, grad_out):
        raise NotImplementedError("dfwfm: the HIP backward kernels are not built yet; run the forward "
                                  "under torch.no_grad()")


def train_forward(model, eng, xi, xv):
    params = [p for p in model.parameters() if p.requires_grad]
    return _FusedForward.apply(eng, xi, xv, *params)


def binary_search_threshold(param, target_percent, total_no):
    """Magnitude threshold hitting a target sparsity by bisection (reference :807-823)."""
    lo, hi = 0.0, 1e2
    mid = (lo + hi) / 2
    for _ in range(101):
        if not lo < hi:
            break
        mid = (lo + hi) / 2
        rate = (param.abs() < mid).sum().item() * 1.0 / total_no
        if abs(rate - target_percent) < 0.0001:
            return mid
        if rate > target_percent:
            hi = mid
        else:
            lo = mid
    return mid


def fit(model, *args, **kwargs):
    raise NotImplementedError("dfwfm: training (fit) needs the HIP backward kernels (next milestone)")
