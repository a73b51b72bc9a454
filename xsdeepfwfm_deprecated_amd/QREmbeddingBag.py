"""Quotient-remainder compositional embedding bag.

Parameter container with the reference's interface and state-dict keys
(``weight_q [ceil(n/c), D]``, ``weight_r [c, D]``; reference
model/QREmbeddingBag.py:112-150).  Inside DeepFMs the lookup itself is done by
the fused HIP forward (phase G of csrc/dfwfm_kernels.hip): row
``weight_q[i // c]`` combined with ``weight_r[i % c]`` by ``*`` or ``+``.

The module's own ``forward`` (used only when called standalone, never on the
DeepFMs hot path) keeps the reference semantics: bags given by ``offsets``
(or rows of a 2-D input), summed (``mode='sum'``) or averaged, then combined
(reference model/QREmbeddingBag.py:156-174).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.parameter import Parameter

_OPS = ("concat", "mult", "add")


class QREmbeddingBag(nn.Module):
    __constants__ = ["num_categories", "embedding_dim", "num_collisions", "operation", "max_norm",
                     "norm_type", "scale_grad_by_freq", "mode", "sparse"]

    def __init__(self, num_categories, embedding_dim, num_collisions, operation="mult", max_norm=None,
                 norm_type=2.0, scale_grad_by_freq=False, mode="mean", sparse=False, _weight=None):
        super().__init__()
        if operation not in _OPS:
            raise AssertionError("Not valid operation!")
        self.num_categories = int(num_categories)
        if isinstance(embedding_dim, int) or len(embedding_dim) == 1:
            dim = int(embedding_dim if isinstance(embedding_dim, int) else embedding_dim[0])
            self.embedding_dim = [dim, dim]
        else:
            self.embedding_dim = [int(d) for d in embedding_dim]
        if operation in ("add", "mult") and self.embedding_dim[0] != self.embedding_dim[1]:
            raise AssertionError("Embedding dimensions do not match!")
        self.num_collisions = int(num_collisions)
        self.operation = operation
        self.max_norm = max_norm
        self.norm_type = norm_type
        self.scale_grad_by_freq = scale_grad_by_freq
        self.num_embeddings = [int(math.ceil(self.num_categories / self.num_collisions)), self.num_collisions]
        if _weight is None:
            self.weight_q = Parameter(torch.empty(self.num_embeddings[0], self.embedding_dim[0]))
            self.weight_r = Parameter(torch.empty(self.num_embeddings[1], self.embedding_dim[1]))
            self.reset_parameters()
        else:
            wq, wr = _weight
            if list(wq.shape) != [self.num_embeddings[0], self.embedding_dim[0]]:
                raise AssertionError("Shape of weight for quotient table does not match num_embeddings and embedding_dim")
            if list(wr.shape) != [self.num_embeddings[1], self.embedding_dim[1]]:
                raise AssertionError("Shape of weight for remainder table does not match num_embeddings and embedding_dim")
            self.weight_q = Parameter(wq)
            self.weight_r = Parameter(wr)
        self.mode = mode
        self.sparse = sparse

    def reset_parameters(self):
        # the reference passes sqrt(1/n) as the LOWER bound of U(a, 1) (its
        # QREmbeddingBag.py:152-154); DeepFMs.init_weights overwrites it anyway
        lo = float(np.sqrt(1.0 / self.num_categories))
        with torch.no_grad():
            self.weight_q.uniform_(lo, 1.0)
            self.weight_r.uniform_(lo, 1.0)

    def forward(self, input, offsets=None, per_sample_weights=None):
        q = torch.div(input, self.num_collisions, rounding_mode="floor").long()
        r = torch.remainder(input, self.num_collisions).long()
        eq = F.embedding_bag(q, self.weight_q, offsets, self.max_norm, self.norm_type,
                             self.scale_grad_by_freq, self.mode, self.sparse, per_sample_weights)
        er = F.embedding_bag(r, self.weight_r, offsets, self.max_norm, self.norm_type,
                             self.scale_grad_by_freq, self.mode, self.sparse, per_sample_weights)
        if self.operation == "concat":
            return torch.cat((eq, er), dim=1)
        if self.operation == "add":
            return eq + er
        return eq * er

    def extra_repr(self):
        s = f"{self.num_embeddings}, {self.embedding_dim}"
        if self.max_norm is not None:
            s += f", max_norm={self.max_norm}"
        if self.norm_type != 2:
            s += f", norm_type={self.norm_type}"
        if self.scale_grad_by_freq is not False:
            s += f", scale_grad_by_freq={self.scale_grad_by_freq}"
        return s + f", mode={self.mode}"
