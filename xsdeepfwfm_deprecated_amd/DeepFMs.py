"""DeepFMs -- drop-in for the reference's ``model.DeepFMs.DeepFMs``
(reference model/DeepFMs.py:47-1102) whose forward is the fused HIP kernel.

Same constructor keywords, same sub-modules and therefore the same
``state_dict`` keys (checkpoints of the reference load unchanged), same
``fit`` / ``eval_by_batch`` / ``predict*`` / ``run_benchmark`` surface.
``forward(Xi, Xv)`` does not run any per-field PyTorch op: it hands the
parameters' device pointers to ``libdfwfm.so`` (include/dfwfm.h) which
computes the logits in one launch on the current HIP stream.

Deliberate deviations (documented in DESIGN.md):
* ``predict`` / ``predict_proba`` accept ``Xi`` in the layout ``fit`` uses,
  ``[-1, field_size - numerical, 1]``; the reference reshapes to
  ``[-1, field_size, 1]`` (model/DeepFMs.py:854,865) and then fails.
* A module on the CPU runs the host kernels of libdfwfm_cpu.so (include/dfwfm_cpu.h: the custom op's CPU
  kernel, for the reference's -use_cuda 0 / -time_on_cuda 0 paths); a module on a HIP device runs
  libdfwfm.so.  Neither falls back to the other or to PyTorch ops: a missing library raises.
* FFM, quantization and multiple deep towers (``num_deeps > 1``) are not part
  of this engine (out of scope) and raise.
"""
from __future__ import annotations

import contextlib
import logging
import math
import os
import random
from time import time, time_ns

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import metrics
from .QREmbeddingBag import QREmbeddingBag
from .engine import CpuEngine, ForwardEngine
from ._lib import DfwfmError, FLAG_INDEX_OUT_OF_RANGE

_log = logging.getLogger("xsDeepFwFM")


class DeepFMs(nn.Module):
    def __init__(self, field_size, feature_sizes, embedding_size=10, is_shallow_dropout=True,
                 dropout_shallow=[0.0, 0.0], h_depth=3, deep_nodes=400, is_deep_dropout=True,
                 dropout_deep=[0.5, 0.5, 0.5, 0.5], eval_metric=metrics.roc_auc_score, n_epochs=64,
                 batch_size=2048, learning_rate=0.001, momentum=0.9, optimizer_type="adam",
                 is_batch_norm=False, verbose=False, random_seed=0, weight_decay=0.0, use_fm=True,
                 use_fwlw=False, use_lw=False, use_ffm=False, use_fwfm=False, use_deep=True,
                 loss_type="logloss", use_cuda=True, n_class=1, greater_is_better=True, sparse=0.9,
                 warm=10, num_deeps=1, numerical=13, use_logit=0, embedding_bag=False,
                 quantization_aware=False, dynamic_quantization=False, static_quantization=False,
                 static_calibrate=False, qr_flag=0, qr_operation="mult", qr_collisions=1,
                 qr_threshold=200, md_flag=0, md_threshold=200, logger=None):
        super().__init__()
        self.logger = logger if logger is not None else _log
        self.field_size = int(field_size)
        self.feature_sizes = [int(s) for s in feature_sizes]
        self.embedding_size = int(embedding_size)
        self.is_shallow_dropout = is_shallow_dropout
        self.dropout_shallow = dropout_shallow
        self.h_depth = int(h_depth)
        self.num_deeps = int(num_deeps)
        self.deep_layers = [int(deep_nodes)] * self.h_depth
        self.is_deep_dropout = is_deep_dropout
        self.dropout_deep = [0.5] * (self.h_depth + 1)  # the reference ignores the argument
        self.n_epochs = n_epochs
        self.batch_size = batch_size
        self.learning_rate = learning_rate
        self.momentum = momentum
        self.optimizer_type = optimizer_type
        self.is_batch_norm = is_batch_norm
        self.verbose = verbose
        self.weight_decay = weight_decay
        self.random_seed = random_seed
        self.use_fm, self.use_ffm, self.use_fwfm = use_fm, use_ffm, use_fwfm
        self.use_fwlw, self.use_lw, self.use_logit, self.use_deep = use_fwlw, use_lw, use_logit, use_deep
        self.loss_type = loss_type
        self.eval_metric = eval_metric
        self.use_cuda = use_cuda
        self.n_class = n_class
        self.greater_is_better = greater_is_better
        self.target_sparse = sparse
        self.warm = warm
        self.num = int(numerical)
        self.embedding_bag = embedding_bag if not qr_flag else qr_flag
        self.quantization_aware = quantization_aware
        self.static_quantization = static_quantization
        self.static_calibrate = static_calibrate
        self.dynamic_quantization = dynamic_quantization
        self.qr_flag = qr_flag
        self.qr_operation = qr_operation
        self.qr_collisions = qr_collisions
        self.qr_threshold = qr_threshold
        self.md_flag = md_flag
        self.md_threshold = md_threshold
        self.strict_index_check = True  # raise IndexError for out-of-range Xi (the kernel's sticky flag)
        self.eval_batch_sets = True  # eval_by_batch runs its full batches as batch sets (dfwfm_forward_batches)
        # inference over pruned hidden layers: the sparse MLP (dfwfm_spmlp.hip) when at most this fraction
        # of their weights is nonzero; 0 (default) keeps the dense MFMA kernel, which is faster at the
        # reference's 90 % masks (34.7 vs 100 us per batch)
        self.sparse_mlp_max_density = 0.0
        # the forward without a deep tower sums the FwFM over R's nonzero pairs when a pruned R
        # (reference :661-666) leaves at most this many (of F (F - 1) / 2); 0 (default) keeps the dense Gram
        # on MFMA, which is as fast at the reference's 73 of 741 pairs
        self.fwfm_pair_max = 0
        # the inference forward gathers from a serving copy of the categorical tables (second-order row and
        # first-order weight in one aligned row, dfwfm_model_pack_tables), rebuilt after weight updates; the values
        # are copied, so the logits are the same bits either way
        self.pack_tables = True
        # the device backward's gradient sums in a fixed order (dfwfm_set_deterministic; like
        # torch.use_deterministic_algorithms): two runs of a training step give the same bits, at ~+7 us (+2.6 %) per
        # step at Criteo-39 (sorted table scatter, split-K slices); on by default, False: float atomics (arrival order)
        self.deterministic = True
        self._defer_index_check = 0     # >0 inside a batched caller: one flag read at its end, not per batch
        self._engine = None

        np.random.seed(self.random_seed)
        random.seed(self.random_seed)
        torch.manual_seed(self.random_seed)

        if quantization_aware or dynamic_quantization or static_quantization:
            raise NotImplementedError("quantization is not part of the MI355X engine (SURVEY.md section 2 #10)")
        if use_ffm:
            raise NotImplementedError("FFM is not part of the MI355X engine (SURVEY.md section 2 #12)")
        if self.num_deeps != 1:
            raise NotImplementedError("num_deeps > 1 is not supported")
        if is_batch_norm:
            raise NotImplementedError("batch norm in the deep tower is not supported")
        if self.use_cuda and not torch.cuda.is_available():
            self.use_cuda = False
            self.logger.info("Cuda is not available, automatically changed into cpu model")

        n_shallow = int(bool(use_fm)) + int(bool(use_ffm)) + int(bool(use_fwfm)) + int(bool(use_logit))
        if n_shallow > 1:
            self.logger.info("only support one type only, please make sure to choose only LR, FM, FFM or FwFM part")
            raise SystemExit(1)
        if n_shallow == 0 and not use_deep:
            self.logger.info("You have to choose more than one of (fm, ffm, fwfm, deep) models to use")
            raise SystemExit(1)
        self.logger.info(self._describe())

        D, Fs = self.embedding_size, self.field_size
        if use_logit or use_fm or use_fwfm:
            self.bias = nn.Parameter(torch.tensor([0.01]))
            if not use_fwlw:
                self.fm_1st_embeddings = self._tables(1)
            if self.dropout_shallow:
                self.fm_first_order_dropout = nn.Dropout(self.dropout_shallow[0])
            if use_fm or use_fwfm:
                self.fm_2nd_embeddings = self._tables(D)
                if self.dropout_shallow:
                    self.fm_second_order_dropout = nn.Dropout(self.dropout_shallow[1])
                if use_lw:
                    self.fm_1st = nn.Linear(Fs, 1, bias=False)
                if use_fwlw:
                    self.fwfm_linear = nn.Linear(D, Fs, bias=False)
                if use_fwfm:
                    self.field_cov = nn.Linear(Fs, Fs, bias=False)
        if use_deep:
            if not use_fm and not use_fwfm:
                self.fm_2nd_embeddings = self._tables(D)
            widths = [Fs * D] + self.deep_layers
            if self.is_deep_dropout:
                self.net_1_linear_0_dropout = nn.Dropout(self.dropout_deep[0])
            for i in range(1, self.h_depth + 1):
                setattr(self, f"net_1_linear_{i}", nn.Linear(widths[i - 1], widths[i]))
                setattr(self, f"net_1_linear_{i}_relu", nn.ReLU())
                if self.is_deep_dropout:
                    setattr(self, f"net_1_linear_{i}_dropout", nn.Dropout(self.dropout_deep[i]))
            self.net_1_fc = nn.Linear(self.deep_layers[-1], 1, bias=False)

    # ------------------------------------------------------------------ build
    def _describe(self):
        if self.use_logit:
            return "The model is logistic regression."
        kind = "fm" if self.use_fm else ("fwfm" if self.use_fwfm else None)
        if kind and self.use_deep:
            return f"The model is deep{kind}({kind}+deep layers)"
        if kind:
            return f"The model is {kind} only"
        return "The model is deep layers only"

    def _tables(self, dim):
        """Per-field tables exactly as the reference builds them (model/DeepFMs.py:197-210, 1066-1091)."""
        if not self.embedding_bag:
            return nn.ModuleList([nn.Embedding(n, dim) for n in self.feature_sizes])
        tables = nn.ModuleList()
        for n in self.feature_sizes:
            if self.qr_flag and n > self.qr_threshold:
                tables.append(QREmbeddingBag(n, dim, self.qr_collisions, operation=self.qr_operation,
                                             mode="sum", sparse=False))
            else:
                bag = nn.EmbeddingBag(n, dim, mode="sum", sparse=False)
                w = np.random.uniform(low=-np.sqrt(1 / n), high=np.sqrt(1 / n), size=(n, dim)).astype(np.float32)
                bag.weight.data = torch.tensor(w)
                tables.append(bag)
        return tables

    def engine_config(self):
        return dict(field_size=self.field_size, numerical=self.num, embedding_size=self.embedding_size,
                    use_fwfm=int(bool(self.use_fwfm)), use_fm=int(bool(self.use_fm)),
                    use_logit=int(bool(self.use_logit)), use_deep=int(bool(self.use_deep)),
                    use_lw=int(bool(self.use_lw)), use_fwlw=int(bool(self.use_fwlw)),
                    h_depth=self.h_depth, deep_nodes=self.deep_layers[0])

    # -------------------------------------------------------------- HIP sync
    @staticmethod
    def _field_desc(mod_2nd, mod_1st):
        """Descriptor of one field's tables; either family may be absent (fwlw: no 1st-order
        tables; logistic regression: no 2nd-order tables).  Both families share QR-ness."""
        def parts(mod):
            if mod is None:
                return None, None
            if isinstance(mod, QREmbeddingBag):
                if mod.operation not in ("mult", "add"):
                    raise NotImplementedError("QR 'concat' changes the field width; unsupported")
                return mod.weight_q.detach(), mod.weight_r.detach()
            return mod.weight.detach(), None
        ref = mod_2nd if mod_2nd is not None else mod_1st
        if isinstance(ref, QREmbeddingBag):
            n, c, op = ref.num_categories, ref.num_collisions, 0 if ref.operation == "mult" else 1
        else:
            n, c, op = ref.weight.shape[0], 0, 0
        e2, e2r = parts(mod_2nd)
        e1, e1r = parts(mod_1st)
        return dict(emb2=e2, emb2_r=e2r, emb1=e1, emb1_r=e1r, n=n, c=c, op=op)

    def _sync_engine(self, device):
        if device.type == "cpu":
            return self._sync_cpu_engine()
        if device.type != "cuda":
            raise DfwfmError(f"DeepFMs forward runs on a HIP device or the CPU, not on {device}")
        if self._engine is None or self._engine.device != device:
            if self._engine is not None:
                self._engine.close()
            self._engine = ForwardEngine(self.engine_config(), device)
        eng = self._engine
        first = getattr(self, "fm_1st_embeddings", None)
        second = getattr(self, "fm_2nd_embeddings", None)
        fields = [self._field_desc(None if second is None else second[f], None if first is None else first[f])
                  for f in range(self.field_size)]
        eng.sync_tables(fields)

        def w(name, attr="weight"):
            m = getattr(self, name, None)
            return None if m is None else getattr(m, attr).detach()

        lin_w = [w(f"net_1_linear_{i}") for i in range(1, self.h_depth + 1)] if self.use_deep else []
        lin_b = [w(f"net_1_linear_{i}", "bias") for i in range(1, self.h_depth + 1)] if self.use_deep else []
        eng.sync_dense(w("field_cov"), w("fwfm_linear"), w("fm_1st") if self.use_lw else None,
                       self.bias.detach(), lin_w, lin_b, w("net_1_fc") if self.use_deep else None)
        return eng

    def _sync_inference(self, device):
        """_sync_engine plus the inference-only derived state: the serving copy of the categorical tables
        (re-packed when a table changed; the training forward reads the tables themselves)."""
        eng = self._sync_engine(device)
        if device.type == "cuda":
            first = getattr(self, "fm_1st_embeddings", None)
            second = getattr(self, "fm_2nd_embeddings", None)
            tabs = []
            for f in range(self.num, self.field_size):
                d = self._field_desc(None if second is None else second[f], None if first is None else first[f])
                tabs.append((d["emb2"], d["emb1"]))
            eng.sync_packed(tabs, self.pack_tables)
        return eng

    def _sync_cpu_engine(self):
        """The host kernels' engine (libdfwfm_cpu.so), re-described on every call (pointers, no copies)."""
        if not isinstance(self._engine, CpuEngine):
            if self._engine is not None:
                self._engine.close()
            self._engine = CpuEngine(self.engine_config())
        first = getattr(self, "fm_1st_embeddings", None)
        second = getattr(self, "fm_2nd_embeddings", None)
        fields = [self._field_desc(None if second is None else second[f], None if first is None else first[f])
                  for f in range(self.field_size)]

        def w(name, attr="weight"):
            m = getattr(self, name, None)
            return None if m is None else getattr(m, attr).detach()
        lin_w = [w(f"net_1_linear_{i}") for i in range(1, self.h_depth + 1)] if self.use_deep else []
        lin_b = [w(f"net_1_linear_{i}", "bias") for i in range(1, self.h_depth + 1)] if self.use_deep else []
        self._engine.sync(fields, w("field_cov"), w("fwfm_linear"), w("fm_1st") if self.use_lw else None,
                          self.bias.detach(), lin_w, lin_b, w("net_1_fc") if self.use_deep else None)
        return self._engine

    def _param_layout(self):
        """The trainable parameters in the C ABI's gradient layout (include/dfwfm.h dfwfm_grads):
        per field (emb2, emb2_r, emb1, emb1_r) and the dense tensors -- Parameters, not copies."""
        def parts(mod):
            if mod is None:
                return None, None
            if isinstance(mod, QREmbeddingBag):
                return mod.weight_q, mod.weight_r
            return mod.weight, None
        first = getattr(self, "fm_1st_embeddings", None)
        second = getattr(self, "fm_2nd_embeddings", None)
        fields = []
        for f in range(self.field_size):
            e2, e2r = parts(None if second is None else second[f])
            e1, e1r = parts(None if first is None else first[f])
            fields.append((e2, e2r, e1, e1r))

        def w(name, attr="weight"):
            m = getattr(self, name, None)
            return None if m is None else getattr(m, attr)
        H = self.h_depth if self.use_deep else 0
        dense = dict(field_cov=w("field_cov"), fwfm_lin=w("fwfm_linear"),
                     fm_1st=w("fm_1st") if self.use_lw else None, bias=getattr(self, "bias", None),
                     lin_w=[w(f"net_1_linear_{i}") for i in range(1, H + 1)],
                     lin_b=[w(f"net_1_linear_{i}", "bias") for i in range(1, H + 1)],
                     fc_w=w("net_1_fc") if self.use_deep else None)
        return fields, dense

    def _prep_inputs(self, Xi, Xv, device):
        ncat = self.field_size - self.num
        Xi = torch.as_tensor(Xi)
        Xv = torch.as_tensor(Xv)
        if Xi.dim() == 3:
            Xi = Xi.reshape(Xi.shape[0], Xi.shape[1])
        if Xi.dim() != 2 or Xi.shape[1] != ncat:
            raise RuntimeError(f"Xi must be [B, {ncat}, 1] or [B, {ncat}], got {tuple(Xi.shape)}")
        if Xv.dim() != 2 or Xv.shape[0] != Xi.shape[0] or Xv.shape[1] < self.num:
            raise RuntimeError(f"Xv must be [B, >= {self.num}], got {tuple(Xv.shape)}")
        Xi = Xi.to(device=device, dtype=torch.int64)
        Xv = Xv.to(device=device, dtype=torch.float32)
        if Xi.stride(1) != 1:
            Xi = Xi.contiguous()
        if Xv.stride(1) != 1:
            Xv = Xv.contiguous()
        return Xi, Xv

    # ---------------------------------------------------------------- forward
    def forward(self, Xi, Xv):
        device = self._device()
        eng = self._sync_engine(device)
        xi, xv = self._prep_inputs(Xi, Xv, device)
        needs_grad = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        if needs_grad:
            from .training import train_forward
            return train_forward(self, eng, xi, xv)
        from . import torch_ops  # torch.ops.dfwfm.forward (the registered custom op)
        if device.type != "cpu":  # (the host kernel has no serving copy or pruned-layout variants)
            self._sync_inference(device)  # the tables' serving copy, re-packed after weight updates
            if self.use_deep:
                # magnitude-pruned hidden layers (fit(prune=1), reference :647-673) run as a sparse MLP when
                # at most sparse_mlp_max_density of their weights are nonzero (checked once per weight update)
                eng.sync_sparse(self.sparse_mlp_max_density)
            elif self.use_fwfm:
                eng.sync_pairs(self.fwfm_pair_max)
        params = [q for q in self.parameters() if q.requires_grad]
        out, _ = torch.ops.dfwfm.forward(torch_ops.register(self), xi, xv, params, False, 0.0, 0)
        if self.strict_index_check and not self._defer_index_check:
            self.check_index_errors()  # reads a device word: synchronises the stream
        return out

    def check_index_errors(self):
        if self._engine is not None and self._engine.read_error_flag() & FLAG_INDEX_OUT_OF_RANGE:
            raise IndexError("index out of range in self (an Xi entry is outside its field's table)")

    @contextlib.contextmanager
    def deferred_index_check(self):
        """Forwards inside the block do not read the out-of-range flag (a host synchronisation per batch);
        it is read once when the block ends and raises IndexError there if any forward saw a bad index --
        the reference raises from the first offending nn.Embedding call (model/DeepFMs.py:334), so a batched
        caller (eval_by_batch, predict, run_benchmark) fails the same way, after its forwards ran."""
        self._defer_index_check = getattr(self, "_defer_index_check", 0) + 1
        ok = False
        try:
            yield
            ok = True
        finally:
            self._defer_index_check -= 1
            if ok and self.strict_index_check and not self._defer_index_check:
                self.check_index_errors()

    # ------------------------------------------------------------ init/train
    def init_weights(self):
        """Same distributions as reference model/DeepFMs.py:472-495, written in place."""
        self.train()
        last_layer_size = 0
        if self.use_fwfm or self.use_fm:
            last_layer_size += self.field_size + self.embedding_size
        if self.use_deep:
            last_layer_size += self.deep_layers[-1] + 1
        glorot = None
        with torch.no_grad():
            for name, p in self.named_parameters():
                if "1st_embeddings" in name:
                    p.normal_()
                elif "2nd_embeddings" in name:
                    p.normal_().mul_(0.01)
                elif "linear" in name:
                    if "weight" in name:
                        glorot = float(np.sqrt(2.0 / np.sum(p.shape)))
                    p.normal_().mul_(glorot)
                elif name == "field_cov.weight":
                    p.normal_().mul_(float(np.sqrt(2.0 / self.field_size / 2)))
                elif name in ("fm_1st.weight", "fm_2nd.weight") or "fc.weight" in name:
                    p.normal_().mul_(float(np.sqrt(2.0 / last_layer_size)))

    def fit(self, Xi_train, Xv_train, y_train, Xi_valid=None, Xv_valid=None, y_valid=None,
            early_stopping=False, refit=False, save_path=None, prune=0, prune_fm=0, prune_r=0,
            prune_deep=0, emb_r=1., emb_corr=1., quantization_aware=False, teacher_model=None):
        from .training import fit
        return fit(self, Xi_train, Xv_train, y_train, Xi_valid, Xv_valid, y_valid, early_stopping, refit,
                   save_path, prune, prune_fm, prune_r, prune_deep, emb_r, emb_corr, teacher_model)

    # ------------------------------------------------------------------ eval
    def _device(self):
        return next(self.parameters()).device

    def _batched_logits(self, Xi, Xv, batch_size):
        """Logits for every row, batch by batch; inputs go to the device once per batch."""
        n = Xi.shape[0]
        out = []
        with torch.no_grad(), self.deferred_index_check():
            for off in range(0, n, batch_size):
                out.append(self(Xi[off:off + batch_size], Xv[off:off + batch_size]))
        return torch.cat(out) if out else torch.empty(0, device=self._device())

    def eval_by_batch(self, Xi, Xv, y, x_size):
        """Reference model/DeepFMs.py:750-784: loss, AUC, PR-AUC, RCE over batches of 8192.  The logits
        stay on the device and the metrics are computed there (metrics.DeviceMetrics, sklearn
        definitions); the loss is the reference's per-batch BCE mean weighted by the batch length."""
        self.eval()
        dev = self._device()
        ncat = self.field_size - self.num
        # row-major on the device: a column-major host array (np.asarray of a DataFrame) keeps its strides
        # through as_tensor / .to(), and the C ABI reads a batch as base pointer + row stride
        Xi_d = torch.as_tensor(np.asarray(Xi)[:x_size]).reshape(x_size, ncat).to(dev, dtype=torch.int64).contiguous()
        Xv_d = torch.as_tensor(np.asarray(Xv)[:x_size], dtype=torch.float32).to(dev).contiguous()
        y_d = torch.as_tensor(np.asarray(y)[:x_size], dtype=torch.float32).to(dev)
        bs = 8192
        logits = torch.empty(x_size, dtype=torch.float32, device=dev)
        total_loss = torch.zeros((), dtype=torch.float64, device=dev)
        with torch.no_grad(), self.deferred_index_check():
            off = 0
            if dev.type == "cuda" and self.eval_batch_sets and x_size >= 2 * bs:
                # the full batches as batch sets (dfwfm_forward_batches: up to 32 resident batches per launch, the
                # same logits as one forward each); the sparse-MLP / pair-list variants keep one forward per batch
                eng = self._sync_inference(dev)
                alt = eng.sync_sparse(self.sparse_mlp_max_density) if self.use_deep else (
                    eng.sync_pairs(self.fwfm_pair_max) if self.use_fwfm else False)
                if not alt:
                    nfull = x_size // bs
                    eng.forward_batches([(Xi_d[i * bs:(i + 1) * bs], Xv_d[i * bs:(i + 1) * bs]) for i in range(nfull)],
                                        [logits[i * bs:(i + 1) * bs] for i in range(nfull)])
                    for i in range(nfull):
                        sl = slice(i * bs, (i + 1) * bs)
                        total_loss += F.binary_cross_entropy_with_logits(logits[sl], y_d[sl]).double() * bs
                    off = nfull * bs
            for off in range(off, x_size, bs):
                end = min(x_size, off + bs)
                out = self(Xi_d[off:end], Xv_d[off:end])
                logits[off:end] = out
                total_loss += F.binary_cross_entropy_with_logits(out, y_d[off:end]).double() * (end - off)
        if self.eval_metric is not metrics.roc_auc_score:  # a user metric gets host arrays, as before
            y_pred = torch.sigmoid(logits).cpu().numpy().astype("float64")
            return (total_loss.item() / x_size, self.eval_metric(np.asarray(y)[:x_size], y_pred),
                    self.compute_prauc(y_pred, np.asarray(y)[:x_size]), self.compute_rce(y_pred, np.asarray(y)[:x_size]))
        if dev.type == "cpu":  # the reference's sklearn metrics on host arrays (:781-783)
            y_pred = torch.sigmoid(logits).numpy().astype("float64")
            yt = np.asarray(y)[:x_size]
            return (total_loss.item() / x_size, metrics.roc_auc_score(yt, y_pred), self.compute_prauc(y_pred, yt),
                    self.compute_rce(y_pred, yt))
        dm = getattr(self, "_dev_metrics", None)
        if dm is None or dm.device != dev:
            dm = self._dev_metrics = metrics.DeviceMetrics(dev)
        m = dm(logits, y_d)
        return total_loss.item() / x_size, m["auc"], m["prauc"], m["rce"]

    def compute_prauc(self, pred, gt):
        return metrics.prauc(gt, pred)

    def calculate_ctr(self, gt):
        return metrics.ctr(gt)

    def compute_rce(self, pred, gt):
        return metrics.rce(gt, pred)

    def cross_entropy(self, predictions, targets):
        return -np.sum(targets * np.log(predictions)) / predictions.shape[0]

    def binary_search_threshold(self, param, target_percent, total_no):
        from .training import binary_search_threshold
        return binary_search_threshold(param, target_percent, total_no)

    def shuffle_in_unison_scary(self, a, b, c):
        state = np.random.get_state()
        for arr in (a, b, c):
            np.random.set_state(state)
            np.random.shuffle(arr)

    def training_termination(self, valid_result):
        if len(valid_result) <= 4:
            return False
        a, b, c, d = valid_result[-1], valid_result[-2], valid_result[-3], valid_result[-4]
        if self.greater_is_better:
            return a < b < c < d
        return a > b > c > d

    def _fit_layout(self, Xi):
        return np.asarray(Xi).reshape((-1, self.field_size - self.num, 1))

    def predict(self, Xi, Xv):
        return self.predict_proba(Xi, Xv) > 0.5

    def predict_proba(self, Xi, Xv):
        # the reference reshapes to [-1, field_size, 1] here (model/DeepFMs.py:865), which cannot
        # match the [-1, field_size - numerical, 1] layout fit() trains on; we take fit's layout.
        Xi = torch.as_tensor(self._fit_layout(Xi))
        Xv = torch.as_tensor(np.asarray(Xv), dtype=torch.float32)
        self.eval()
        with torch.no_grad(), self.deferred_index_check():
            p = torch.sigmoid(self(Xi, Xv))
        return p.cpu().numpy()

    def inner_predict(self, Xi, Xv):
        return self.inner_predict_proba(Xi, Xv) > 0.5

    def inner_predict_proba(self, Xi, Xv):
        self.eval()
        with torch.no_grad(), self.deferred_index_check():
            p = torch.sigmoid(self(Xi, Xv))
        return p.cpu().numpy()

    def evaluate(self, Xi, Xv, y):
        return self.eval_metric(y.cpu().numpy(), self.inner_predict_proba(Xi, Xv))

    def print_size_of_model(self):
        """Checkpoint size and (non-zero) parameter counts, as reference :905-945."""
        self.logger.info("========")
        self.logger.info("MODEL SIZE")
        path = f"temp_{os.getpid()}.p"
        torch.save(self.state_dict(), path)
        size = os.path.getsize(path)
        os.remove(path)
        self.logger.info("\tSize (MB):\t" + str(size / 1e6))
        counts = metrics.parameter_counts(self)
        self.logger.info(f"\tSummation of feature sizes: {sum(self.feature_sizes):,}")
        self.logger.info(f"\tNumber of 1st order embeddings: {counts['emb1']:,}")
        self.logger.info(f"\tNumber of 2nd order embeddings: {counts['emb2']:,}")
        if self.use_fwfm:
            self.logger.info(f"\tNumber of 2nd order interactions: {counts['r_nonzero']:,}")
        if self.use_deep:
            self.logger.info(f"\tNumber of DNN parameters: {counts['dnn']:,}")
        self.logger.info(f"\tNumber of total parameters: {counts['nonzero']:,}")
        self.logger.info(f"\tNon pruned model parameters: \t{counts['total']:,}")
        self.logger.info(f"\tPruned Parameters: \t{counts['total'] - counts['nonzero']:,}")
        self.logger.info("========")
        return size

    def time_forward_pass(self, model, batch_xi, batch_xv, cuda=True):
        """Milliseconds for one forward (reference :1012-1028): HIP events on the current stream for a module on
        the device; on the CPU a host clock (fractional ms -- the reference's time_ns() // 1e6 truncates to whole
        milliseconds, :1024-1027, which reads 0 for most forwards of the host kernel)."""
        dev = self._device()
        batch_xi = batch_xi.to(dev)
        batch_xv = batch_xv.to(dev)
        if dev.type == "cpu":
            t0 = time_ns()
            with torch.no_grad():
                model(batch_xi, batch_xv)
            return (time_ns() - t0) / 1e6
        start = torch.cuda.Event(enable_timing=True)
        end = torch.cuda.Event(enable_timing=True)
        start.record()
        with torch.no_grad():
            model(batch_xi, batch_xv)
        end.record()
        torch.cuda.synchronize()
        return start.elapsed_time(end)

    def run_benchmark(self, Xi, Xv, y, batch_size=8192, cuda=True, quantization_aware=False):
        """Reference :947-1009: metrics, per-batch and per-sample forward times -- on the device with HIP events,
        or (a module on the CPU) the reference's thread sweep: per-batch times at 1 and 4 threads
        (torch.set_num_threads, the host kernel's thread count) and 1000 single-sample latencies at 1 thread."""
        if self._device().type == "cpu":
            return self._run_benchmark_cpu(Xi, Xv, y, batch_size)
        Xi = self._fit_layout(Xi)
        Xv = np.asarray(Xv)
        y = np.asarray(y)
        x_size = Xi.shape[0]
        loss, total_metric, prauc, rce = self.eval_by_batch(Xi, Xv, y, x_size)
        self.logger.info("\tLoss: " + str(loss))
        self.logger.info("\tAcc: " + str(total_metric))
        self.logger.info("\tPRAUC: " + str(prauc))
        self.logger.info("\tRCE: " + str(rce))
        self.eval()
        # the timed forwards never synchronise on the index flag: it is read once, after the timing loops
        with self.deferred_index_check():
            spent = []
            for off in range(0, (x_size // batch_size) * batch_size, batch_size):
                spent.append(self.time_forward_pass(self, torch.as_tensor(Xi[off:off + batch_size]),
                                                    torch.as_tensor(Xv[off:off + batch_size], dtype=torch.float32)))
            if spent:
                self.logger.info("\tAvg forward pass time per batch (HIP)(ms):\t{:.3f}".format(np.mean(spent)))
                self.logger.info("\tAvg forward pass time (batch) (HIP)(ms):\t{:.6f}".format(
                    np.sum(spent) / len(spent) / batch_size))
            single = [self.time_forward_pass(self, torch.as_tensor(Xi[i:i + 1]),
                                             torch.as_tensor(Xv[i:i + 1], dtype=torch.float32))
                      for i in range(min(1000, x_size))]
            if single:
                self.logger.info("\tAvg forward pass time (ms):\t{:.3f}".format(np.mean(single)))
        return loss, total_metric, prauc, rce

    def _run_benchmark_cpu(self, Xi, Xv, y, batch_size):
        Xi = self._fit_layout(Xi)
        Xv = np.asarray(Xv)
        y = np.asarray(y)
        x_size = Xi.shape[0]
        loss, total_metric, prauc, rce = self.eval_by_batch(Xi, Xv, y, x_size)
        self.logger.info("\tLoss: " + str(loss))
        self.logger.info("\tAcc: " + str(total_metric))
        self.logger.info("\tPRAUC: " + str(prauc))
        self.logger.info("\tRCE: " + str(rce))
        self.eval()
        prev = torch.get_num_threads()
        batch_iter = x_size // batch_size
        try:
            with self.deferred_index_check():
                for threads in (1, 4):
                    torch.set_num_threads(threads)
                    spent = [self.time_forward_pass(self, torch.as_tensor(Xi[i * batch_size:(i + 1) * batch_size]),
                                                    torch.as_tensor(Xv[i * batch_size:(i + 1) * batch_size],
                                                                    dtype=torch.float32))
                             for i in range(batch_iter)]
                    # logged even without a full batch (nan), as the reference does
                    mean = float(np.mean(spent)) if spent else float("nan")
                    self.logger.info("\tAvg forward pass time per batch ({}-Threads)(ms):\t{:.3f}".format(threads, mean))
                    self.logger.info("\tAvg forward pass time (batch) ({}-Threads)(ms):\t{:.6f}".format(
                        threads, mean / batch_size))
                torch.set_num_threads(1)
                single = [self.time_forward_pass(self, torch.as_tensor(Xi[i:i + 1]),
                                                 torch.as_tensor(Xv[i:i + 1], dtype=torch.float32))
                          for i in range(min(1000, x_size))]
                if single:
                    self.logger.info("\tAvg forward pass time (ms):\t{:.3f}".format(np.mean(single)))
        finally:
            torch.set_num_threads(prev)
        return loss, total_metric, prauc, rce

    def fetch_teacher_outputs(self, teacher_model, Xi, Xv, x_size):
        teacher_model.eval()
        outs = []
        with torch.no_grad():
            for off in range(0, x_size, self.batch_size):
                outs.append(teacher_model(torch.as_tensor(Xi[off:off + self.batch_size]),
                                          torch.as_tensor(Xv[off:off + self.batch_size], dtype=torch.float32))
                            .cpu().numpy())
        return outs

    def loss_fn_kd(self, outputs, teacher_outputs, y):
        alpha, T = 0.9, 20
        kd = nn.KLDivLoss()(F.log_softmax(outputs / T, dim=0), F.softmax(teacher_outputs / T, dim=0))
        return kd * (alpha * T * T) + F.binary_cross_entropy_with_logits(outputs, y) * (1. - alpha)

    # ----------------------------------------------------------- pickling
    def __getstate__(self):
        d = self.__dict__.copy()
        if "logger" in d and not isinstance(d["logger"], str):
            d["logger"] = d["logger"].name
        d["_engine"] = None
        return d

    def __setstate__(self, d):
        if "logger" in d and isinstance(d["logger"], str):
            d["logger"] = logging.getLogger(d["logger"])
        self.__dict__.update(d)
