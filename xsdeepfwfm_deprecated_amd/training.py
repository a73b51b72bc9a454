"""Training path of DeepFMs (reference model/DeepFMs.py:497-748, 807-823) on the HIP kernels.

* ``train_forward``: ``torch.ops.dfwfm.forward`` in training mode (torch_ops.py: the fused HIP
  forward keeping its activations, deep-tower dropout from a counter hash) whose registered backward
  is the fused HIP backward (csrc/dfwfm_train.hip) writing every parameter's gradient -- dense, like
  the reference's ``nn.Embedding(sparse=False)`` -- into one flat per-step buffer.
* ``Adam``: ``torch.optim.Adam`` (coupled L2, bias correction) as one HIP kernel per <= 40 tensors,
  same defaults and ``state_dict`` layout.
* ``fit``: the reference's epoch loop -- init_weights, optimizer, BCE-with-logits (or the KD loss),
  magnitude pruning, per-epoch eval, shuffle, save, early stopping -- with the training set
  resident in HBM and, under ``torch.distributed``, data parallelism: each rank takes its slice of
  every global batch and the flat gradient buffer is all-reduced (RCCL) before the step.

A module on the CPU trains through the host kernels (libdfwfm_cpu.so: the custom op's CPU kernel and its
backward) with torch.optim.Adam -- the reference's -use_cuda 0 path; a module on the device never leaves it.
"""
from __future__ import annotations

import ctypes
import logging
import math
import os
from time import time

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib
from . import engine as _engine


# --------------------------------------------------------------------------------------- autograd
def _grad_buffer(params, need, device):
    """One zeroed flat buffer holding every needed gradient (a single memset and, under data
    parallelism, a single all-reduce); returns it and per-parameter views (None where not needed)."""
    sizes = [p.numel() if n else 0 for p, n in zip(params, need)]
    flat = torch.zeros(sum(sizes), dtype=torch.float32, device=device)
    views, off = [], 0
    for p, n, sz in zip(params, need, sizes):
        views.append(flat[off:off + sz].view_as(p) if n else None)
        off += sz
    return flat, views


def train_forward(model, eng, xi, xv):
    """Logits with a HIP backward attached (reference forward in training mode, :285-469)."""
    if model.training and model.is_shallow_dropout and model.dropout_shallow and \
            any(float(p) != 0.0 for p in model.dropout_shallow[:2]):
        raise NotImplementedError("dfwfm: shallow dropout p > 0 is not supported (the reference default is 0)")
    p = 0.0
    if model.training and model.use_deep and model.is_deep_dropout:
        p = float(model.dropout_deep[0])
        if any(float(d) != p for d in model.dropout_deep):
            raise NotImplementedError("dfwfm: per-layer dropout rates must be equal")
    seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if p > 0 else 0
    from . import torch_ops
    params = [q for q in model.parameters() if q.requires_grad]
    out, _ = torch.ops.dfwfm.forward(torch_ops.register(model), xi, xv, params, True, p, seed)
    return out


# --------------------------------------------------------------------------------------- Adam
class Adam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad=False, maximize=False) with the update on the HIP kernel.

    Same hyper-parameters, same per-parameter state (``step``, ``exp_avg``, ``exp_avg_sq``), so a
    ``state_dict`` moves between this and torch's Adam.  Parameters must be float32 HIP tensors."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if lr < 0.0 or eps < 0.0 or weight_decay < 0.0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError("invalid Adam hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                                      amsgrad=False, maximize=False, foreach=None, capturable=False,
                                      differentiable=False, fused=None))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            if group.get("amsgrad") or group.get("maximize"):
                raise NotImplementedError("dfwfm Adam: amsgrad / maximize")
            by_step = {}
            device = None
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("dfwfm Adam: sparse gradients are not supported")
                if p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous():
                    raise RuntimeError("dfwfm Adam: parameters must be contiguous float32 HIP tensors")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                by_step.setdefault(int(st["step"].item()), []).append((p, g, st["exp_avg"], st["exp_avg_sq"]))
                device = p.device
            b1, b2 = group["betas"]
            for step, entries in by_step.items():
                _engine.adam_step(entries, group["lr"], b1, b2, group["eps"], group["weight_decay"], step, device)
                for p, *_ in entries:
                    torch.autograd.graph.increment_version(p)  # in-place update behind torch's back
        return loss


# --------------------------------------------------------------------------------------- fused step
def gather_packed(dist, send, recv, async_op=True):
    """All-gather of one packed byte buffer per rank (touched-row lists: [dest | rows | counts], fixed
    capacity, so no size exchange and no host synchronisation) into recv [world, nbytes]: one collective
    (RCCL all_gather_into_tensor; gloo: the list form)."""
    if dist.get_backend() == "nccl":
        return dist.all_gather_into_tensor(recv.view(-1), send, async_op=async_op)
    return dist.all_gather(list(recv.unbind(0)), send, async_op=async_op)


def packed_layout(fams):
    """Byte layout of one rank's touched-row lists in the exchanged buffer: [dest int64 per family | rows f32 per
    family | counts int32], for fams = [{"cap": entries, "w": row width}, ...]; sets each family's o_dest / o_rows /
    o_cnt and returns the buffer's size.  Every section starts 16-byte aligned and the size is a multiple of 16, so
    each rank's slice of the all-gathered [world, nbytes] buffer keeps the int64 destination lists aligned."""
    a16 = lambda x: (x + 15) & ~15  # noqa: E731
    nbytes = 0
    for f in fams:
        f["o_dest"] = nbytes
        nbytes = a16(nbytes + 8 * f["cap"])
    for f in fams:
        f["o_rows"] = nbytes
        nbytes = a16(nbytes + 4 * f["cap"] * f["w"])
    for i, f in enumerate(fams):
        f["o_cnt"] = nbytes + 4 * i
    return a16(nbytes + 4 * len(fams))


# the exchange's receive workspace: world x packed bytes, all-gathered in one collective and walked by
# dfwfm_sparse_grads_apply, whose grid and per-list counts are 32-bit (DFWFM_DP_EXCHANGE_MAX_BYTES lowers it)
EXCHANGE_MAX_BYTES = 2 ** 31 - 1


def check_exchange(world, nbytes, fams, max_bytes=None):
    """Refuse, before anything is allocated or captured, a data-parallel exchange whose all-gathered receive buffer
    (world x nbytes of packed touched-row lists) would exceed the exchange workspace, or a list too long for the
    apply kernel's 32-bit counts / grid.  Returns the receive buffer's size in bytes."""
    limit = int(max_bytes if max_bytes is not None else
                os.environ.get("DFWFM_DP_EXCHANGE_MAX_BYTES", EXCHANGE_MAX_BYTES))
    total = int(world) * int(nbytes)
    if world < 1:
        raise ValueError(f"data-parallel exchange: world size {world}")
    if total > limit:
        raise ValueError(f"data-parallel exchange: {world} ranks x {nbytes:,} bytes of packed touched-row lists = "
                         f"{total:,} bytes exceed the exchange workspace ({limit:,} bytes); use fewer ranks, a "
                         f"smaller per-rank batch, or sparse_exchange=False (dense all-reduce of the tables)")
    for f in fams:
        if f["cap"] * f["w"] > 2 ** 31 - 1:
            raise ValueError(f"data-parallel exchange: a list of {f['cap']:,} rows x {f['w']} floats exceeds the "
                             "apply kernel's 32-bit grid")
    return total




class FusedTrainStep:
    """One reference training step -- fit()'s inner-loop body (:619-637): zero_grad, forward,
    BCE-with-logits, backward, Adam(lr, weight_decay) -- as HIP launches on pre-built pointers, captured
    once into a HIP graph and replayed (no per-step host work beyond the input copies).

    Gradients and Adam moments live in flat device buffers (``p.grad`` are views into the gradient
    buffer, so a data-parallel all-reduce is one call).  Adam's step counter and bias corrections, and
    the dropout seed, are read from device memory, so every replay is a fresh step.  Under
    torch.distributed the loss is normalised by the global batch and the step is split into two graphs
    around an RCCL all-reduce of the gradient buffer.

    resident_inputs: full batches whose (xi, xv, y) tensors recur (a ring of device-resident input buffers,
    e.g. a loader double-buffering into fixed tensors) are read in place -- one captured graph set per buffer
    set (at most ``max_graph_sets``, least recently used dropped) -- instead of being copied into the step's
    own input buffers first (three copy launches per step).  step_many (several steps per graph) needs it: its
    graphs read their batches in place and live in a cache of their own (``max_many_sets``)."""

    def __init__(self, model, batch_size, lr=1e-3, weight_decay=0.0, betas=(0.9, 0.999), eps=1e-8,
                 use_graph=True, dist=None, sparse_exchange=True, resident_inputs=False, max_graph_sets=8,
                 max_many_sets=2, deterministic=None):
        dev = model._device()
        if dev.type != "cuda":
            raise _lib.DfwfmError("FusedTrainStep runs only on a HIP device")
        self.model, self.dev = model, dev
        self.B = int(batch_size)
        self.lr, self.wd, self.betas, self.eps = float(lr), float(weight_decay), tuple(betas), float(eps)
        self.dist = dist
        self.use_graph = use_graph
        self.resident_inputs = bool(resident_inputs)
        self.max_graph_sets = max(1, int(max_graph_sets))
        self._graph_sets = {}  # (denom, drop, deterministic, workspace generation, input pointers) -> (graphs, inputs)
        self.max_many_sets = max(1, int(max_many_sets))
        self._many_sets = {}  # step_many's K-step graphs, keyed like _graph_sets (their own LRU: no evictions of step()'s)
        self.eng = model._sync_engine(dev)
        self.L = _lib.lib()
        # fixed-order gradient sums (bit-identical runs); default: the model's `deterministic` switch
        self.deterministic = bool(model.deterministic if deterministic is None else deterministic)
        params = [p for p in model.parameters() if p.requires_grad]
        fields, dense = model._param_layout()
        known = {id(t) for tup in fields for t in tup if t is not None}
        known |= {id(v) for k, v in dense.items() if not isinstance(v, list) and v is not None}
        known |= {id(t) for t in dense["lin_w"] + dense["lin_b"]}
        if any(id(p) not in known for p in params):
            raise NotImplementedError("FusedTrainStep: a trainable parameter outside the kernels' layout")
        # gradient buffer order: [categorical tables | the rest of what the backward's first part writes
        # (numerical-field tables, shallow dense, net_1_fc) | the MLP weights / biases the weight-gradient
        # GEMM writes last].  Under data parallelism the tables go over the sparse touched-row exchange
        # (sparse_exchange, dfwfm_sparse_grads_local) and the two dense buckets over all-reduces, the first one
        # overlapping the GEMM; with sparse_exchange=False the tables join the first all-reduce (dense, like
        # the reference's nn.Embedding(sparse=False) gradients)
        mlp_ids = {id(t) for t in dense["lin_w"] + dense["lin_b"]}
        cat_ids = {id(t) for f, tup in enumerate(fields) if f >= model.num for t in tup if t is not None}
        params = [p for p in params if id(p) in cat_ids] + \
            [p for p in params if id(p) not in mlp_ids and id(p) not in cat_ids] + \
            [p for p in params if id(p) in mlp_ids]
        # every tensor's slice starts 16-byte aligned (offsets padded to 4 floats; the pads stay zero), so
        # the Adam kernel takes its 16-byte path on every tensor
        offs, total = [], 0
        for p in params:
            offs.append(total)
            total += (p.numel() + 3) & ~3
        self.n_tables = next((offs[i] for i, p in enumerate(params) if id(p) not in cat_ids), total)
        self.n_bucket_a = next((offs[i] for i, p in enumerate(params) if id(p) in mlp_ids), total)
        self.sparse = dist is not None and bool(sparse_exchange) and self.n_tables > 0
        self.grad = torch.zeros(total, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(total, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(total, dtype=torch.float32, device=dev)
        self.state = torch.zeros(_lib.ADAM_STATE_BYTES // 8, dtype=torch.int64, device=dev)
        # under data parallelism Adam runs as two launches -- everything but the MLP
        # (state), the MLP weights and biases (state_b) -- so that the first can overlap the weight-gradient GEMM;
        # each state's step counter is bumped once per step, so both hold the same step and bias corrections.  On one
        # process the split is tables (state_t) / everything else (state) instead (split_adam, below)
        self.state_b = torch.zeros_like(self.state)
        # one process: the categorical tables' Adam runs on the scatter's side stream right behind it (its own
        # counter, state_t), beside the weight-gradient GEMM; everything else on `state` after the GEMM
        self.state_t = torch.zeros_like(self.state)
        views = {}
        adam = (_lib.dfwfm_adam_tensor * len(params))()
        for i, p in enumerate(params):
            n, off = p.numel(), offs[i]
            g, m, v = (t[off:off + n].view_as(p) for t in (self.grad, self.exp_avg, self.exp_avg_sq))
            p.grad = g
            views[id(p)] = g
            adam[i] = _lib.dfwfm_adam_tensor(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), n)
        self.params, self.adam, self.n_adam = params, adam, len(params)
        self.n_main = sum(1 for p in params if id(p) not in mlp_ids)  # params are ordered with the MLP last
        self.adam_mlp = ctypes.cast(ctypes.addressof(adam) + self.n_main * ctypes.sizeof(_lib.dfwfm_adam_tensor),
                                    ctypes.POINTER(_lib.dfwfm_adam_tensor))
        self.n_cat = sum(1 for p in params if id(p) in cat_ids)  # params are ordered with the tables first
        self.adam_rest = ctypes.cast(ctypes.addressof(adam) + self.n_cat * ctypes.sizeof(_lib.dfwfm_adam_tensor),
                                     ctypes.POINTER(_lib.dfwfm_adam_tensor))
        # one process: Adam as two launches, the categorical tables (state_t) and the rest (state), on every path
        # (eager, graph, step_many), so the two counters always hold the same step
        self.split_adam = dist is None and 0 < self.n_cat < len(params)
        ptr = lambda t: None if t is None else views[id(t)].data_ptr()  # noqa: E731
        # sparse exchange: the backward scatters the categorical tables' gradients into a rank-local buffer (same
        # offsets as in self.grad, whose categorical region the lists fill); dfwfm_sparse_grads_local turns its
        # touched rows into the lists (and clears them), and every rank adds every rank's lists (_apply_sparse)
        if self.sparse:
            self.grad_local = torch.zeros(self.n_tables, dtype=torch.float32, device=dev)
            self.stamp = torch.empty(self.n_tables, dtype=torch.int32, device=dev)  # scratch, any contents
            lbase, gbase = self.grad_local.data_ptr(), self.grad.data_ptr()
            lptr = lambda t: None if t is None else lbase + (views[id(t)].data_ptr() - gbase)  # noqa: E731
        self.fg = (_lib.dfwfm_field_grads * len(fields))(
            *[_lib.dfwfm_field_grads(*[(lptr(t) if (self.sparse and f >= model.num) else ptr(t)) for t in tup])
              for f, tup in enumerate(fields)])
        H = len(dense["lin_w"])
        self.gW = (ctypes.c_void_p * max(H, 1))(*[ptr(t) for t in dense["lin_w"]])
        self.gB = (ctypes.c_void_p * max(H, 1))(*[ptr(t) for t in dense["lin_b"]])
        self.grads = _lib.dfwfm_grads(self.fg, ptr(dense["field_cov"]), ptr(dense["fwfm_lin"]), ptr(dense["fm_1st"]),
                                      ptr(dense["bias"]), self.gW if H else None, self.gB if H else None,
                                      ptr(dense["fc_w"]))
        # set_dense arguments (re-packed inside every step: Adam changes the weights)
        d = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
        self.pW = (ctypes.c_void_p * max(H, 1))(*[t.data_ptr() for t in dense["lin_w"]])
        self.pB = (ctypes.c_void_p * max(H, 1))(*[t.data_ptr() for t in dense["lin_b"]])
        self.dense_args = (d(dense["field_cov"]), d(dense["fwfm_lin"]), d(dense["fm_1st"]), d(dense["bias"]),
                           self.pW if H else None, self.pB if H else None, d(dense["fc_w"]))
        ncat, num = model.field_size - model.num, model.num
        self.ncat, self.num = ncat, num
        self.xi = torch.zeros(self.B, max(ncat, 1), dtype=torch.int64, device=dev)
        self.xv = torch.zeros(self.B, max(num, 1), dtype=torch.float32, device=dev)
        self.y = torch.zeros(self.B, dtype=torch.float32, device=dev)
        self._in = (self.xi, self.xv, self.y)  # the inputs _part1 launches on
        self.out = torch.zeros(self.B, dtype=torch.float32, device=dev)
        self.dlogit = torch.zeros(self.B, dtype=torch.float32, device=dev)
        self.loss_sum = torch.zeros(1, dtype=torch.float32, device=dev)
        self.drop_train = 0.0
        if model.use_deep and model.is_deep_dropout:
            self.drop_train = float(model.dropout_deep[0])
        self.drop = self.drop_train
        self.seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
        _lib.check(self.L.dfwfm_set_step_source(self.eng.handle, ctypes.c_void_p(self.state.data_ptr())),
                   "dfwfm_set_step_source")
        self._attached = True
        self.graphs = None
        self.steps = 0
        if self.sparse:
            self._setup_sparse(fields, views)

    # -- touched-row exchange of the categorical tables' gradients (data parallelism) ------------------
    def _setup_sparse(self, fields, views):
        """Per table family (second-order rows of width D, first-order rows of width 1) the list buffers of
        dfwfm_sparse_grads_local, packed into ONE byte buffer per rank so the exchange is one all-gather:
        [dest int64 per family | rows f32 per family | counts int32]."""
        L, h = self.L, self.eng.handle
        base = self.grad.data_ptr()

        def off(t):
            return -1 if t is None else (views[id(t)].data_ptr() - base) // 4
        fams = []
        for fam, (iq, ir) in ((_lib.FAMILY_SECOND, (0, 1)), (_lib.FAMILY_FIRST, (2, 3))):
            dest = (_lib.dfwfm_sparse_dest * len(fields))(
                *[_lib.dfwfm_sparse_dest(off(tup[iq]) if f >= self.model.num else -1,
                                         off(tup[ir]) if f >= self.model.num else -1)
                  for f, tup in enumerate(fields)])
            cap, w, ws = ctypes.c_int64(0), ctypes.c_int32(0), ctypes.c_int64(0)
            _lib.check(L.dfwfm_sparse_grads_size(h, fam, self.B, ctypes.byref(cap), ctypes.byref(w), ctypes.byref(ws)),
                       "dfwfm_sparse_grads_size")
            if cap.value > 0:
                fams.append(dict(fam=fam, dest=dest, cap=int(cap.value), w=int(w.value), ws_bytes=int(ws.value)))
        nbytes = packed_layout(fams)
        world = self.dist.get_world_size()
        check_exchange(world, nbytes, fams)  # refused before any buffer is allocated or a graph captured
        self.sp_send = torch.zeros(nbytes, dtype=torch.uint8, device=self.dev)
        self.sp_recv = torch.zeros(world, nbytes, dtype=torch.uint8, device=self.dev)
        self.sp_fams = fams
        self.sp_bytes = nbytes

    def _sparse_lists(self, st):
        """This rank's touched-row lists of the step just run (part of the first graph): the touched rows of the
        rank-local dense table gradients the backward scattered (claimed once each, copied, cleared)."""
        for f in self.sp_fams:
            sb = self.sp_send.data_ptr()
            _lib.check(self.L.dfwfm_sparse_grads_local(
                self.eng.handle, f["fam"], f["dest"], f["cap"], ctypes.c_void_p(self.grad_local.data_ptr()),
                ctypes.c_void_p(self.stamp.data_ptr()), self.n_tables, ctypes.c_void_p(sb + f["o_dest"]),
                ctypes.c_void_p(sb + f["o_rows"]), ctypes.c_void_p(sb + f["o_cnt"]), st), "dfwfm_sparse_grads_local")

    def _gather_sparse(self):
        return gather_packed(self.dist, self.sp_send, self.sp_recv)

    def _apply_sparse(self):
        """Every rank adds rank 0's lists, then rank 1's, ... into its dense table gradients (zeroed at the
        step's start): the same additions in the same order on every rank -> bit-identical replicas."""
        st = self._stream()
        g = ctypes.c_void_p(self.grad.data_ptr())
        for r in range(self.sp_recv.shape[0]):
            rb = self.sp_recv[r].data_ptr()
            for f in self.sp_fams:
                _lib.check(self.L.dfwfm_sparse_grads_apply(g, f["w"], ctypes.c_void_p(rb + f["o_dest"]),
                                                           ctypes.c_void_p(rb + f["o_rows"]),
                                                           ctypes.c_void_p(rb + f["o_cnt"]), f["cap"], st),
                           "dfwfm_sparse_grads_apply")

    def close(self):
        """Detach the engine from this step's device counter (the engine outlives the trainer: a later
        train forward must not read the freed counter).  Idempotent; also run by __del__."""
        eng = getattr(self, "eng", None)
        if eng is not None and eng.handle is not None and eng.handle.value and getattr(self, "_attached", False):
            self.L.dfwfm_set_step_source(eng.handle, None)
        self._attached = False
        self.graphs = None
        self._graph_sets = {}
        self._many_sets = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _ws_generation(self):
        g = ctypes.c_int64(0)
        _lib.check(self.L.dfwfm_workspace_generation(self.eng.handle, ctypes.byref(g)), "dfwfm_workspace_generation")
        return int(g.value)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)

    def _part1(self, n, denom, phases=None):
        L, st, h = self.L, self._stream(), self.eng.handle
        self.eng.set_deterministic(self.deterministic)  # read when the backward launches are enqueued / captured
        # the dense weights re-packed and the gradient buffer zeroed in one launch
        _lib.check(L.dfwfm_model_set_dense_zero(h, *self.dense_args, ctypes.c_void_p(self.grad.data_ptr()),
                                                self.grad.numel(), st), "dfwfm_model_set_dense_zero")
        xi, xv, y = self._in
        _lib.check(L.dfwfm_train_forward(h, ctypes.c_void_p(xi.data_ptr()), xi.stride(0),
                                         ctypes.c_void_p(xv.data_ptr()), xv.stride(0), n,
                                         ctypes.c_void_p(self.out.data_ptr()), self.drop, self.seed, st),
                   "dfwfm_train_forward")
        if phases is None:
            phases = _lib.BWD_TABLES if self._bucketed() else (_lib.BWD_TABLES | _lib.BWD_MLP_WEIGHTS)
        # the loss gradient rides in the per-tile backward (dfwfm_backward_phases_bce: the same dlogit bits as
        # dfwfm_bce_grad, one launch fewer)
        _lib.check(L.dfwfm_backward_phases_bce(h, ctypes.c_void_p(self.out.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                                               float(denom), ctypes.c_void_p(self.dlogit.data_ptr()),
                                               ctypes.c_void_p(self.loss_sum.data_ptr()), ctypes.byref(self.grads),
                                               phases, st), "dfwfm_backward_phases_bce")
        if self.sparse:
            self._sparse_lists(st)

    def _backward_phase(self, phases):
        self.eng.set_deterministic(self.deterministic)
        _lib.check(self.L.dfwfm_backward_phases(self.eng.handle, ctypes.c_void_p(self.dlogit.data_ptr()),
                                                ctypes.byref(self.grads), phases, self._stream()),
                   "dfwfm_backward_phases")

    def _part1b(self):
        """The MLP weight gradients (dW_l, db_l): the backward's second part under data parallelism."""
        self.eng.set_deterministic(self.deterministic)
        _lib.check(self.L.dfwfm_backward_phases(self.eng.handle, ctypes.c_void_p(self.dlogit.data_ptr()),
                                                ctypes.byref(self.grads), _lib.BWD_MLP_WEIGHTS, self._stream()),
                   "dfwfm_backward_phases")

    def _one_process_step(self, denom, s, s1):
        """One step on one process, captured on stream s: forward, loss gradient, per-tile backward; the table scatter
        on s1 beside the reductions' final sums + weight-gradient GEMM on s; Adam after both."""
        self._part1(self.B, denom, phases=_lib.BWD_TILES)
        # (the scatter alone first, then the GEMM beside the tables' Adam: 0.2799-0.2818 ms against 0.2715-0.2720,
        # profiles/r06/r06_layout.log -- the latency-bound scatter is best hidden under the GEMM)
        s1.wait_stream(s)
        with torch.cuda.stream(s1):
            self._backward_phase(_lib.BWD_SCATTER)
            if self.split_adam:  # the tables' Adam right behind their scatter, beside the GEMM
                self._adam_range(self.adam, self.n_cat, self.state_t)
        self._backward_phase(_lib.BWD_REDUCE | _lib.BWD_MLP_WEIGHTS)
        if self.split_adam:
            self._adam_range(self.adam_rest, self.n_adam - self.n_cat, self.state)
        else:
            self._part2()
        s.wait_stream(s1)

    def _adam_range(self, tensors, n, state):
        b1, b2 = self.betas
        _lib.check(self.L.dfwfm_adam_step_dev(tensors, n, self.lr, b1, b2, self.eps, self.wd,
                                              ctypes.c_void_p(state.data_ptr()), self._stream()),
                   "dfwfm_adam_step_dev")

    def _bucketed(self):
        return self.dist is not None and self.n_bucket_a < self.grad.numel()

    def _adam_main(self):
        b1, b2 = self.betas
        if self.n_main:
            _lib.check(self.L.dfwfm_adam_step_dev(self.adam, self.n_main, self.lr, b1, b2, self.eps, self.wd,
                                                  ctypes.c_void_p(self.state.data_ptr()), self._stream()),
                       "dfwfm_adam_step_dev")

    def _adam_mlp(self):
        b1, b2 = self.betas
        if self.n_adam > self.n_main:
            _lib.check(self.L.dfwfm_adam_step_dev(self.adam_mlp, self.n_adam - self.n_main, self.lr, b1, b2, self.eps,
                                                  self.wd, ctypes.c_void_p(self.state_b.data_ptr()), self._stream()),
                       "dfwfm_adam_step_dev")

    def _part2(self):
        if self.split_adam:  # the tables (state_t) then the rest (state): both counters bumped every step
            self._adam_range(self.adam, self.n_cat, self.state_t)
            self._adam_range(self.adam_rest, self.n_adam - self.n_cat, self.state)
            return
        if self.dist is None:
            self._adam_all()  # one counter (`state`) for every step of this instance, graph-replayed or not
            return
        self._adam_main()
        self._adam_mlp()

    def _adam_all(self):
        """Every tensor's Adam in one launch (one step counter, `state`): one process without categorical tables."""
        b1, b2 = self.betas
        _lib.check(self.L.dfwfm_adam_step_dev(self.adam, self.n_adam, self.lr, b1, b2, self.eps, self.wd,
                                              ctypes.c_void_p(self.state.data_ptr()), self._stream()),
                   "dfwfm_adam_step_dev")

    def _exchange(self, run_part1b, run_apply=None):
        """Data parallelism: all-reduce the gradient buffer (RCCL).  Bucketed: the first bucket (every
        gradient but the MLP weights') goes out as soon as the backward's first part is done and runs
        while the weight-gradient GEMM (run_part1b) forms the second bucket; otherwise one call."""
        if self.dist is None:
            run_part1b()
            return
        if self.sparse:
            # dense bucket (everything but the categorical tables and the MLP) and the touched-row lists go
            # out while the weight-gradient GEMM runs; then the MLP bucket; then every rank's lists are added
            lo, hi = self.n_tables, self.n_bucket_a
            works = [self._gather_sparse()]
            if hi > lo:
                works.append(self.dist.all_reduce(self.grad[lo:hi], async_op=True))
            run_part1b()
            if self.grad.numel() > hi:
                works.append(self.dist.all_reduce(self.grad[hi:], async_op=True))
            for w in works:
                w.wait()
            run_apply()
            return
        if not self._bucketed():
            run_part1b()
            self.dist.all_reduce(self.grad)
            return
        wa = self.dist.all_reduce(self.grad[:self.n_bucket_a], async_op=True)
        run_part1b()
        wb = self.dist.all_reduce(self.grad[self.n_bucket_a:], async_op=True)
        wa.wait()
        wb.wait()

    def _replay_dp(self, g1b, ga, g2, g2b):
        """The data-parallel step after the first graph, as two streams: a side stream runs the weight-gradient
        GEMM (queued first, so the GPU has it while the host issues the collectives), the MLP bucket's
        all-reduce and the MLP's Adam; the current stream waits for the first bucket (and the touched-row
        lists), adds the lists and runs the main Adam (tables and the shallow part).  The two halves write
        disjoint parameters and Adam states, so the order between them is free."""
        if self.dist is None:  # one process without an MLP: the backward is whole in the first graph
            g2.replay()
            return
        cur = torch.cuda.current_stream(self.dev)
        if g1b is not None:
            if getattr(self, "_side", None) is None:
                self._side = torch.cuda.Stream(self.dev)
            side = self._side
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                g1b.replay()
        lo, hi = (self.n_tables if self.sparse else 0), self.n_bucket_a
        works = [self._gather_sparse()] if self.sparse else []
        if hi > lo:
            works.append(self.dist.all_reduce(self.grad[lo:hi], async_op=True))
        if g1b is not None:
            with torch.cuda.stream(side):
                if self.grad.numel() > hi:
                    self.dist.all_reduce(self.grad[hi:], async_op=True).wait()
                g2b.replay()
        for w in works:
            w.wait()
        if ga is not None:
            ga.replay()
        g2.replay()
        if g1b is not None:
            cur.wait_stream(side)

    def _comm_in_graph(self):
        """Whether the step's collectives are captured into its graph: RCCL (gloo's are host calls), unless
        DFWFM_DP_GRAPH_COMM=0."""
        return (self.dist is not None and self.dist.get_backend() == "nccl"
                and os.environ.get("DFWFM_DP_GRAPH_COMM", "1") != "0")

    def _capture(self, denom):
        """Graphs: forward + backward (its MLP-weight part separately under DP, see _exchange), then Adam;
        the RCCL all-reduces run between them.  Captures are thread-local: the process group's watchdog thread
        queries its events while a step is being captured, which under the global mode invalidates the capture."""
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        g1, g1b, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        ga = None
        if self.dist is None and self.n_adam > self.n_main:
            # one process, one graph: fill, re-pack, forward, loss gradient and per-tile backward; then the table
            # scatter and the tables' Adam on a side stream beside the reductions' final sums + weight-gradient GEMM
            # (one launch) and the other tensors' Adam.  The scatter (latency-bound: one 512-thread workgroup per
            # bucket, 60 KB of LDS) fits on the CUs beside the GEMM's 225 register-heavy four-wave workgroups, and the
            # tables' HBM-bound Adam streams beside its MFMAs: 0.2722 -> 0.2665 ms per step with the scatter alone
            # there (profiles/r06/r06_fork.log), -8 us more with the tables' Adam (r06_splitadam.log).  (Round 4's
            # forks -- the GEMM and the MLP's Adam beside the reductions / atomic scatter / main Adam -- measured
            # level: what ran beside the GEMM was starved of CU slots.)
            s1 = torch.cuda.Stream(self.dev)
            with torch.cuda.stream(s):
                with torch.cuda.graph(g1, stream=s, capture_error_mode="thread_local"):
                    self._one_process_step(denom, s, s1)
            torch.cuda.current_stream(self.dev).wait_stream(s)
            return g1, None, None, None, None
        if self._comm_in_graph():
            # RCCL: the collectives are captured too, so the whole data-parallel step is one graph (no host
            # round trips between its parts).  The first bucket and the lists go out right after the backward's
            # first part; the weight-gradient GEMM, the MLP bucket and the MLP's Adam fork onto s1 (the RCCL
            # stream runs the collectives in issue order: lists, first bucket, then the MLP bucket behind the GEMM)
            s1 = torch.cuda.Stream(self.dev)
            lo, hi = (self.n_tables if self.sparse else 0), self.n_bucket_a
            with torch.cuda.stream(s):
                with torch.cuda.graph(g1, stream=s, capture_error_mode="thread_local"):
                    self._part1(self.B, denom)
                    bucketed = self._bucketed()
                    if bucketed:
                        s1.wait_stream(s)
                    if self.sparse:
                        gather_packed(self.dist, self.sp_send, self.sp_recv, async_op=False)
                    if hi > lo:
                        self.dist.all_reduce(self.grad[lo:hi])
                    if bucketed:
                        with torch.cuda.stream(s1):
                            self._part1b()
                            if self.grad.numel() > hi:
                                self.dist.all_reduce(self.grad[hi:])
                            self._adam_mlp()
                    if self.sparse:
                        self._apply_sparse()
                    if bucketed:
                        self._adam_main()
                        s.wait_stream(s1)
                    else:
                        self._part2()
            torch.cuda.current_stream(self.dev).wait_stream(s)
            return g1, None, None, None, None
        with torch.cuda.stream(s):
            with torch.cuda.graph(g1, stream=s, capture_error_mode="thread_local"):
                self._part1(self.B, denom)
            if self._bucketed():
                with torch.cuda.graph(g1b, stream=s, capture_error_mode="thread_local"):
                    self._part1b()
            else:
                g1b = None
            if self.sparse:
                ga = torch.cuda.CUDAGraph()
                with torch.cuda.graph(ga, stream=s, capture_error_mode="thread_local"):
                    self._apply_sparse()
            # bucketed: the MLP's Adam is its own graph, replayed on a side stream behind the weight-gradient
            # GEMM and the MLP bucket's all-reduce, while the main Adam runs behind the first bucket (_replay_dp)
            g2b = None
            with torch.cuda.graph(g2, stream=s, capture_error_mode="thread_local"):
                if g1b is not None:
                    self._adam_main()
                else:
                    self._part2()
            if g1b is not None:
                g2b = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g2b, stream=s, capture_error_mode="thread_local"):
                    self._adam_mlp()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        return g1, g1b, ga, g2, g2b

    def _direct_inputs(self, xi, xv, y, n):
        """(xi, xv, y) as the graphs can read them in place, or None (then they are copied): a full batch of
        row-contiguous int64 indices, float32 values and float32 labels on this device."""
        xi2 = xi.reshape(n, -1) if xi.is_contiguous() else None
        if (xi2 is None or xi2.dtype != torch.int64 or xi2.device != self.dev or xi2.shape[1] != self.xi.shape[1]
                or y.dtype != torch.float32 or y.device != self.dev or y.dim() != 1 or not y.is_contiguous()
                or y.shape[0] != n):
            return None
        if self.num:
            if (xv.dtype != torch.float32 or xv.device != self.dev or xv.dim() != 2 or xv.stride(1) != 1
                    or xv.shape[1] < self.num or xv.shape[0] < n):
                return None
        else:
            xv = self.xv
        return (xi2, xv, y)

    def step(self, xi, xv, y, n_global=None):
        """One step on device tensors xi [n, F-num] int64, xv [n, num] f32, y [n] f32 (n <= batch_size);
        n_global = rows of the global batch under data parallelism (loss normaliser)."""
        n = int(xi.shape[0])
        if n > self.B:
            raise ValueError(f"batch of {n} rows exceeds the step's {self.B}")
        denom = float(max(n_global if n_global is not None else n, 1))
        full = n == self.B
        use_graph = self.use_graph and full and self.steps >= 1
        direct = self._direct_inputs(xi, xv, y, n) if (use_graph and self.resident_inputs) else None
        if direct is None:
            if n:
                self.xi[:n].copy_(xi.reshape(n, -1))
                if self.num:
                    self.xv[:n].copy_(xv[:, :self.num])
                self.y[:n].copy_(y)
            inputs = (self.xi, self.xv, self.y)
        else:
            inputs = direct
        self.drop = self.drop_train if self.model.training else 0.0  # nn.Dropout is off in eval mode
        if not self._attached:
            raise RuntimeError("FusedTrainStep.step after close()")
        if use_graph:
            # the graphs bake in the engine's activation workspace: a train forward at a larger batch
            # elsewhere (e.g. autograd) re-allocates it, and then the graphs are re-captured; and they bake in
            # the input pointers: one graph set per resident input buffer set
            # (slices of one large resident array get a new key per step: each is a capture, so fit() copies
            # its batches -- resident_inputs is for a fixed ring of input buffers)
            # (deterministic too: the graphs bake in the scatter / split-K form chosen at capture)
            key = (denom, self.drop, self.deterministic, self._ws_generation(),
                   tuple((t.data_ptr(), tuple(t.stride())) for t in inputs))
            hit = self._graph_sets.pop(key, None)
            if hit is None:
                if len(self._graph_sets) >= self.max_graph_sets:
                    self._graph_sets.pop(next(iter(self._graph_sets)))
                self._in = inputs
                hit = (self._capture(denom), inputs)
            self._graph_sets[key] = hit  # most recently used last
            self.graphs = hit[0]
            self._graph_key = key
            g1, g1b, ga, g2, g2b = self.graphs
            g1.replay()
            if g2 is not None:  # else the whole step (backward parts and Adam) is in g1
                self._replay_dp(g1b, ga, g2, g2b)
        else:
            self._in = inputs
            self._part1(n, denom)
            self._exchange(self._part1b if self._bucketed() else (lambda: None), self._apply_sparse)
            self._part2()
        self.steps += 1
        self.eng._dense_key = None  # weights changed behind torch's version counters: re-pack on next use
        self.eng._packed_key = None  # (the tables' serving copy too)
        self.eng.invalidate_derived()  # and the pair list / sparse tower built from the old weights are stale
        return self.loss_sum

    def step_many(self, batches):
        """Consecutive steps over a list of full, resident batches [(xi, xv, y), ...] (a loader's ring of device
        input buffers), captured as ONE graph of len(batches) steps: the same kernels and the same results as
        calling step() on each in turn (the dropout seed and Adam's step count come from the device counter every
        step bumps), without the ~9 us of idle between two graph replays.  One process only;
        otherwise (data parallelism, the first step, a batch that is not full or not readable in
        place, or resident_inputs=False: each new set of input pointers would be a K-step capture) it runs step()
        per batch.  Returns the running loss sum like step()."""
        direct = [self._direct_inputs(xi, xv, y, int(xi.shape[0])) for xi, xv, y in batches] \
            if self.resident_inputs else [None]
        if (not batches or not self.use_graph or self.dist is not None or self.steps < 1
                or any(int(xi.shape[0]) != self.B for xi, _, _ in batches) or any(d is None for d in direct)):
            for xi, xv, y in batches:
                loss = self.step(xi, xv, y)
            return self.loss_sum if not batches else loss
        if not self._attached:
            raise RuntimeError("FusedTrainStep.step_many after close()")
        self.drop = self.drop_train if self.model.training else 0.0
        denom = float(self.B)
        key = ("many", denom, self.drop, self.deterministic, self._ws_generation(),
               tuple((t.data_ptr(), tuple(t.stride())) for d in direct for t in d))
        hit = self._many_sets.pop(key, None)
        if hit is None:
            if len(self._many_sets) >= self.max_many_sets:
                self._many_sets.pop(next(iter(self._many_sets)))
            s = torch.cuda.Stream(self.dev)
            s.wait_stream(torch.cuda.current_stream(self.dev))
            g = torch.cuda.CUDAGraph()
            s1 = torch.cuda.Stream(self.dev)
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    for d in direct:
                        self._in = d
                        self._one_process_step(denom, s, s1)
            torch.cuda.current_stream(self.dev).wait_stream(s)
            hit = ((g, None, None, None, None), direct)
        self._many_sets[key] = hit
        hit[0][0].replay()
        self.steps += len(batches)
        self.eng._dense_key = None
        self.eng._packed_key = None
        self.eng.invalidate_derived()
        return self.loss_sum

    _graph_key = None
    _attached = False


# --------------------------------------------------------------------------------------- pruning
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


class DevicePruner:
    """The reference's magnitude pruning on the device (C ABI dfwfm_prune_*): the reference's own bisection,
    12 rounds resolved per histogram pass over the magnitudes (dfwfm_prune.hip) -- the same thresholds and
    masks as binary_search_threshold, without its up-to-101 host-synchronised passes."""

    def __init__(self, device):
        self.device = device
        self.ws = torch.empty(0, dtype=torch.uint8, device=device)
        self.thr = torch.zeros(1, dtype=torch.float64, device=device)
        self.L = _lib.lib()

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def threshold(self, sources, target):
        """sources: [(tensor, sym_f)]; returns a 1-element float64 device tensor (not synchronised)."""
        arr = (_lib.dfwfm_prune_source * len(sources))()
        total = 0
        for i, (t, sym) in enumerate(sources):
            if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
                raise RuntimeError("dfwfm pruning: sources must be contiguous float32 HIP tensors")
            arr[i] = _lib.dfwfm_prune_source(t.data_ptr(), t.numel(), int(sym), 0)
            total += t.numel()
        need = int(self.L.dfwfm_prune_workspace_bytes(total))
        if self.ws.numel() < need:
            self.ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        thr = torch.empty(1, dtype=torch.float64, device=self.device)
        _lib.check(self.L.dfwfm_prune_threshold(arr, len(sources), float(target), ctypes.c_void_p(thr.data_ptr()),
                                                ctypes.c_void_p(self.ws.data_ptr()), self.ws.numel(), self._stream()),
                   "dfwfm_prune_threshold")
        return thr

    def apply(self, t, thr, sym_f=0):
        _lib.check(self.L.dfwfm_prune_apply(ctypes.c_void_p(t.data_ptr()), t.numel(), int(sym_f),
                                            ctypes.c_void_p(thr.data_ptr()), self._stream()), "dfwfm_prune_apply")
        torch.autograd.graph.increment_version(t)


def prune_step(model, adaptive_sparse, prune_fm, prune_r, prune_deep, emb_r, emb_corr):
    """The reference's in-loop magnitude pruning (:647-673) on the device: the second-order tables share
    one threshold (:652-656), every `*linear*weight` gets its own (:661-664, including
    fwfm_linear.weight), field_cov is masked by its symmetric part (:666-670)."""
    dev = model._device()
    if dev.type == "cpu":
        return _prune_step_host(model, adaptive_sparse, prune_fm, prune_r, prune_deep, emb_r, emb_corr)
    if dev.type != "cuda":
        raise _lib.DfwfmError(f"pruning runs on a HIP device or the CPU, not on {dev}")
    pr = getattr(model, "_pruner", None)
    if pr is None or pr.device != dev:
        pr = model._pruner = DevicePruner(dev)
    with torch.no_grad():
        named = list(model.named_parameters())
        if prune_fm != 0:
            embs = [p.data for n, p in named if "fm_2nd_embeddings" in n]
            thr = pr.threshold([(e, 0) for e in embs], adaptive_sparse * emb_r)
            for e in embs:
                pr.apply(e, thr)
        for name, param in named:
            if "linear" in name and "weight" in name and prune_deep != 0:
                pr.apply(param.data, pr.threshold([(param.data, 0)], adaptive_sparse))
            if name == "field_cov.weight" and prune_r != 0:
                F_ = param.shape[0]
                pr.apply(param.data, pr.threshold([(param.data, F_)], adaptive_sparse * emb_corr), F_)


def _prune_step_host(model, adaptive_sparse, prune_fm, prune_r, prune_deep, emb_r, emb_corr):
    """prune_step for a module on the CPU: the reference's host bisection (:647-673, :807-823) as it stands."""
    with torch.no_grad():
        named = list(model.named_parameters())
        if prune_fm != 0:
            embs = [p.data for n, p in named if "fm_2nd_embeddings" in n]
            flat = torch.cat([e.reshape(-1) for e in embs])
            thr = binary_search_threshold(flat, adaptive_sparse * emb_r, flat.numel())
            for e in embs:
                e[e.abs() < thr] = 0
        for name, param in named:
            if "linear" in name and "weight" in name and prune_deep != 0:
                thr = binary_search_threshold(param.data, adaptive_sparse, param.numel())
                param.data[param.data.abs() < thr] = 0
            if name == "field_cov.weight" and prune_r != 0:
                sym = (param.data + param.data.t()) * 0.5
                thr = binary_search_threshold(sym, adaptive_sparse * emb_corr, param.numel())
                param.data[sym.abs() < thr] = 0


# --------------------------------------------------------------------------------------- fit
def _dist():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist
    return None


def allreduce_grads(model):
    """Sum the gradients over ranks (the loss is already normalised by the global batch): one
    all-reduce of the flat buffer the backward filled when every grad still lives in it."""
    dist = _dist()
    if dist is None:
        return
    params = [p for p in model.parameters() if p.grad is not None]
    flat = getattr(model, "_grad_flat", None)
    if flat is not None and params:
        lo, hi = flat.data_ptr(), flat.data_ptr() + flat.numel() * 4
        if all(lo <= p.grad.data_ptr() < hi for p in params):
            dist.all_reduce(flat)
            return
    grads = [p.grad for p in params]
    buf = torch._utils._flatten_dense_tensors(grads)
    dist.all_reduce(buf)
    for g, r in zip(grads, torch._utils._unflatten_dense_tensors(buf, grads)):
        g.copy_(r)


def make_optimizer(model):
    """Reference :553-561: SGD(momentum) unless adam / rmsp / adag; adam runs on the HIP kernel for a module on
    the device, and is torch.optim.Adam -- the reference's own optimizer -- for a module on the CPU."""
    if model.optimizer_type == "adam":
        if model._device().type == "cpu":
            return torch.optim.Adam(model.parameters(), lr=model.learning_rate, weight_decay=model.weight_decay)
        return Adam(model.parameters(), lr=model.learning_rate, weight_decay=model.weight_decay)
    if model.optimizer_type == "rmsp":
        return torch.optim.RMSprop(model.parameters(), lr=model.learning_rate, weight_decay=model.weight_decay)
    if model.optimizer_type == "adag":
        return torch.optim.Adagrad(model.parameters(), lr=model.learning_rate, weight_decay=model.weight_decay)
    return torch.optim.SGD(model.parameters(), lr=model.learning_rate, momentum=model.momentum,
                           weight_decay=model.weight_decay)


def _param_summary(model, log, nonzero=False):
    tot = e1 = e2 = dnn = 0
    nz_r = 0
    for name, p in model.named_parameters():
        c = int((p != 0).sum().item()) if nonzero else p.numel()
        tot += c
        if "1st_embeddings" in name:
            e1 += c
        if "2nd_embeddings" in name:
            e2 += c
        if "linear_" in name:
            dnn += c
        if name == "field_cov.weight":
            nz_r = int((0.5 * (p.data + p.data.t()) != 0).sum().item())
    return tot, e1, e2, dnn, nz_r


def fit(model, Xi_train, Xv_train, y_train, Xi_valid=None, Xv_valid=None, y_valid=None, early_stopping=False,
        refit=False, save_path=None, prune=0, prune_fm=0, prune_r=0, prune_deep=0, emb_r=1., emb_corr=1.,
        teacher_model=None):
    """Reference DeepFMs.fit (:497-748).  ``model.batch_size`` is the per-rank batch; under
    torch.distributed every global batch of world * batch_size rows is split over the ranks."""
    log = model.logger
    device = model._device()
    if device.type not in ("cuda", "cpu"):
        from ._lib import DfwfmError
        raise DfwfmError(f"fit runs on a HIP device or the CPU, not on {device}")
    dist = _dist()
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
    ncat = model.field_size - model.num
    Xi_train = np.asarray(Xi_train).reshape((-1, ncat, 1))
    Xv_train = np.asarray(Xv_train)
    y_train = np.asarray(y_train)
    x_size = Xi_train.shape[0]
    is_valid = Xi_valid is not None and len(Xi_valid) > 0
    if is_valid:
        Xi_valid = np.asarray(Xi_valid).reshape((-1, ncat, 1))
        Xv_valid = np.asarray(Xv_valid)
        y_valid = np.asarray(y_valid)

    log.info("init_weights")
    model.init_weights()
    if dist:  # every rank starts from rank 0's weights
        for p in model.parameters():
            dist.broadcast(p.data, 0)
    model.train()
    if teacher_model and dist:
        # loss_fn_kd softmaxes over the batch dimension (dim=0, reference :1060-1061): the loss couples
        # every sample of the batch, so a rank's shard cannot form its share of the gradient
        raise NotImplementedError("knowledge distillation under data parallelism: the KD loss is a softmax over "
                                  "the whole batch (model/DeepFMs.py:1060-1061) and does not split over ranks")
    # Adam without distillation (the reference default) runs as a graph-replayed fused step;
    # other optimizers / the KD loss go through autograd + the optimizer
    fused = model.optimizer_type == "adam" and not teacher_model and getattr(model, "fused_fit", True) and \
        device.type == "cuda"  # on the CPU: the host kernels through autograd + torch.optim.Adam
    bs = model.batch_size
    gbs = bs * world
    trainer = FusedTrainStep(model, bs, lr=model.learning_rate, weight_decay=model.weight_decay,
                             dist=dist) if fused else None
    try:
        return _fit_loop(model, trainer, dist, rank, world, Xi_train, Xv_train, y_train, x_size, ncat, is_valid,
                         Xi_valid if is_valid else None, Xv_valid if is_valid else None,
                         y_valid if is_valid else None, early_stopping, save_path, prune, prune_fm, prune_r,
                         prune_deep, emb_r, emb_corr, teacher_model)
    finally:
        if trainer is not None:
            trainer.close()


def _fit_loop(model, trainer, dist, rank, world, Xi_train, Xv_train, y_train, x_size, ncat, is_valid, Xi_valid,
              Xv_valid, y_valid, early_stopping, save_path, prune, prune_fm, prune_r, prune_deep, emb_r, emb_corr,
              teacher_model):
    log = model.logger
    device = model._device()
    fused = trainer is not None
    bs = model.batch_size
    gbs = bs * world
    x_valid_size = Xi_valid.shape[0] if is_valid else 0
    optimizer = None if fused else make_optimizer(model)
    num_total, e1, e2, dnn, nz_r = _param_summary(model, log)
    log.info("========")
    log.info(f"Summation of feature sizes: {sum(model.feature_sizes):,}")
    log.info(f"Number of 1st order embeddings: {e1:,}")
    log.info(f"Number of 2nd order embeddings: {e2:,}")
    if model.use_fwfm:
        log.info(f"Number of 2nd order interactions: {nz_r:,}")
    if model.use_deep:
        log.info(f"Number of DNN parameters: {dnn:,}")
    log.info(f"Number of total parameters: {num_total:,}")
    log.info("========")
    num_total_original = num_total

    # the training set lives in HBM; each epoch's shuffle is a device gather by the reference's
    # numpy permutation (same order as the reference's host-side shuffle)
    Xi_d = torch.as_tensor(Xi_train.reshape(x_size, ncat), dtype=torch.int64).to(device)
    Xv_d = torch.as_tensor(Xv_train, dtype=torch.float32).to(device)
    y_d = torch.as_tensor(y_train, dtype=torch.float32).to(device)
    train_result, valid_result = [], []
    n_iter = 0
    for epoch in range(model.n_epochs):
        total_loss = 0.0
        win_rows = 0  # rows this rank trained on since the last log line (fused: the device loss sum's window)
        if fused:
            trainer.loss_sum.zero_()
        batch_iter = x_size // gbs
        epoch_begin = batch_begin = time()
        teacher_outputs = None
        if teacher_model:
            t0 = time()
            teacher_model.eval()
            teacher_outputs = model.fetch_teacher_outputs(teacher_model, Xi_train, Xv_train, x_size)
            logging.info("- Finished computing teacher outputs after {} secs..".format(math.ceil(time() - t0)))
        for i in range(batch_iter + 1):
            if epoch >= model.warm:
                n_iter += 1
            offset = i * gbs
            end = min(x_size, offset + gbs)
            if offset == end:
                break
            lo = min(end, offset + rank * bs)
            hi = min(end, lo + bs)
            n_global = end - offset
            xi, xv, yb = Xi_d[lo:hi], Xv_d[lo:hi], y_d[lo:hi]
            win_rows += hi - lo
            if fused:
                trainer.step(xi, xv, yb, n_global if dist else None)
                if epoch == 0 and i == 0:
                    model.check_index_errors()  # an out-of-range Xi raises IndexError as nn.Embedding does
            else:
                optimizer.zero_grad()
                if hi > lo:
                    outputs = model(xi, xv)
                    if teacher_model:
                        tb = torch.as_tensor(teacher_outputs[i]).to(device)
                        loss = model.loss_fn_kd(outputs, tb, yb)
                    else:
                        # mean over the global batch: the rank's sum / n_global, summed over ranks below
                        loss = F.binary_cross_entropy_with_logits(outputs, yb, reduction="sum") / n_global \
                            if dist else F.binary_cross_entropy_with_logits(outputs, yb)
                    loss.backward()
                else:
                    loss = torch.zeros((), device=device)
                    for p in model.parameters():
                        p.grad = torch.zeros_like(p)
                allreduce_grads(model)
                optimizer.step()
                if model.verbose:
                    total_loss += loss.item()
            if model.verbose and i % 100 == 99:
                if fused:
                    # the window's summed per-sample BCE -> 100 x its mean (the reference prints total / 100 of
                    # 100 batch means); the device sum restarts every window, so it never grows large in f32
                    total_loss = float(trainer.loss_sum.item()) * 100.0 / max(win_rows, 1)
                    trainer.loss_sum.zero_()
                    model.check_index_errors()  # the stream is synchronised here anyway: surface a bad Xi early
                win_rows = 0
                # (the reference's evaluate() leaves the model in eval mode -- dropout off -- for the
                # rest of training, :627-630, :880-893; kept as is)
                ev = model.evaluate(xi, xv, yb) if hi > lo else float("nan")
                log.info("[%d, %5d] loss: %.6f metric: %.6f time: %.1f s" %
                         (epoch + 1, i + 1, total_loss / 100.0, ev, time() - batch_begin))
                total_loss = 0.0
                batch_begin = time()
            if prune and (i == batch_iter or i % 10 == 9) and epoch >= model.warm:
                model.adaptive_sparse = model.target_sparse * (1 - 0.99 ** (n_iter / 100.))
                prune_step(model, model.adaptive_sparse, prune_fm, prune_r, prune_deep, emb_r, emb_corr)

        model.check_index_errors()  # once per epoch: the sticky flag of every training forward since the last read
        no_non_sparse = sum(int((p != 0).sum().item()) for p in model.parameters())
        log.info("Model parameters %d, sparse rate %.2f%%" % (no_non_sparse, 100 - no_non_sparse * 100. / num_total))
        train_loss, train_eval, train_prauc, train_rce = model.eval_by_batch(Xi_train, Xv_train, y_train, x_size)
        train_result.append(train_eval)
        log.info("Training [%d] loss: %.6f metric: %.6f prauc: %.4f rce: %.2f sparse %.2f%% time: %.1f s" %
                 (epoch + 1, train_loss, train_eval, train_prauc, train_rce,
                  100 - no_non_sparse * 100. / num_total, time() - epoch_begin))
        if is_valid:
            valid_loss, valid_eval, valid_prauc, valid_rce = model.eval_by_batch(Xi_valid, Xv_valid, y_valid,
                                                                                 x_valid_size)
            valid_result.append(valid_eval)
            log.info("Validation [%d] loss: %.6f metric: %.6f prauc: %.4f rce: %.2f sparse %.2f%% time: %.1f s" %
                     (epoch + 1, valid_loss, valid_eval, valid_prauc, valid_rce,
                      100 - no_non_sparse * 100. / num_total, time() - epoch_begin))
        log.info("*" * 50)
        # no model.train() here: the reference's eval_by_batch leaves the model in eval mode, so from the
        # second epoch on it trains without dropout (model/DeepFMs.py:694-714, :766); kept for parity
        perm = np.random.permutation(x_size)
        Xi_train, Xv_train, y_train = Xi_train[perm], Xv_train[perm], y_train[perm]
        pd = torch.as_tensor(perm).to(device)
        Xi_d, Xv_d, y_d = Xi_d[pd], Xv_d[pd], y_d[pd]
        if save_path and rank == 0:
            torch.save(model.state_dict(), save_path)
        if is_valid and early_stopping and model.training_termination(valid_result):
            log.info("early stop at [%d] epoch!" % (epoch + 1))
            break

    if prune:
        tot, e1, e2, dnn, nz_r = _param_summary(model, log, nonzero=True)
        log.info("========")
        log.info(f"Number of pruned 1st order embeddings: {e1:,}")
        log.info(f"Number of pruned 2nd order embeddings: {e2:,}")
        log.info(f"Number of pruned 2nd order interactions: {nz_r:,}")
        log.info(f"Number of pruned DNN parameters: {dnn:,}")
        log.info(f"Number of pruned total parameters: {tot:,}")
        log.info(f"Non pruned model parameters: \t{num_total_original:,}")
        log.info(f"Pruned Parameters: \t{num_total_original - tot:,}")
        log.info("========")
    return train_result, valid_result
