"""Host-side driver of the HIP forward: owns a ``dfwfm_model`` handle and keeps
it in sync with a DeepFMs module's parameters.

* Embedding tables are passed to the kernel by pointer (no copy): a re-upload
  of the 39 field descriptors happens only when a table is re-allocated
  (``.cuda()``, ``load_state_dict`` into new storage, ...).
* Dense parameters (R, fwlw, lw, bias, MLP) are re-packed into the kernel's
  fragment layout on the current stream whenever any of them changes
  (tracked with the tensors' in-place version counters), e.g. after every
  optimizer step -- never per forward otherwise.
* Training: ``train_forward`` keeps the activations in engine-owned device
  memory and ``backward`` consumes them; every train forward gets a token and a
  backward for a stale token raises (one forward/backward pair at a time).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream_handle(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_f32_cuda(t, name, device):
    if t.dtype != torch.float32 or not t.is_cuda or t.device != device:
        raise RuntimeError(f"dfwfm: {name} must be a float32 tensor on {device}, got {t.dtype} on {t.device}")
    if not t.is_contiguous():
        raise RuntimeError(f"dfwfm: {name} must be contiguous")


def _require_rows(t, name, dtype, device, width):
    """The C ABI takes a batch as a base pointer + a row stride: each row's `width` entries must be contiguous
    (a column-major array, e.g. np.asarray of a pandas DataFrame, would be read as the wrong entries)."""
    if t.dtype != dtype or t.device != device:
        raise ValueError(f"dfwfm: {name} must be a {dtype} tensor on {device}, got {t.dtype} on {t.device}")
    if t.dim() < 1 or t.shape[0] == 0 or width == 0:
        return
    inner = 1
    for d in range(t.dim() - 1, 0, -1):  # dims after the batch dim: row-major and dense
        if t.shape[d] != 1 and t.stride(d) != inner:
            raise ValueError(f"dfwfm: {name} rows must be contiguous (got strides {tuple(t.stride())}); "
                             "pass .contiguous()")
        inner *= t.shape[d]
    if inner < width:
        raise ValueError(f"dfwfm: {name} has {inner} entries per row, the model needs {width}")


class ForwardEngine:
    """Binds one DeepFMs module to one device-resident dfwfm_model."""

    def __init__(self, cfg: dict, device: torch.device):
        self.device = device
        self.cfg = dict(cfg)
        c = _lib.dfwfm_config(**{k: int(v) for k, v in cfg.items()})
        h = ctypes.c_void_p()
        L = _lib.lib()
        with torch.cuda.device(device):
            _lib.check(L.dfwfm_model_create(ctypes.byref(c), ctypes.byref(h)), "dfwfm_model_create")
        self.handle = h
        self._tables_key = None
        self._dense_key = None
        self._keep = None  # host-side descriptor array kept alive

    def close(self):
        if self.handle is not None and self.handle.value:
            _lib.lib().dfwfm_model_destroy(self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- parameter sync ----------------------------------------------------
    def sync_tables(self, fields):
        """fields: list of dicts(emb2, emb2_r, emb1, emb1_r, n, c, op) of tensors/ints."""
        names = ("emb2", "emb2_r", "emb1", "emb1_r")
        key = tuple(tuple(None if f[nm] is None else f[nm].data_ptr() for nm in names) for f in fields)
        if key == self._tables_key:
            return
        arr = (_lib.dfwfm_field_tables * len(fields))()
        for i, f in enumerate(fields):
            for nm in ("emb2", "emb2_r", "emb1", "emb1_r"):
                if f[nm] is not None:
                    _require_f32_cuda(f[nm], f"field {i} {nm}", self.device)
            arr[i] = _lib.dfwfm_field_tables(
                *[None if f[nm] is None else f[nm].data_ptr() for nm in names],
                int(f["n"]), int(f["c"]), int(f["op"]), 0)
        _lib.check(_lib.lib().dfwfm_model_set_tables(self.handle, arr, len(fields),
                                                     _stream_handle(self.device)), "dfwfm_model_set_tables")
        self._packed_key = None  # set_tables drops the serving copy
        self._keep = arr
        self._tables_key = key

    def sync_dense(self, field_cov, fwfm_lin, fm_1st, bias, lin_w, lin_b, fc_w):
        tensors = [field_cov, fwfm_lin, fm_1st, bias, fc_w] + list(lin_w) + list(lin_b)
        key = tuple(None if t is None else (t.data_ptr(), t._version) for t in tensors)
        if key == self._dense_key:
            return
        for i, t in enumerate(tensors):
            if t is not None:
                _require_f32_cuda(t, f"dense parameter {i}", self.device)
        H = len(lin_w)
        W = (ctypes.c_void_p * max(H, 1))(*[t.data_ptr() for t in lin_w])
        B = (ctypes.c_void_p * max(H, 1))(*[t.data_ptr() for t in lin_b])
        self.__dict__.pop("_ws_cache", None)  # set_dense turns the sparse tower off until sync_sparse
        self.invalidate_derived()
        _lib.check(_lib.lib().dfwfm_model_set_dense(
            self.handle, _ptr(field_cov), _ptr(fwfm_lin), _ptr(fm_1st), _ptr(bias),
            W if H else None, B if H else None, _ptr(fc_w), _stream_handle(self.device)),
            "dfwfm_model_set_dense")
        self._dense_key = key

    def invalidate_derived(self):
        """Forget the pruned FwFM pair list and the sparse deep tower: dfwfm_model_set_dense turns both off in
        the library (and a captured training step re-packs the weights they were built from), so the next
        sync_pairs / sync_sparse must rebuild them rather than report the cached state."""
        self._pairs_key = None
        self._sparse_key = None

    def sync_packed(self, tables, enable: bool = True) -> bool:
        """dfwfm_model_pack_tables: the serving copy of the categorical tables (second-order row + first-order
        weight in one aligned row) for the forward without a deep tower, rebuilt whenever a table tensor moved or
        changed (torch's version counters; the fused training step resets the key, its updates bypass them).
        tables: the categorical fields' (emb2, emb1) tensors.  Returns whether the copy is in use."""
        key = (bool(enable),) + tuple((t.data_ptr(), t._version) for pair in tables for t in pair if t is not None)
        if key == getattr(self, "_packed_key", None):
            return self._packed_on
        en = ctypes.c_int32(0)
        _lib.check(_lib.lib().dfwfm_model_pack_tables(self.handle, int(bool(enable)), ctypes.byref(en),
                                                      _stream_handle(self.device)), "dfwfm_model_pack_tables")
        self._packed_on = bool(en.value)
        self._packed_key = key
        return self._packed_on

    def sync_pairs(self, max_pairs: int) -> bool:
        """(Re)build the pruned FwFM's nonzero pair list after a weight update (syncs the stream once per
        update): the forward without a deep tower then sums the listed pairs when there are at most
        max_pairs.  Returns whether the pair path is on."""
        key = (self._dense_key, int(max_pairs))
        if key == getattr(self, "_pairs_key", None):
            return self._pairs_on
        en = ctypes.c_int32(0)
        _lib.check(_lib.lib().dfwfm_model_build_fwfm_pairs(self.handle, int(max_pairs), ctypes.byref(en),
                                                           _stream_handle(self.device)),
                   "dfwfm_model_build_fwfm_pairs")
        self._pairs_on = bool(en.value)
        self._pairs_key = key
        return self._pairs_on

    def sync_sparse(self, max_density: float) -> bool:
        """(Re)build the pruned deep tower's nonzero lists after a weight update (inference only; syncs
        the stream once per update): dfwfm_forward_ws then runs the sparse MLP when the hidden layers'
        nonzero fraction is <= max_density.  Returns whether the sparse path is on."""
        key = (self._dense_key, float(max_density))
        if key == getattr(self, "_sparse_key", None):
            return self._sparse_on
        en = ctypes.c_int32(0)
        _lib.check(_lib.lib().dfwfm_model_build_sparse_mlp(self.handle, float(max_density), ctypes.byref(en),
                                                           _stream_handle(self.device)),
                   "dfwfm_model_build_sparse_mlp")
        self._sparse_on = bool(en.value)
        self._sparse_key = key
        self.__dict__.pop("_ws_cache", None)  # the workspace a batch needs changes with the path
        return self._sparse_on

    # -- hot path ----------------------------------------------------------
    def forward(self, xi: torch.Tensor, xv: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        B = xi.shape[0]
        ncat = self.cfg["field_size"] - self.cfg["numerical"]
        num = self.cfg["numerical"]
        _require_rows(xi, "Xi", torch.int64, self.device, ncat)
        _require_rows(xv, "Xv", torch.float32, self.device, num)
        if out is None:
            out = torch.empty(B, dtype=torch.float32, device=self.device)
        xs = xi.stride(0) if ncat > 0 else 0
        vs = xv.stride(0) if num > 0 else 0
        ws_bytes = self._ws_bytes(B)
        # split forward (gather launch + MLP launch): its workspace comes from torch's stream-ordered
        # caching allocator, so batches in flight on several streams never share one
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=self.device) if ws_bytes else None
        rc = _lib.lib().dfwfm_forward_ws(self.handle, ctypes.c_void_p(xi.data_ptr()), xs,
                                         ctypes.c_void_p(xv.data_ptr()), vs, B,
                                         ctypes.c_void_p(out.data_ptr()), _ptr(ws), ws_bytes,
                                         _stream_handle(self.device))
        _lib.check(rc, "dfwfm_forward")
        return out

    def forward_batches(self, batches, outs) -> list:
        """dfwfm_forward_batches: the forward of every (xi, xv) in `batches` (same batch size and row strides),
        all in one launch per 32 batches; logits into outs[i], bit-identical to forward() on each batch alone."""
        nb = len(batches)
        if nb == 0:
            return outs
        if len(outs) != nb:
            raise ValueError("forward_batches: one output per batch")
        ncat = self.cfg["field_size"] - self.cfg["numerical"]
        num = self.cfg["numerical"]
        xi0, xv0 = batches[0]
        B = xi0.shape[0]
        xs = xi0.stride(0) if ncat > 0 else 0
        vs = xv0.stride(0) if num > 0 else 0
        for xi, xv in batches:
            _require_rows(xi, "Xi", torch.int64, self.device, ncat)
            _require_rows(xv, "Xv", torch.float32, self.device, num)
            if xi.shape[0] != B or (ncat > 0 and xi.stride(0) != xs) or (num > 0 and xv.stride(0) != vs):
                raise ValueError("forward_batches: every batch needs the same size and row strides")
        for o in outs:
            if o.numel() < B:
                raise ValueError("forward_batches: output smaller than the batch")
        P = ctypes.c_void_p * nb
        pxi = P(*[xi.data_ptr() for xi, _ in batches])
        pxv = P(*[xv.data_ptr() for _, xv in batches])
        pout = P(*[o.data_ptr() for o in outs])
        rc = _lib.lib().dfwfm_forward_batches(self.handle, nb, pxi, xs, pxv, vs, B, pout, _stream_handle(self.device))
        _lib.check(rc, "dfwfm_forward_batches")
        return outs

    def forward_gather(self, xi: torch.Tensor, xv: torch.Tensor, deep_emb: torch.Tensor | None = None,
                       first_second: torch.Tensor | None = None):
        """dfwfm_forward_gather: the gather / shallow half of a deep model's forward alone -- deep_emb
        [B, ceil(F D / 16) 16] (zero padded) and first + second order [B]."""
        B = xi.shape[0]
        ncat = self.cfg["field_size"] - self.cfg["numerical"]
        num = self.cfg["numerical"]
        _require_rows(xi, "Xi", torch.int64, self.device, ncat)
        _require_rows(xv, "Xv", torch.float32, self.device, num)
        W = -(-self.cfg["field_size"] * self.cfg["embedding_size"] // 16) * 16
        if deep_emb is None:
            deep_emb = torch.empty(B, W, dtype=torch.float32, device=self.device)
        if first_second is None:
            first_second = torch.empty(B, dtype=torch.float32, device=self.device)
        rc = _lib.lib().dfwfm_forward_gather(self.handle, ctypes.c_void_p(xi.data_ptr()),
                                             xi.stride(0) if ncat > 0 else 0, ctypes.c_void_p(xv.data_ptr()),
                                             xv.stride(0) if num > 0 else 0, B, ctypes.c_void_p(deep_emb.data_ptr()),
                                             deep_emb.stride(0), ctypes.c_void_p(first_second.data_ptr()),
                                             _stream_handle(self.device))
        _lib.check(rc, "dfwfm_forward_gather")
        return deep_emb, first_second

    def _ws_bytes(self, B: int) -> int:
        cache = self.__dict__.setdefault("_ws_cache", {})
        if B not in cache:
            n = ctypes.c_size_t(0)
            _lib.check(_lib.lib().dfwfm_forward_workspace_bytes(self.handle, B, ctypes.byref(n)),
                       "dfwfm_forward_workspace_bytes")
            cache[B] = int(n.value)
        return cache[B]

    # -- training step -------------------------------------------------------
    def train_forward(self, xi, xv, out, dropout_p: float, seed: int) -> int:
        """Forward of a training step; returns the token the matching backward must present."""
        B = xi.shape[0]
        ncat = self.cfg["field_size"] - self.cfg["numerical"]
        _require_rows(xi, "Xi", torch.int64, self.device, ncat)
        _require_rows(xv, "Xv", torch.float32, self.device, self.cfg["numerical"])
        xs = xi.stride(0) if ncat > 0 else 0
        vs = xv.stride(0) if self.cfg["numerical"] > 0 else 0
        rc = _lib.lib().dfwfm_train_forward(self.handle, ctypes.c_void_p(xi.data_ptr()), xs,
                                            ctypes.c_void_p(xv.data_ptr()), vs, B, ctypes.c_void_p(out.data_ptr()),
                                            float(dropout_p), int(seed) & 0xFFFFFFFF, _stream_handle(self.device))
        _lib.check(rc, "dfwfm_train_forward")
        self._token = getattr(self, "_token", 0) + 1
        return self._token

    def set_deterministic(self, on: bool) -> None:
        """dfwfm_set_deterministic: fixed-order gradient sums (table scatter, split-K) for the backwards after it."""
        on = bool(on)
        if getattr(self, "_deterministic", None) != on:
            _lib.check(_lib.lib().dfwfm_set_deterministic(self.handle, int(on)), "dfwfm_set_deterministic")
            self._deterministic = on

    def backward(self, token: int, dlogit, field_grads, dense):
        """field_grads: per field (emb2, emb2_r, emb1, emb1_r) grad tensors or None; dense: dict of
        field_cov, fwfm_lin, fm_1st, bias, fc_w (tensor or None), lin_w / lin_b (lists)."""
        if token != getattr(self, "_token", None):
            raise RuntimeError("dfwfm: backward of a stale training forward (another train forward ran in "
                               "between; one forward/backward pair at a time)")
        fg = (_lib.dfwfm_field_grads * len(field_grads))()
        for i, tup in enumerate(field_grads):
            fg[i] = _lib.dfwfm_field_grads(*[None if t is None else t.data_ptr() for t in tup])
        lw, lb = dense.get("lin_w") or [], dense.get("lin_b") or []
        W = (ctypes.c_void_p * max(len(lw), 1))(*[None if t is None else t.data_ptr() for t in lw])
        Bv = (ctypes.c_void_p * max(len(lb), 1))(*[None if t is None else t.data_ptr() for t in lb])
        g = _lib.dfwfm_grads(fg, *[None if dense.get(k) is None else dense[k].data_ptr()
                                   for k in ("field_cov", "fwfm_lin", "fm_1st", "bias")],
                             W if lw else None, Bv if lb else None,
                             None if dense.get("fc_w") is None else dense["fc_w"].data_ptr())
        _lib.check(_lib.lib().dfwfm_backward(self.handle, ctypes.c_void_p(dlogit.data_ptr()), ctypes.byref(g),
                                             _stream_handle(self.device)), "dfwfm_backward")

    def read_error_flag(self) -> int:
        v = ctypes.c_int32(0)
        _lib.check(_lib.lib().dfwfm_read_error_flag(self.handle, ctypes.byref(v), _stream_handle(self.device)),
                   "dfwfm_read_error_flag")
        return int(v.value)


def adam_step(entries, lr, beta1, beta2, eps, weight_decay, step, device):
    """One torch.optim.Adam step over [(param, grad, exp_avg, exp_avg_sq)] (float32, contiguous, on
    `device`) on the current stream; no model handle needed."""
    arr = (_lib.dfwfm_adam_tensor * max(len(entries), 1))()
    for i, (p, g, m, v) in enumerate(entries):
        arr[i] = _lib.dfwfm_adam_tensor(p.data_ptr(), None if g is None else g.data_ptr(), m.data_ptr(),
                                        v.data_ptr(), p.numel())
    _lib.check(_lib.lib().dfwfm_adam_step(arr, len(entries), float(lr), float(beta1), float(beta2), float(eps),
                                          float(weight_decay), int(step), _stream_handle(device)),
               "dfwfm_adam_step")


class CpuEngine:
    """The host counterpart of ForwardEngine for a DeepFMs module on the CPU (include/dfwfm_cpu.h,
    libdfwfm_cpu.so): the CPU kernel of torch.ops.dfwfm.forward and its backward -- the reference's
    -use_cuda 0 / -time_on_cuda 0 paths (main_all.py:42-63).  Parameters are read in place through their
    host pointers (re-described on every sync: no copies).  Threads: torch.get_num_threads(), the knob the
    reference's benchmark turns (model/DeepFMs.py:983, 1000)."""

    device = torch.device("cpu")

    def __init__(self, cfg: dict):
        self.cfg = dict(cfg)
        self.c = _lib.dfwfm_config(**{k: int(v) for k, v in cfg.items()})
        self.flags = 0
        self._token = 0
        self._saved = None
        self._keep = None
        _lib.cpu_lib()  # must load: no fallback to torch ops

    def close(self):
        self._saved = None

    def sync(self, fields, field_cov, fwfm_lin, fm_1st, bias, lin_w, lin_b, fc_w):
        """fields: list of dicts(emb2, emb2_r, emb1, emb1_r, n, c, op) of CPU tensors / ints; dense tensors."""
        names = ("emb2", "emb2_r", "emb1", "emb1_r")
        arr = (_lib.dfwfm_field_tables * len(fields))()
        tensors = []
        for i, f in enumerate(fields):
            for nm in names:
                if f[nm] is not None:
                    _require_f32_cpu(f[nm], f"field {i} {nm}")
                    tensors.append(f[nm])
            arr[i] = _lib.dfwfm_field_tables(*[None if f[nm] is None else f[nm].data_ptr() for nm in names],
                                             int(f["n"]), int(f["c"]), int(f["op"]), 0)
        dense = [field_cov, fwfm_lin, fm_1st, bias, fc_w] + list(lin_w) + list(lin_b)
        for i, t in enumerate(dense):
            if t is not None:
                _require_f32_cpu(t, f"dense parameter {i}")
        H = len(lin_w)
        W = (ctypes.c_void_p * max(H, 1))(*[t.data_ptr() for t in lin_w])
        Bv = (ctypes.c_void_p * max(H, 1))(*[t.data_ptr() for t in lin_b])
        self.model = _lib.dfwfm_cpu_model(self.c, arr, *[None if t is None else t.data_ptr() for t in
                                                         (field_cov, fwfm_lin, fm_1st, bias)],
                                          W if H else None, Bv if H else None, None if fc_w is None else fc_w.data_ptr())
        self._keep = (arr, W, Bv, tensors, dense)

    def _inputs(self, xi, xv):
        ncat = self.cfg["field_size"] - self.cfg["numerical"]
        xs = xi.stride(0) if ncat > 0 else 0
        vs = xv.stride(0) if self.cfg["numerical"] > 0 else 0
        return ctypes.c_void_p(xi.data_ptr()), xs, ctypes.c_void_p(xv.data_ptr()), vs

    def forward(self, xi, xv, out=None):
        B = xi.shape[0]
        if out is None:
            out = torch.empty(B, dtype=torch.float32)
        p, xs, v, vs = self._inputs(xi, xv)
        flag = ctypes.c_int32(0)
        _lib.check_cpu(_lib.cpu_lib().dfwfm_cpu_forward(ctypes.byref(self.model), p, xs, v, vs, B,
                                                        ctypes.c_void_p(out.data_ptr()), None, 0.0, 0,
                                                        ctypes.byref(flag), torch.get_num_threads()),
                       "dfwfm_cpu_forward")
        self.flags |= flag.value
        return out

    def train_forward(self, xi, xv, out, dropout_p: float, seed: int) -> int:
        B = xi.shape[0]
        per = int(_lib.cpu_lib().dfwfm_cpu_saved_floats(ctypes.byref(self.c)))
        self._saved = torch.empty(max(B * per, 1), dtype=torch.float32)
        p, xs, v, vs = self._inputs(xi, xv)
        flag = ctypes.c_int32(0)
        _lib.check_cpu(_lib.cpu_lib().dfwfm_cpu_forward(ctypes.byref(self.model), p, xs, v, vs, B,
                                                        ctypes.c_void_p(out.data_ptr()),
                                                        ctypes.c_void_p(self._saved.data_ptr()), float(dropout_p),
                                                        int(seed) & 0xFFFFFFFF, ctypes.byref(flag),
                                                        torch.get_num_threads()), "dfwfm_cpu_forward (train)")
        self.flags |= flag.value
        self._token += 1
        self._train = (xi, xv, B, float(dropout_p), int(seed) & 0xFFFFFFFF)
        return self._token

    def set_deterministic(self, on: bool) -> None:
        """The host backward's sums are in a fixed order already (per-thread partials added in thread order)."""

    def backward(self, token, dlogit, field_grads, dense):
        if token != self._token or self._saved is None:
            raise RuntimeError("dfwfm: backward of a stale training forward (another train forward ran in "
                               "between; one forward/backward pair at a time)")
        xi, xv, B, p_drop, seed = self._train
        fg = (_lib.dfwfm_field_grads * len(field_grads))()
        for i, tup in enumerate(field_grads):
            fg[i] = _lib.dfwfm_field_grads(*[None if t is None else t.data_ptr() for t in tup])
        lw, lb = dense.get("lin_w") or [], dense.get("lin_b") or []
        W = (ctypes.c_void_p * max(len(lw), 1))(*[None if t is None else t.data_ptr() for t in lw])
        Bv = (ctypes.c_void_p * max(len(lb), 1))(*[None if t is None else t.data_ptr() for t in lb])
        g = _lib.dfwfm_grads(fg, *[None if dense.get(k) is None else dense[k].data_ptr()
                                   for k in ("field_cov", "fwfm_lin", "fm_1st", "bias")],
                             W if lw else None, Bv if lb else None,
                             None if dense.get("fc_w") is None else dense["fc_w"].data_ptr())
        p, xs, v, vs = self._inputs(xi, xv)
        dl = dlogit.contiguous()
        _lib.check_cpu(_lib.cpu_lib().dfwfm_cpu_backward(ctypes.byref(self.model), p, xs, v, vs, B,
                                                         ctypes.c_void_p(dl.data_ptr()),
                                                         ctypes.c_void_p(self._saved.data_ptr()), p_drop, seed,
                                                         ctypes.byref(g), torch.get_num_threads()),
                       "dfwfm_cpu_backward")
        self._saved = None

    def read_error_flag(self) -> int:
        v, self.flags = self.flags, 0
        return v


def _require_f32_cpu(t, name):
    if t.dtype != torch.float32 or t.device.type != "cpu":
        raise RuntimeError(f"dfwfm (CPU): {name} must be a float32 CPU tensor, got {t.dtype} on {t.device}")
    if not t.is_contiguous():
        raise RuntimeError(f"dfwfm (CPU): {name} must be contiguous")
