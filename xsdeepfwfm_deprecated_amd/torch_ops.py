"""The forward as a PyTorch custom operator: ``torch.ops.dfwfm.forward``.

Registered with ``torch.library`` (schema, fake/meta kernel, autograd formula), so the dispatcher sees
one op per DeepFMs forward (reference ``model/DeepFMs.py:285-469``) whose backward is the HIP backward
(``csrc/dfwfm_train.hip``) -- the surface BASELINE.json's north star asks for ("PyTorch-ROCm custom
ops so main_all.py's fit()/predict() API is unchanged").  ``DeepFMs.forward`` calls it.

    logits, token = torch.ops.dfwfm.forward(model_id, xi, xv, params, train, dropout_p, seed)

* ``model_id``: handle of a registered DeepFMs (``register(model)``); its ForwardEngine holds the
  device-side table descriptors and packed dense weights (synced by the module before the call).
* ``xi`` int64 [B, F-num], ``xv`` float32 [B, >= num] (row strides free), on the module's device.
* ``params``: the module's trainable parameters in ``parameters()`` order -- inputs of the op, so
  autograd routes the HIP backward's gradients to them.
* ``train``: keep the activations for the backward (and apply deep-tower dropout ``dropout_p`` with
  counter-hash ``seed``); ``token`` (int64 CPU scalar) names that saved state for the backward.

Kernels: HIP (libdfwfm.so) for tensors on the device, the host kernel (libdfwfm_cpu.so) for tensors on the CPU;
neither stands in for the other, and a missing library raises.
"""
import itertools
import weakref
from typing import List, Tuple

import torch

_models: "weakref.WeakValueDictionary[int, torch.nn.Module]" = weakref.WeakValueDictionary()
_ids = itertools.count(1)


def register(model) -> int:
    """Give a DeepFMs module an id the op can find it by (kept as a weak reference)."""
    mid = getattr(model, "_op_id", None)
    if mid is None or _models.get(mid) is not model:
        mid = next(_ids)
        _models[mid] = model
        model._op_id = mid
    return mid


def _model(mid: int):
    m = _models.get(int(mid))
    if m is None:
        raise RuntimeError(f"dfwfm::forward: no registered DeepFMs with id {mid}")
    return m


def _run(model_id, xi, xv, train, dropout_p, seed, engine_type):
    m = _model(model_id)
    eng = m._engine
    if eng is None or not isinstance(eng, engine_type) or eng.device != xi.device:
        raise RuntimeError("dfwfm::forward: the module's engine is not synced to this device")
    out = torch.empty(xi.shape[0], dtype=torch.float32, device=xi.device)
    token = 0
    if train:
        token = eng.train_forward(xi, xv, out, dropout_p, seed)
    else:
        eng.forward(xi, xv, out)
    return out, torch.tensor(token, dtype=torch.int64)


@torch.library.custom_op("dfwfm::forward", mutates_args=(), device_types="cuda")
def forward(model_id: int, xi: torch.Tensor, xv: torch.Tensor, params: List[torch.Tensor], train: bool,
            dropout_p: float, seed: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """HIP kernel (libdfwfm.so, include/dfwfm.h)."""
    from .engine import ForwardEngine
    return _run(model_id, xi, xv, train, dropout_p, seed, ForwardEngine)


@forward.register_kernel("cpu")
def _forward_cpu(model_id, xi, xv, params, train, dropout_p, seed):
    """CPU kernel (libdfwfm_cpu.so, include/dfwfm_cpu.h): a module on the CPU, the reference's -use_cuda 0 /
    -time_on_cuda 0 paths; selected by the tensors' device, never as a stand-in for the HIP kernel."""
    from .engine import CpuEngine
    return _run(model_id, xi, xv, train, dropout_p, seed, CpuEngine)


@forward.register_fake
def _(model_id, xi, xv, params, train, dropout_p, seed):
    return xi.new_empty(xi.shape[0], dtype=torch.float32), torch.empty((), dtype=torch.int64, device="cpu")


def _setup_context(ctx, inputs, output):
    model_id, xi, xv, params, train, dropout_p, seed = inputs
    ctx.model_id = model_id
    ctx.train = train
    ctx.token = int(output[1]) if train else None
    ctx.n_params = len(params)
    ctx.param_ids = [id(p) for p in params]
    # the backward kernels re-read the indices (and values) through the pointers the train forward
    # recorded: keep the tensors alive until then, or the caching allocator hands their memory out
    ctx.save_for_backward(xi, xv)


def _backward(ctx, grad_out, grad_token):
    if not ctx.train:
        raise RuntimeError("dfwfm::forward: backward of an inference forward (call with train=True)")
    from .training import _grad_buffer
    m = _model(ctx.model_id)
    eng = m._engine
    params = [p for p in m.parameters() if p.requires_grad]
    if [id(p) for p in params] != ctx.param_ids:
        raise RuntimeError("dfwfm::forward: the module's parameters changed between forward and backward")
    need = [True] * len(params)
    flat, views = _grad_buffer(params, need, eng.device)
    by_id = {id(p): g for p, g in zip(params, views)}
    fields, dense = m._param_layout()
    fg = [tuple(None if t is None else by_id.get(id(t)) for t in tup) for tup in fields]
    dg = {k: (None if v is None else by_id.get(id(v))) for k, v in dense.items() if not isinstance(v, list)}
    dg["lin_w"] = [by_id.get(id(t)) for t in dense["lin_w"]]
    dg["lin_b"] = [by_id.get(id(t)) for t in dense["lin_b"]]
    xi, xv = ctx.saved_tensors  # alive (see _setup_context) until the backward is enqueued
    eng.set_deterministic(getattr(m, "deterministic", True))
    eng.backward(ctx.token, grad_out.contiguous(), fg, dg)
    m._grad_flat = flat
    del xi, xv
    return None, None, None, list(views), None, None, None


forward.register_autograd(_backward, setup_context=_setup_context)
