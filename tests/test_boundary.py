"""CPU: the C-ABI library loads and exports every symbol include/dfwfm.h declares; the DeepFMs
mirror keeps the reference's state-dict contract; no compute without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO, golden_names, load_golden, model_kwargs


@pytest.fixture(scope="module")
def built():
    from xsdeepfwfm_deprecated_amd import _lib
    _lib.build()
    return _lib


def header_functions():
    src = open(os.path.join(REPO, "include", "dfwfm.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dfwfm_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_api():
    assert header_functions() == sorted([
        "dfwfm_abi_version", "dfwfm_adam_step", "dfwfm_adam_step_dev", "dfwfm_backward", "dfwfm_backward_phases",
        "dfwfm_bce_grad", "dfwfm_backward_phases_bce", "dfwfm_model_set_dense_zero",
        "dfwfm_diag_stamps", "dfwfm_eval_metrics", "dfwfm_forward", "dfwfm_forward_batches",
        "dfwfm_forward_workspace_bytes", "dfwfm_forward_gather",
        "dfwfm_forward_ws", "dfwfm_last_error", "dfwfm_model_build_fwfm_pairs", "dfwfm_model_build_sparse_mlp", "dfwfm_model_create", "dfwfm_model_destroy", "dfwfm_model_pack_tables",
        "dfwfm_metrics_workspace_bytes", "dfwfm_model_set_dense", "dfwfm_model_set_tables", "dfwfm_prune_apply", "dfwfm_prune_threshold",
        "dfwfm_prune_workspace_bytes", "dfwfm_read_error_flag", "dfwfm_set_deterministic", "dfwfm_set_step_source", "dfwfm_sparse_grads_apply", "dfwfm_sparse_grads_local", "dfwfm_sparse_grads_size",
        "dfwfm_train_forward", "dfwfm_workspace_generation"])


def test_library_exports_every_header_symbol(built):
    L = ctypes.CDLL(built.LIB_PATH)
    for name in header_functions():
        assert hasattr(L, name), name
    assert set(built.SIGNATURES) == set(header_functions())


def test_abi_version_and_error_string(built):
    L = built.lib()
    assert L.dfwfm_abi_version() == 4
    assert isinstance(L.dfwfm_last_error(), bytes)
    # invalid arguments are reported, never abort (no HIP call is reached)
    assert L.dfwfm_model_create(None, None) == -1
    assert b"null" in L.dfwfm_last_error()
    assert L.dfwfm_forward(None, None, 0, None, 0, 0, None, None) == -1
    assert L.dfwfm_forward_batches(None, 2, None, 0, None, 0, 0, None, None) == -1
    assert L.dfwfm_train_forward(None, None, 0, None, 0, 0, None, 0.0, 0, None) == -1
    assert L.dfwfm_backward(None, None, None, None) == -1
    assert L.dfwfm_adam_step(None, 3, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1, None) == -1
    assert L.dfwfm_adam_step(None, 0, 1e-3, 0.9, 0.999, 1e-8, 0.0, 0, None) == -1  # step >= 1
    assert L.dfwfm_adam_step_dev(None, 0, 1e-3, 0.9, 0.999, 1e-8, 0.0, None, None) == -1
    assert L.dfwfm_bce_grad(None, None, 4, 4.0, None, None, None) == -1
    assert L.dfwfm_bce_grad(None, None, 0, 0.0, None, None, None) == -1  # denom > 0
    assert L.dfwfm_set_step_source(None, None) == -1
    assert L.dfwfm_prune_threshold(None, 0, 0.5, None, None, 0, None) == -1
    assert L.dfwfm_prune_apply(None, 4, 0, None, None) == -1
    assert L.dfwfm_prune_workspace_bytes(1000) >= 8000  # host-only query (histogram-select sizing, no launch)
    assert ctypes.sizeof(built.dfwfm_prune_source) == 24
    assert L.dfwfm_eval_metrics(None, None, 4, None, None, 0, None) == -1
    assert L.dfwfm_metrics_workspace_bytes(1000) >= 32 * 1000  # keys, labels (x2), ranks above, group starts


def test_struct_layouts_match_header(built):
    assert ctypes.sizeof(built.dfwfm_config) == 11 * 4
    assert ctypes.sizeof(built.dfwfm_field_tables) == 4 * 8 + 2 * 8 + 2 * 4
    assert ctypes.sizeof(built.dfwfm_field_grads) == 4 * 8
    assert ctypes.sizeof(built.dfwfm_grads) == 8 * 8
    assert ctypes.sizeof(built.dfwfm_adam_tensor) == 5 * 8


@pytest.mark.parametrize("name", golden_names())
def test_state_dict_contract_matches_reference(name):
    """Parameter names and shapes equal the reference model's (recorded by gen_golden.py)."""
    from xsdeepfwfm_deprecated_amd import DeepFMs
    cfg, params, *_ = load_golden(name)
    m = DeepFMs(**model_kwargs(cfg))
    sd = m.state_dict()
    assert {k: list(v.shape) for k, v in sd.items()} == cfg["param_shapes"]
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    for k, v in m.state_dict().items():
        assert np.array_equal(v.numpy(), params[k])


def test_cpu_module_runs_the_host_library_never_torch_ops(monkeypatch):
    """A module on the CPU runs libdfwfm_cpu.so (include/dfwfm_cpu.h) -- not the HIP library and not PyTorch's
    generic ops: with the host library made unloadable the forward raises (no fallback either way)."""
    from xsdeepfwfm_deprecated_amd import DeepFMs, DfwfmError, _lib
    cfg, params, xi, xv, *_ = load_golden("deepfwfm_lw")
    m = DeepFMs(**model_kwargs(cfg))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    monkeypatch.setattr(_lib, "_cpu", None)
    monkeypatch.setattr(_lib, "CPU_PATH", "/nonexistent/libdfwfm_cpu.so")
    with pytest.raises(DfwfmError):
        with torch.no_grad():
            m(torch.from_numpy(xi), torch.from_numpy(xv))
    with pytest.raises(DfwfmError):
        m._sync_engine(torch.device("meta"))


def cpu_header_functions():
    src = open(os.path.join(REPO, "include", "dfwfm_cpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dfwfm_cpu_[a-z_]+)\s*\(", src)))


def test_cpu_library_exports_every_header_symbol(built):
    assert cpu_header_functions() == sorted(["dfwfm_cpu_abi_version", "dfwfm_cpu_backward", "dfwfm_cpu_forward",
                                             "dfwfm_cpu_last_error", "dfwfm_cpu_saved_floats"])
    L = ctypes.CDLL(built.CPU_PATH)
    for name in cpu_header_functions():
        assert hasattr(L, name), name
    assert set(built.CPU_SIGNATURES) == set(cpu_header_functions())
    C = built.cpu_lib()
    assert C.dfwfm_cpu_abi_version() == 1
    assert C.dfwfm_cpu_forward(None, None, 0, None, 0, 4, None, None, 0.0, 0, None, 1) == -1
    assert b"null" in C.dfwfm_cpu_last_error()
    assert C.dfwfm_cpu_backward(None, None, 0, None, 0, 4, None, None, 0.0, 0, None, 1) == -1
    assert ctypes.sizeof(built.dfwfm_cpu_model) == 11 * 4 + 4 + 8 * 8


def test_init_weights_distributions():
    from xsdeepfwfm_deprecated_amd import DeepFMs
    cfg, *_ = load_golden("deepfwfm_fwlw_lw")
    m = DeepFMs(**model_kwargs(cfg))
    m.init_weights()
    assert abs(m.fm_2nd_embeddings[20].weight.std().item() - 0.01) < 2e-3
    assert abs(m.field_cov.weight.std().item() - np.sqrt(1 / 39)) < 0.03
    assert abs(m.net_1_linear_2.weight.std().item() - np.sqrt(2 / 800)) < 0.005
    assert abs(m.fm_1st.weight.std().item() - np.sqrt(2 / 450)) < 0.03
    assert m.bias.item() == pytest.approx(0.01)


def test_unsupported_variants_raise():
    from xsdeepfwfm_deprecated_amd import DeepFMs
    cfg, *_ = load_golden("deepfwfm_lw")
    kw = model_kwargs(cfg)
    with pytest.raises(NotImplementedError):
        DeepFMs(**dict(kw, use_fwfm=0, use_ffm=1))
    with pytest.raises(NotImplementedError):
        DeepFMs(**kw, static_quantization=True)
    with pytest.raises(SystemExit):
        DeepFMs(**dict(kw, use_fm=1))  # fwfm and fm together


def test_custom_op_is_registered_with_schema():
    """torch.ops.dfwfm.forward: the forward surfaced as a PyTorch custom operator (torch_ops.py)."""
    import torch
    import xsdeepfwfm_deprecated_amd  # noqa: F401  -- registers the op
    schema = str(torch.ops.dfwfm.forward.default._schema)
    assert schema == ("dfwfm::forward(SymInt model_id, Tensor xi, Tensor xv, Tensor[] params, bool train, "
                      "float dropout_p, SymInt seed) -> (Tensor, Tensor)")


def test_no_library_sort_or_scan_in_kernels():
    """Every kernel of the path is hand-written: no hipcub / rocprim / rocthrust in csrc/ (the eval
    metrics' ranking was the last library-kernel component)."""
    import glob
    import re
    csrc = os.path.join(REPO, "xsdeepfwfm_deprecated_amd", "csrc")
    for path in glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h")):
        with open(path) as f:
            src = f.read()
        assert not re.search(r"#include\s*[<\"](hipcub|rocprim|thrust|rocthrust)", src), path
        assert "hipcub::" not in src and "rocprim::" not in src, path
