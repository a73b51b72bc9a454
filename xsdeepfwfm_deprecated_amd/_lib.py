"""ctypes binding of libdfwfm.so (the C ABI declared in include/dfwfm.h).

The shared library is built in-tree with hipcc for gfx950 (``build()``) and
loaded after ``torch`` so that it binds to the HIP runtime torch already
loaded (both carry the SONAME ``libamdhip64.so.7``): torch's device memory and
streams are then directly usable by the kernels.

There is no CPU fallback: if the library cannot be loaded, every entry point
raises.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import torch  # noqa: F401  -- must precede the library load (shared HIP runtime)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "libdfwfm.so")
# A/B of build variants only (e.g. libdfwfm_ns4.so built with DFWFM_HIPCC_FLAGS=-DDFWFM_NSETS=4)
LOAD_PATH = os.path.join(PKG_DIR, os.environ["DFWFM_LIB"]) if os.environ.get("DFWFM_LIB") else LIB_PATH
SOURCES = ["dfwfm_kernels.hip", "dfwfm_fwd32.hip", "dfwfm_ftrain.hip", "dfwfm_train.hip", "dfwfm_prune.hip", "dfwfm_metrics.hip", "dfwfm_sparse.hip",
           "dfwfm_spmlp.hip", "dfwfm_capi.hip"]
# the forward / backward kernel templates are instantiated once per embedding size, each size in its own
# translation unit (-DDFWFM_KD=<D>) so they compile in parallel; the plain object holds everything else
EMB_SIZES = (4, 8, 10, 16, 32)
PER_D_SOURCES = ["dfwfm_kernels.hip", "dfwfm_train.hip"]


def _units():
    """(source, object, extra flags) of every translation unit of libdfwfm.so."""
    u = [(s, os.path.splitext(s)[0] + ".o", []) for s in SOURCES]
    for s in PER_D_SOURCES:
        u += [(s, f"{os.path.splitext(s)[0]}_d{d}.o", [f"-DDFWFM_KD={d}"]) for d in EMB_SIZES]
    return u
HEADERS = ["dfwfm_internal.h", "dfwfm_device.h", os.path.join("..", "..", "include", "dfwfm.h")]
ARCH = os.environ.get("DFWFM_OFFLOAD_ARCH", "gfx950")
CPU_PATH = os.path.join(PKG_DIR, "libdfwfm_cpu.so")
CPU_SOURCES = ["dfwfm_cpu.cpp"]
CPU_HEADERS = [os.path.join("..", "..", "include", "dfwfm_cpu.h"), os.path.join("..", "..", "include", "dfwfm.h")]
INGEST_PATH = os.path.join(PKG_DIR, "libdfwfm_ingest.so")
INGEST_SOURCES = ["dfwfm_ingest.cpp"]
INGEST_HEADERS = [os.path.join("..", "..", "include", "dfwfm_ingest.h")]

DFWFM_OK = 0
STATUS = {0: "ok", -1: "invalid argument", -2: "unsupported", -3: "HIP error", -4: "bad state"}
FLAG_INDEX_OUT_OF_RANGE = 1
BWD_TABLES, BWD_MLP_WEIGHTS, BWD_TILES, BWD_SPREAD, BWD_REDUCE, BWD_SCATTER = 1, 2, 4, 8, 16, 32  # dfwfm_backward_phases
FAMILY_SECOND, FAMILY_FIRST = 0, 1  # dfwfm_sparse_grads_local
ADAM_STATE_BYTES = 48


class DfwfmError(RuntimeError):
    pass


class dfwfm_config(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "field_size", "numerical", "embedding_size", "use_fwfm", "use_fm", "use_logit",
        "use_deep", "use_lw", "use_fwlw", "h_depth", "deep_nodes")]


class dfwfm_field_tables(ctypes.Structure):
    _fields_ = [
        ("emb2", ctypes.c_void_p), ("emb2_r", ctypes.c_void_p),
        ("emb1", ctypes.c_void_p), ("emb1_r", ctypes.c_void_p),
        ("num_categories", ctypes.c_int64), ("qr_collisions", ctypes.c_int64),
        ("qr_operation", ctypes.c_int32), ("reserved", ctypes.c_int32),
    ]


class dfwfm_field_grads(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("emb2", "emb2_r", "emb1", "emb1_r")]


class dfwfm_grads(ctypes.Structure):
    _fields_ = [
        ("fields", ctypes.POINTER(dfwfm_field_grads)),
        ("field_cov", ctypes.c_void_p), ("fwfm_lin", ctypes.c_void_p), ("fm_1st", ctypes.c_void_p),
        ("bias", ctypes.c_void_p), ("lin_w", ctypes.POINTER(ctypes.c_void_p)),
        ("lin_b", ctypes.POINTER(ctypes.c_void_p)), ("fc_w", ctypes.c_void_p),
    ]


class dfwfm_adam_tensor(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("numel", ctypes.c_int64)]


class dfwfm_sparse_dest(ctypes.Structure):
    _fields_ = [("q", ctypes.c_int64), ("r", ctypes.c_int64)]


class dfwfm_prune_source(ctypes.Structure):
    _fields_ = [("values", ctypes.c_void_p), ("numel", ctypes.c_int64), ("sym_f", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


# name -> (restype, argtypes); every symbol include/dfwfm.h declares
_P = ctypes.c_void_p
SIGNATURES = {
    "dfwfm_model_create": (ctypes.c_int, [ctypes.POINTER(dfwfm_config), ctypes.POINTER(_P)]),
    "dfwfm_model_destroy": (None, [_P]),
    "dfwfm_model_set_tables": (ctypes.c_int, [_P, ctypes.POINTER(dfwfm_field_tables), ctypes.c_int32, _P]),
    "dfwfm_model_set_dense": (ctypes.c_int, [_P, _P, _P, _P, _P, ctypes.POINTER(_P), ctypes.POINTER(_P), _P, _P]),
    "dfwfm_model_set_dense_zero": (ctypes.c_int, [_P, _P, _P, _P, _P, ctypes.POINTER(_P), ctypes.POINTER(_P), _P, _P,
                                                  ctypes.c_int64, _P]),
    "dfwfm_forward": (ctypes.c_int, [_P, _P, ctypes.c_int64, _P, ctypes.c_int64, ctypes.c_int64, _P, _P]),
    "dfwfm_forward_batches": (ctypes.c_int, [_P, ctypes.c_int32, _P, ctypes.c_int64, _P, ctypes.c_int64,
                                             ctypes.c_int64, _P, _P]),
    "dfwfm_forward_workspace_bytes": (ctypes.c_int, [_P, ctypes.c_int64, ctypes.POINTER(ctypes.c_size_t)]),
    "dfwfm_forward_ws": (ctypes.c_int, [_P, _P, ctypes.c_int64, _P, ctypes.c_int64, ctypes.c_int64, _P, _P,
                                        ctypes.c_size_t, _P]),
    "dfwfm_model_build_sparse_mlp": (ctypes.c_int, [_P, ctypes.c_double, ctypes.POINTER(ctypes.c_int32), _P]),
    "dfwfm_model_build_fwfm_pairs": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), _P]),
    "dfwfm_model_pack_tables": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), _P]),
    "dfwfm_forward_gather": (ctypes.c_int, [_P, _P, ctypes.c_int64, _P, ctypes.c_int64, ctypes.c_int64, _P,
                                            ctypes.c_int64, _P, _P]),
    "dfwfm_train_forward": (ctypes.c_int, [_P, _P, ctypes.c_int64, _P, ctypes.c_int64, ctypes.c_int64, _P,
                                           ctypes.c_float, ctypes.c_uint32, _P]),
    "dfwfm_backward": (ctypes.c_int, [_P, _P, ctypes.POINTER(dfwfm_grads), _P]),
    "dfwfm_backward_phases": (ctypes.c_int, [_P, _P, ctypes.POINTER(dfwfm_grads), ctypes.c_int32, _P]),
    "dfwfm_adam_step": (ctypes.c_int, [ctypes.POINTER(dfwfm_adam_tensor), ctypes.c_int32, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_int64, _P]),
    "dfwfm_set_step_source": (ctypes.c_int, [_P, _P]),
    "dfwfm_workspace_generation": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int64)]),
    "dfwfm_adam_step_dev": (ctypes.c_int, [ctypes.POINTER(dfwfm_adam_tensor), ctypes.c_int32, ctypes.c_double,
                                           ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                           _P, _P]),
    "dfwfm_bce_grad": (ctypes.c_int, [_P, _P, ctypes.c_int64, ctypes.c_double, _P, _P, _P]),
    "dfwfm_backward_phases_bce": (ctypes.c_int, [_P, _P, _P, ctypes.c_double, _P, _P, ctypes.POINTER(dfwfm_grads),
                                                 ctypes.c_int32, _P]),
    "dfwfm_sparse_grads_size": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                                               ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64)]),
    "dfwfm_sparse_grads_apply": (ctypes.c_int, [_P, ctypes.c_int32, _P, _P, _P, ctypes.c_int64, _P]),
    "dfwfm_sparse_grads_local": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.POINTER(dfwfm_sparse_dest), ctypes.c_int64,
                                                _P, _P, ctypes.c_int64, _P, _P, _P, _P]),
    "dfwfm_prune_workspace_bytes": (ctypes.c_int64, [ctypes.c_int64]),
    "dfwfm_prune_threshold": (ctypes.c_int, [ctypes.POINTER(dfwfm_prune_source), ctypes.c_int32, ctypes.c_double,
                                             _P, _P, ctypes.c_int64, _P]),
    "dfwfm_prune_apply": (ctypes.c_int, [_P, ctypes.c_int64, ctypes.c_int32, _P, _P]),
    "dfwfm_metrics_workspace_bytes": (ctypes.c_int64, [ctypes.c_int64]),
    "dfwfm_eval_metrics": (ctypes.c_int, [_P, _P, ctypes.c_int64, _P, _P, ctypes.c_int64, _P]),
    "dfwfm_read_error_flag": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int32), _P]),
    "dfwfm_last_error": (ctypes.c_char_p, []),
    "dfwfm_diag_stamps": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int64, _P]),
    "dfwfm_abi_version": (ctypes.c_int, []),
    "dfwfm_set_deterministic": (ctypes.c_int, [_P, ctypes.c_int32]),
}

_lib = None
_lock = threading.Lock()


def _stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _stale_ingest() -> bool:
    if not os.path.exists(INGEST_PATH):
        return True
    t = os.path.getmtime(INGEST_PATH)
    deps = [os.path.join(CSRC, s) for s in INGEST_SOURCES + INGEST_HEADERS]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_ingest(force: bool = False, verbose: bool = False) -> str:
    """Compile the host-only ingest library (g++, no GPU code)."""
    if not force and not _stale_ingest():
        return INGEST_PATH
    cxx = os.environ.get("CXX", "g++")
    tmp = INGEST_PATH + ".tmp"
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", tmp] + \
        [os.path.join(CSRC, s) for s in INGEST_SOURCES]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(tmp, INGEST_PATH)
    return INGEST_PATH


def _stale_cpu() -> bool:
    if not os.path.exists(CPU_PATH):
        return True
    t = os.path.getmtime(CPU_PATH)
    deps = [os.path.join(CSRC, s) for s in CPU_SOURCES + CPU_HEADERS]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_cpu(force: bool = False, verbose: bool = False) -> str:
    """Compile the host forward / backward library (g++, AVX2 + FMA, std::thread; include/dfwfm_cpu.h): the CPU
    kernel of torch.ops.dfwfm.forward for modules on the CPU."""
    if not force and not _stale_cpu():
        return CPU_PATH
    cxx = os.environ.get("CXX", "g++")
    tmp = CPU_PATH + ".tmp"
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-mavx2", "-mfma", "-o", tmp] + \
        [os.path.join(CSRC, s) for s in CPU_SOURCES]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(tmp, CPU_PATH)
    return CPU_PATH


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile libdfwfm.so for gfx950 in-tree (hipcc cross-compiles without a GPU): one object per
    translation unit, compiled in parallel, then linked; and the host-only ingest and CPU-kernel libraries."""
    build_ingest(force, verbose)
    build_cpu(force, verbose)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC"] + os.environ.get("DFWFM_HIPCC_FLAGS", "").split()
    stamp = os.path.join(CSRC, ".build_flags")  # objects (and the library) built with other flags are stale
    if not os.path.exists(stamp) or open(stamp).read() != " ".join(flags):
        force = True
    if not force and not _stale():
        return LIB_PATH
    from concurrent.futures import ThreadPoolExecutor
    units = _units()
    objs = [os.path.join(CSRC, o) for _, o, _ in units]
    hdr_m = max(os.path.getmtime(os.path.join(CSRC, h)) for h in HEADERS)

    def compile_one(i):
        src, _, extra = units[i]
        src = os.path.join(CSRC, src)
        if not force and os.path.exists(objs[i]) and \
                os.path.getmtime(objs[i]) >= max(os.path.getmtime(src), hdr_m):
            return  # object up to date (kept between builds; *.o is git- and gpurun-ignored)
        cmd = [hipcc] + flags + extra + ["-c", "-o", objs[i], src]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True, cwd=CSRC)

    jobs = int(os.environ.get("MAX_JOBS", "0")) or min(len(units), max(1, len(os.sched_getaffinity(0))))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(compile_one, range(len(units))))
    with open(stamp, "w") as f:
        f.write(" ".join(flags))
    tmp = LIB_PATH + ".tmp"
    subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-o", tmp] + objs, check=True, cwd=CSRC)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


_ingest = None
INGEST_SIGNATURES = {
    "dfwfm_csv_open": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p),
                                      ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32)]),
    "dfwfm_csv_parse": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_int32]),
    "dfwfm_csv_close": (None, [ctypes.c_void_p]),
    "dfwfm_feature_map_counts": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]),
    "dfwfm_ingest_last_error": (ctypes.c_char_p, []),
}


class dfwfm_cpu_model(ctypes.Structure):
    _fields_ = [("cfg", dfwfm_config), ("fields", ctypes.POINTER(dfwfm_field_tables)),
                ("field_cov", ctypes.c_void_p), ("fwfm_lin", ctypes.c_void_p), ("fm_1st", ctypes.c_void_p),
                ("bias", ctypes.c_void_p), ("lin_w", ctypes.POINTER(ctypes.c_void_p)),
                ("lin_b", ctypes.POINTER(ctypes.c_void_p)), ("fc_w", ctypes.c_void_p)]


_cpu = None
CPU_SIGNATURES = {
    "dfwfm_cpu_saved_floats": (ctypes.c_int64, [ctypes.POINTER(dfwfm_config)]),
    "dfwfm_cpu_forward": (ctypes.c_int, [ctypes.POINTER(dfwfm_cpu_model), _P, ctypes.c_int64, _P, ctypes.c_int64,
                                         ctypes.c_int64, _P, _P, ctypes.c_float, ctypes.c_uint32,
                                         ctypes.POINTER(ctypes.c_int32), ctypes.c_int32]),
    "dfwfm_cpu_backward": (ctypes.c_int, [ctypes.POINTER(dfwfm_cpu_model), _P, ctypes.c_int64, _P, ctypes.c_int64,
                                          ctypes.c_int64, _P, _P, ctypes.c_float, ctypes.c_uint32,
                                          ctypes.POINTER(dfwfm_grads), ctypes.c_int32]),
    "dfwfm_cpu_last_error": (ctypes.c_char_p, []),
    "dfwfm_cpu_abi_version": (ctypes.c_int, []),
}


def cpu_lib():
    """The host-kernel library (include/dfwfm_cpu.h); raises DfwfmError if it is missing."""
    global _cpu
    if _cpu is not None:
        return _cpu
    with _lock:
        if _cpu is None:
            if not os.path.exists(CPU_PATH):
                raise DfwfmError(f"{CPU_PATH} is missing: run xsdeepfwfm_deprecated_amd.build()")
            L = ctypes.CDLL(CPU_PATH)
            for name, (res, args) in CPU_SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            if L.dfwfm_cpu_abi_version() != 1:
                raise DfwfmError("libdfwfm_cpu ABI mismatch")
            _cpu = L
    return _cpu


def check_cpu(rc: int, what: str) -> None:
    if rc != DFWFM_OK:
        msg = cpu_lib().dfwfm_cpu_last_error().decode(errors="replace")
        raise DfwfmError(f"{what} failed ({STATUS.get(rc, rc)}): {msg}")


def ingest_lib():
    """The host ingest library (include/dfwfm_ingest.h); raises DfwfmError if it is missing."""
    global _ingest
    if _ingest is not None:
        return _ingest
    with _lock:
        if _ingest is None:
            if not os.path.exists(INGEST_PATH):
                raise DfwfmError(f"{INGEST_PATH} is missing: run xsdeepfwfm_deprecated_amd.build()")
            L = ctypes.CDLL(INGEST_PATH)
            for name, (res, args) in INGEST_SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _ingest = L
    return _ingest


def lib():
    """The loaded library; raises DfwfmError if it is missing (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LOAD_PATH):
            raise DfwfmError(f"{LOAD_PATH} is missing: run xsdeepfwfm_deprecated_amd.build() "
                             "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        L = ctypes.CDLL(LOAD_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.dfwfm_abi_version() != 4:
            raise DfwfmError("libdfwfm ABI mismatch")
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != DFWFM_OK:
        msg = lib().dfwfm_last_error().decode(errors="replace")
        raise DfwfmError(f"{what} failed ({STATUS.get(rc, rc)}): {msg}")
