"""Time the backward's table scatter alone (DFWFM_BWD_SCATTER after one train forward + per-tile backward) at
Criteo-39 sizes, B = 4096, with the diagnostic phase switches DFWFM_DIAG scatter= (results invalid when set);
--stamps: the sorted scatter's per-workgroup phase clocks (DFWFM_DIAG stamps=3), summarised per task.

    python tools/scatter_diag.py [--iters 50] [--stamps]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def one(iters, stamps=False):
    import torch
    from xsdeepfwfm_deprecated_amd import DeepFMs, _lib, synth
    dev = torch.device("cuda:0")
    sizes = synth.CRITEO_FEATURE_SIZES
    m = DeepFMs(field_size=39, feature_sizes=sizes, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1,
                is_deep_dropout=False).to(dev).train()
    m.init_weights()
    B = 4096
    xi, xv = synth.synth_inputs(sizes, 13, B, seed=3)
    xi_d, xv_d = torch.from_numpy(xi).to(dev), torch.from_numpy(xv).to(dev)
    eng = m._sync_engine(dev)
    eng.set_deterministic(os.environ.get("SCATTER_MODE", "sorted") == "sorted")  # the sorted scatter is deterministic mode's
    out = torch.empty(B, device=dev)
    eng.train_forward(xi_d, xv_d, out, 0.0, 0)
    fields, dense = m._param_layout()
    grads = {id(p): torch.zeros_like(p) for p in m.parameters()}
    ptr = lambda t: None if t is None else grads[id(t)].data_ptr()  # noqa: E731
    fg = (_lib.dfwfm_field_grads * len(fields))(*[_lib.dfwfm_field_grads(*[ptr(t) for t in tup]) for tup in fields])
    H = len(dense["lin_w"])
    gW = (ctypes.c_void_p * H)(*[ptr(t) for t in dense["lin_w"]])
    gB = (ctypes.c_void_p * H)(*[ptr(t) for t in dense["lin_b"]])
    g = _lib.dfwfm_grads(fg, ptr(dense["field_cov"]), ptr(dense["fwfm_lin"]), ptr(dense["fm_1st"]), ptr(dense["bias"]),
                         gW, gB, ptr(dense["fc_w"]))
    L = _lib.lib()
    dl = torch.full((B,), 1e-3, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _lib.check(L.dfwfm_backward_phases(eng.handle, ctypes.c_void_p(dl.data_ptr()), ctypes.byref(g), _lib.BWD_TILES, st),
               "tiles")
    for _ in range(5):
        _lib.check(L.dfwfm_backward_phases(eng.handle, ctypes.c_void_p(dl.data_ptr()), ctypes.byref(g),
                                           _lib.BWD_SCATTER, st), "scatter")
    if stamps:
        import numpy as np
        os.environ["DFWFM_DIAG"] = ",".join(x for x in (os.environ.get("DFWFM_DIAG", ""), "stamps=3") if x)
        for _ in range(3):
            _lib.check(L.dfwfm_backward_phases(eng.handle, ctypes.c_void_p(dl.data_ptr()), ctypes.byref(g),
                                               _lib.BWD_SCATTER, st), "scatter")
        torch.cuda.synchronize()
        n = 512 * 16
        buf = (ctypes.c_uint64 * n)()
        got = L.dfwfm_diag_stamps(eng.handle, buf, n, st)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 16)[:got].astype(np.int64)
        a = a[a[:, 0] > 0]
        names = ["load", "scan", "sort", "flags", "sums", "cuts"]
        rows = []
        for task in np.unique(a[:, 8]):
            w = a[a[:, 8] == task]
            d = np.diff(w[:, 0:7], axis=1)
            rows.append({"task": int(task), "wgs": len(w), "keys_max": int(w[:, 9].max()),
                         "unsorted": int(w[:, 10].sum()),
                         "life": int((w[:, 6] - w[:, 0]).max()),
                         **{k: int(d[:, i].max()) for i, k in enumerate(names)}})
        for r in rows:
            print(json.dumps(r))
        print("per-workgroup shader-clock cycles (max over the task's workgroups); longest life:",
              int((a[:, 6] - a[:, 0]).max()))
        return 0.0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        _lib.check(L.dfwfm_backward_phases(eng.handle, ctypes.c_void_p(dl.data_ptr()), ctypes.byref(g),
                                           _lib.BWD_SCATTER, st), "scatter")
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--stamps", action="store_true")
    a = ap.parse_args()
    if a.stamps:
        one(5, stamps=True)
        sys.exit(0)
    if a.child:
        print(json.dumps({"us": one(a.iters)}))
        sys.exit(0)
    res = {}
    for name, env in [("atomic", {"SCATTER_MODE": "atomic"}), ("sorted", {}), ("nosort", {"DFWFM_DIAG": "scatter=1"}),
                      ("nosums", {"DFWFM_DIAG": "scatter=2"}), ("noadds", {"DFWFM_DIAG": "scatter=4"}),
                      ("keys_only", {"DFWFM_DIAG": "scatter=3"}), ("empty", {"DFWFM_DIAG": "scatter=8"}),
                      ("loads_only", {"DFWFM_DIAG": "scatter=16"})]:
        e = dict(os.environ)
        e.update(env)
        p = subprocess.run([sys.executable, __file__, "--child", "--iters", str(a.iters)], env=e, capture_output=True,
                           text=True, timeout=300)
        line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        res[name] = json.loads(line[0])["us"] if line else p.stderr[-300:]
        print(name, res[name], flush=True)
    print(json.dumps(res))
