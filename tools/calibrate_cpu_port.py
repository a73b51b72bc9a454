"""Calibrate the CPU baseline port (oracle/torch_port.py) against the real reference forward.

Run in the build container only (imports /root/reference; never on the GPU box):

    python tools/calibrate_cpu_port.py [--ref /root/reference] [--iters 5]

For the bench workloads (Criteo-39 tables, batch 4096, bench.py's synthetic weights and inputs) it times
the reference ``model.DeepFMs.DeepFMs.forward`` (reference model/DeepFMs.py:285-469, eval, no_grad) and
``oracle.torch_port.forward`` side by side at 1 thread and at every core of this container, checks that
they return the same logits, and writes ``profiles/cpu_calibration.json``: per (workload, threads) the
mean ms per batch of both and the ratio port / reference.  bench.py reports that file's ratio next to its
GPU-box ``cpu_baseline`` (the port is trusted only with this ratio on record).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import platform
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oracle import torch_port  # noqa: E402
from xsdeepfwfm_deprecated_amd import synth  # noqa: E402

WORKLOADS = {
    # bench.py --config deepfwfm (BASELINE configs[1]) and --config fwfm (configs[0]'s model at Criteo-39)
    "deepfwfm_lw": dict(use_deep=1),
    "fwfm_lw": dict(use_deep=0),
}


def cfg_of(w):
    return dict(field_size=39, numerical=13, embedding_size=10, use_fwfm=1, use_fm=0, use_logit=0,
                use_deep=WORKLOADS[w]["use_deep"], use_lw=1, use_fwlw=0, h_depth=3, deep_nodes=400, embedding_bag=0,
                qr_flag=0, qr_operation="mult", qr_collisions=4, qr_threshold=200)


def time_fn(fn, iters):
    fn()
    t = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return 1e3 * float(np.mean(t))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    sys.path.insert(0, a.ref)
    from model.DeepFMs import DeepFMs as RefDeepFMs  # noqa: E402

    sizes = synth.CRITEO_FEATURE_SIZES
    xi, xv = synth.synth_inputs(sizes, 13, 4096, seed=99)  # bench.py's cpu_baseline batch
    Xi, Xv = torch.from_numpy(xi), torch.from_numpy(xv)
    cores = len(os.sched_getaffinity(0))
    out = {"host": platform.processor() or platform.machine(), "cores": cores, "batch": 4096,
           "torch": torch.__version__, "entries": []}
    try:
        out["host"] = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    for w in WORKLOADS:
        cfg = cfg_of(w)
        ref = RefDeepFMs(field_size=39, feature_sizes=sizes, embedding_size=10, verbose=False, use_cuda=False,
                         use_fm=0, use_fwfm=1, use_ffm=0, use_deep=cfg["use_deep"], h_depth=3, deep_nodes=400,
                         numerical=13, use_lw=1, use_fwlw=0, use_logit=0, logger=logging.getLogger("calib"))
        shapes = {k: tuple(v.shape) for k, v in ref.state_dict().items()}
        params = synth.synth_state(shapes, 39, 10, 400, True, bool(cfg["use_deep"]), seed=1234)
        ref.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
        ref.eval()
        tp = {k: torch.from_numpy(v) for k, v in params.items()}
        with torch.no_grad():
            a_ = ref(Xi.reshape(4096, 26, 1), Xv).double()
            b_ = torch_port.forward(cfg, tp, Xi, Xv).double()
        rel = float(((a_ - b_).abs() / a_.abs().clamp(min=1.0)).max())
        for th in sorted({1, cores}):
            torch.set_num_threads(th)
            with torch.no_grad():
                t_ref = time_fn(lambda: ref(Xi.reshape(4096, 26, 1), Xv), a.iters)
                t_port = time_fn(lambda: torch_port.forward(cfg, tp, Xi, Xv), a.iters)
            e = {"workload": w, "threads": th, "ref_ms_per_batch": round(t_ref, 2),
                 "port_ms_per_batch": round(t_port, 2), "port_over_ref_time": round(t_port / t_ref, 4),
                 "max_rel_logit_diff": rel}
            print(json.dumps(e), flush=True)
            out["entries"].append(e)
    path = os.path.join(REPO, "profiles", "cpu_calibration.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
