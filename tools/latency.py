"""Forward latency, one call at a time (the reference's run_benchmark / time_forward_pass, model/DeepFMs.py:982-1019:
per-sample latency = single-sample forwards timed one by one; per-batch latency = one batch forward at a time).

Criteo-39 DeepFwFM (lw) and the FwFM-only model on one MI355X, synthetic inputs of the real field sizes, weights with
the init_weights scales.  Each call is one forward through the C ABI (eng.forward) on an otherwise idle GPU, timed
with HIP events around it (device time) and by the host clock around launch + synchronize (what a caller waits); a
batch's forward is also replayed from a one-forward hipGraph (launch overhead of a serving loop that captures).
Prints one JSON line.

  python tools/latency.py [--calls 1000] [--batches 1,16,64,256,1024,4096,8192]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def build(deep, dev):
    from xsdeepfwfm_deprecated_amd import DeepFMs, synth
    sizes = synth.CRITEO_FEATURE_SIZES
    m = DeepFMs(field_size=39, feature_sizes=sizes, embedding_size=10, use_fwfm=1, use_fm=0, use_deep=deep,
                use_lw=1, numerical=13, use_cuda=True)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    params = synth.synth_state(shapes, 39, 10, 400, True, bool(deep), seed=1234)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    m = m.to(dev).eval()
    m.strict_index_check = False
    return m, sizes


def measure(eng, xi, xv, out, calls, dev):
    """median / p99 device time per call (events), median host time per call (launch + synchronize), and the
    median device time of a one-forward graph replay"""
    st = torch.cuda.current_stream(dev)
    for _ in range(20):
        eng.forward(xi, xv, out)
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(calls)]
    host = []
    for e0, e1 in ev:
        t0 = time.perf_counter()
        e0.record(st)
        eng.forward(xi, xv, out)
        e1.record(st)
        e1.synchronize()
        host.append(time.perf_counter() - t0)
    dev_us = np.array([e0.elapsed_time(e1) * 1e3 for e0, e1 in ev])
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        eng.forward(xi, xv, out)
    torch.cuda.synchronize(dev)
    ghost = []
    for _ in range(calls):
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize(dev)
        ghost.append(time.perf_counter() - t0)
    # back to back: 20 calls per graph, replayed without a host sync in between (a serving loop's steady state;
    # the idle gap of a synchronised call lets the chip lower its clock)
    g20 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g20):
        for _ in range(20):
            eng.forward(xi, xv, out)
    reps = max(5, calls // 20)
    for _ in range(reps):
        g20.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        g20.replay()
    e1.record(st)
    e1.synchronize()
    return {"device_us_median": round(float(np.median(dev_us)), 2), "device_us_p99": round(float(np.percentile(dev_us, 99)), 2),
            "host_us_median": round(float(np.median(host)) * 1e6, 2),
            "graph_host_us_median": round(float(np.median(ghost)) * 1e6, 2),
            "back_to_back_us": round(e0.elapsed_time(e1) * 1e3 / (reps * 20), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=1000)
    ap.add_argument("--batches", default="1,16,64,256,1024,4096,8192")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from xsdeepfwfm_deprecated_amd import synth
    res = {"what": "forward latency, one call at a time on an idle MI355X (reference run_benchmark per-sample / "
                   "per-batch latency, model/DeepFMs.py:982-1019); reference published 1.979 ms per sample on CPU "
                   "(data/results/criteo.md:5)", "calls": a.calls, "models": {}}
    for name, deep in (("deepfwfm", 1), ("fwfm", 0)):
        m, sizes = build(deep, dev)
        rows = {}
        with torch.no_grad():
            eng = m._sync_engine(dev)
            for b in [int(x) for x in a.batches.split(",")]:
                xi, xv = synth.synth_inputs(sizes, 13, b, seed=7)
                xi, xv = torch.from_numpy(xi).to(dev), torch.from_numpy(xv).to(dev)
                out = torch.empty(b, dtype=torch.float32, device=dev)
                r = measure(eng, xi, xv, out, a.calls if b <= 256 else max(100, a.calls // 10), dev)
                r["samples_per_s_one_call_at_a_time"] = round(b / (r["device_us_median"] * 1e-6), 1)
                if deep:  # f32 MFMA fraction of the back-to-back rate (967,620 FLOP per sample, 157.3 TF/s)
                    r["mfma_frac_back_to_back"] = round(967620 * b / (r["back_to_back_us"] * 1e-6) / 157.3e12, 4)
                rows[str(b)] = r
        res["models"][name] = rows
    print(json.dumps(res))


if __name__ == "__main__":
    main()
