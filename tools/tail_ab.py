"""Batch-set tail experiment (diagnostic): a 20-batch set as one fwd32 launch against the set split into a main part
(fwd32, 32-sample workgroups) and a tail of k batches (16-sample workgroups: fwd_kernel) on a second stream, with and
without stream priorities (main high, tail low: the tail's small workgroups are dispatched as the main launch's last
workgroups drain).  Prints per-variant median us per 20 batches and checks the logits stay bit-identical.

    python tools/tail_ab.py [--reps 30]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xsdeepfwfm_deprecated_amd import DeepFMs, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--nb", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda:0")
sizes = synth.CRITEO_FEATURE_SIZES
m = DeepFMs(field_size=39, feature_sizes=sizes, embedding_size=10, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1,
            numerical=13, use_cuda=True)
shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
m.load_state_dict({k: torch.from_numpy(v) for k, v in synth.synth_state(shapes, 39, 10, 400, True, True).items()})
m = m.to(dev).eval()
m.strict_index_check = False
B, NB = 4096, a.nb
data = []
for i in range(NB):
    xi, xv = synth.synth_inputs(sizes, 13, B, seed=5 + i)
    data.append((torch.from_numpy(xi).to(dev), torch.from_numpy(xv).to(dev)))
outs = [torch.empty(B, device=dev) for _ in data]
m._sync_inference(dev)
eng = m._sync_engine(dev)
print("priority range", torch.cuda.Stream.priority_range(), flush=True)
lo_p, hi_p = torch.cuda.Stream.priority_range()
streams = {"hi": torch.cuda.Stream(priority=hi_p), "lo": torch.cuda.Stream(priority=lo_p),
           "p1": torch.cuda.Stream(), "p2": torch.cuda.Stream()}


def run(k, prio, tail_first=False):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(2_000_000)  # the GPU busy while the host enqueues: the interval holds no host time
    e0.record(s)
    if k == 0:
        eng.forward_batches(data, outs)
        e1.record(s)
        return e0, e1
    sa, sb = (streams["hi"], streams["lo"]) if prio else (streams["p1"], streams["p2"])
    sa.wait_event(e0)
    sb.wait_event(e0)

    def main():
        with torch.cuda.stream(sa):
            eng.forward_batches(data[:NB - k], outs[:NB - k])

    def tail():
        with torch.cuda.stream(sb):
            eng.forward_batches(data[NB - k:], outs[NB - k:])
    if tail_first:
        tail(); main()
    else:
        main(); tail()
    s.wait_stream(sa)
    s.wait_stream(sb)
    e1.record(s)
    return e0, e1


variants = [(0, False, False)] + [(k, p, f) for k in (1, 2, 3, 4) for p in (False, True) for f in (False, True)]
ref = None
res = {}
for v in variants:
    for _ in range(5):
        run(*v)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        e0, e1 = run(*v)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    got = torch.stack([o.clone() for o in outs]).cpu().numpy()
    if ref is None:
        ref = got
    name = f"k{v[0]}{'_prio' if v[1] else ''}{'_tailfirst' if v[2] else ''}"
    res[name] = round(float(np.median(ts)), 1)
    print(name, res[name], "us per", NB, "batches;", round(res[name] / NB, 2), "us/batch; bit-identical",
          bool(np.array_equal(got, ref)), flush=True)
print(json.dumps(res))
