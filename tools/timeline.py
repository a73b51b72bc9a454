"""Cross-launch timeline of the fused forward (diagnostic): S streams x G graph-captured forwards,
every workgroup's start / end on the 100 MHz clock, its CU, and its phase boundaries (shader clock,
mapped onto the workgroup's own start..end).  Shows how the streams' workgroups share the CUs.

    python tools/timeline.py [--streams 2] [--graph-steps 20]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ap = argparse.ArgumentParser()
ap.add_argument("--streams", type=int, default=2)
ap.add_argument("--graph-steps", type=int, default=20)
ap.add_argument("--replays", type=int, default=5)
ap.add_argument("--fwfm", action="store_true", help="FwFM-only model (use_deep=0)")
a = ap.parse_args()
from _diag import diag_set  # noqa: E402
diag_set("stamps", 1)
diag_set("ring", a.streams * a.graph_steps)

from xsdeepfwfm_deprecated_amd import DeepFMs, _lib, synth  # noqa: E402

B = 4096
dev = torch.device("cuda:0")
sizes = synth.CRITEO_FEATURE_SIZES
m = DeepFMs(field_size=39, feature_sizes=sizes, embedding_size=10, use_fwfm=1, use_fm=0, use_deep=0 if a.fwfm else 1, use_lw=1,
            numerical=13, use_cuda=True)
shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
m.load_state_dict({k: torch.from_numpy(v) for k, v in synth.synth_state(shapes, 39, 10, 400, True, True).items()
                   if k in shapes})
m = m.to(dev).eval()
m.strict_index_check = False
S, G = a.streams, a.graph_steps
bufs = []
for i in range(4):
    xi, xv = synth.synth_inputs(sizes, 13, B, seed=i)
    bufs.append((torch.from_numpy(xi).to(dev), torch.from_numpy(xv).to(dev)))
outs = [torch.empty(B, device=dev) for _ in range(S)]
with torch.no_grad():
    eng = m._sync_engine(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    for k in range(S):
        streams[k].wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(streams[k]):
            eng.forward(*bufs[k], outs[k])
    torch.cuda.synchronize()
    graphs = []
    for k in range(S):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=streams[k]):
            for i in range(G):
                eng.forward(*bufs[(i + k) % 4], outs[k])
        graphs.append(g)
    for _ in range(a.replays):
        for k in range(S):
            with torch.cuda.stream(streams[k]):
                graphs[k].replay()
    torch.cuda.synchronize()

grid = B // 16
n_slots = S * G * grid * 16
buf = (ctypes.c_uint64 * n_slots)()
n = _lib.lib().dfwfm_diag_stamps(eng.handle, buf, n_slots, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
st = np.frombuffer(buf, dtype=np.uint64).reshape(S * G, grid, 16)
# slot (launch order during capture): stream k's forward i is launch k*G + i
t0 = (st[:, :, 14] & ((1 << 48) - 1)).astype(np.int64)
t1 = (st[:, :, 15] & ((1 << 48) - 1)).astype(np.int64)
cu = ((st[:, :, 15] >> 48) & 0xFFF).astype(np.int64)
base = t0.min()
t0 = (t0 - base) * 10  # ns
t1 = (t1 - base) * 10
mt = st[:, :, :14].astype(np.int64)
frac_mlp = ((mt[:, :, 3] - mt[:, :, 0]) / np.maximum(1, mt[:, :, 8] - mt[:, :, 0])) if not a.fwfm else np.ones_like(mt[:, :, 0], dtype=float)
tm = t0 + (t1 - t0) * frac_mlp  # MLP start, ns

print(f"launches {S}x{G}, {grid} workgroups each, distinct CUs seen {len(np.unique(cu))}")
for k in range(S):
    for i in range(min(G, 6)):
        L = k * G + i
        d = t1[L] - t0[L]
        print(f"  stream {k} fwd {i}: start {t0[L].min()/1e3:8.2f} us  starts spread {(t0[L].max()-t0[L].min())/1e3:6.2f}  "
              f"end {t1[L].max()/1e3:8.2f}  launch {(t1[L].max()-t0[L].min())/1e3:6.2f} us  "
              f"wg dur p10/50/90 {np.percentile(d,10)/1e3:5.1f}/{np.median(d)/1e3:5.1f}/{np.percentile(d,90)/1e3:5.1f}  "
              f"pre-MLP median {np.median(tm[L]-t0[L])/1e3:5.2f}")
# steady-state window: after every stream's 3rd launch started, before any stream's last launch ended
lo = max(t0[k * G + 2].min() for k in range(S))
hi = min(t1[k * G + G - 3].max() for k in range(S))
step = 100  # ns
ts = np.arange(lo, hi, step)
cus = np.unique(cu)
occ = np.zeros((len(cus), len(ts)), np.int8)
mlp = np.zeros((len(cus), len(ts)), np.int8)
idx = {c: j for j, c in enumerate(cus)}
for L in range(S * G):
    for w in range(grid):
        j = idx[cu[L, w]]
        a0 = np.searchsorted(ts, t0[L, w])
        a1 = np.searchsorted(ts, t1[L, w])
        am = np.searchsorted(ts, tm[L, w])
        occ[j, a0:a1] += 1
        mlp[j, am:a1] += 1
tot = occ.size
print(f"steady window {(hi-lo)/1e3:.1f} us over {len(cus)} CUs: resident workgroups per CU "
      + ", ".join(f"{v}: {100*np.mean(occ==v):.1f}%" for v in range(4)))
print("  workgroups in MLP per CU " + ", ".join(f"{v}: {100*np.mean(mlp==v):.1f}%" for v in range(3)))
print("  CU with >=1 in MLP and another pre-MLP: "
      f"{100*np.mean((mlp>=1)&(occ>mlp)):.1f}%   both pre-MLP: {100*np.mean((mlp==0)&(occ>=2)):.1f}%")
per_cu = np.array([np.sum(cu == c) for c in cus])
print(f"  workgroups per CU over all launches: min {per_cu.min()} max {per_cu.max()} (ideal {S*G*grid/len(cus):.1f})")
names = [("stage", 0, 1), ("gather", 1, 2), ("fwlw", 2, 9), ("FwFM MFMA", 9, 10), ("barrier", 10, 11),
         ("sums", 11, 3), ("MLP L1 K loop", 3, 12), ("L1 epilogue", 12, 13), ("L1 barrier", 13, 4),
         ("MLP L2", 4, 5), ("MLP L3", 5, 6), ("combine", 6, 8)]
if a.fwfm:
    names = [("stage", 0, 1), ("gather", 1, 2), ("fwlw", 2, 9), ("FwFM MFMA", 9, 10), ("  piece 1 loads+MFMA issue", 9, 3),
             ("  piece 1 epilogue", 3, 4), ("  piece 2", 4, 5), ("  piece 3", 5, 6), ("barrier", 10, 11),
             ("sums + store", 11, 8)]
sel = mt[2 * S:(G - 2) * S]
tot = np.median(sel[:, :, 8] - sel[:, :, 0])
print(f"phase medians (shader cycles), total {tot:.0f}:")
for nm, x, y in names:
    d = sel[:, :, y] - sel[:, :, x]
    print(f"  {nm:16s} {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}")
