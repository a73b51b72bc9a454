"""Phase timing of the wave-specialised forwards from in-kernel s_memtime stamps (diagnostic, DFWFM_DIAG_STAMPS=1).

    python tools/ws_stamps.py [--kernel fwd16ws|fwdp] [--batches 20]

fwd16ws (one 4096-row batch): MLP wave 0 passes barrier A (slot 1), ends layer 1's K loop (12), its epilogue (13),
layers (4-6), the end (8); gather wave 8: passes A (2), its rows written (9), passes B (3), FwFM pieces done (10),
sums done (11).  fwdp (a set of `--batches` batches of 4096): prologue by gather wave 8 (rows 1, FwFM 2, sums 3),
MLP wave 0 starts tile 0 (9); for the workgroup's second tile: MLP start (4), K loop of layer h done (5 + h), end
(8); gather wave 8 preparing the third tile: rows (11), FwFM (12), sums (13).  Cycles relative to slot 0.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["DFWFM_DIAG_STAMPS"] = "1"

from xsdeepfwfm_deprecated_amd import DeepFMs, _lib, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kernel", choices=["fwd16ws", "fwdp"], default="fwd16ws")
ap.add_argument("--batches", type=int, default=20)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
dev = torch.device("cuda:0")
sizes = synth.CRITEO_FEATURE_SIZES
m = DeepFMs(field_size=39, feature_sizes=sizes, embedding_size=10, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1,
            numerical=13, use_cuda=True)
shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
m.load_state_dict({k: torch.from_numpy(v) for k, v in synth.synth_state(shapes, 39, 10, 400, True, True).items()})
m = m.to(dev).eval()
m.strict_index_check = False
eng = m._sync_engine(dev)
nb = 1 if a.kernel == "fwd16ws" else a.batches
data = []
for i in range(nb):
    xi, xv = synth.synth_inputs(sizes, 13, 4096, seed=5 + i)
    data.append((torch.from_numpy(xi).to(dev), torch.from_numpy(xv).to(dev)))
outs = [torch.empty(4096, device=dev) for _ in data]
with torch.no_grad():
    for _ in range(a.iters):
        if nb == 1:
            eng.forward(data[0][0], data[0][1], outs[0])
        else:
            eng.forward_batches(data, outs)
torch.cuda.synchronize()
grid = nb * 256
buf = (ctypes.c_uint64 * (grid * 16))()
n = _lib.lib().dfwfm_diag_stamps(eng.handle, buf, grid * 16, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
st = np.frombuffer(buf, dtype=np.uint64).reshape(grid, 16)[:n].astype(np.int64)
if a.kernel == "fwdp":
    st = st[:256]
    st = st[st[:, 8] > st[:, 0]]  # workgroups with a second tile
rel = st - st[:, :1]
names = ({1: "MLP passes A", 2: "gather passes A", 9: "gather rows written", 3: "gather passes B",
          10: "gather FwFM pieces done", 11: "gather sums done", 12: "MLP layer-1 K loop done", 13: "MLP epilogue 1 done",
          4: "MLP layer 1 done", 5: "MLP layer 2 done", 6: "MLP layer 3 done", 8: "end"}
         if a.kernel == "fwd16ws" else
         {1: "prologue: gather rows", 2: "prologue: FwFM", 3: "prologue: sums", 9: "MLP starts tile 0",
          4: "tile 1 start", 5: "tile 1 L1 K loop done", 11: "gather (tile 2) rows done", 6: "tile 1 L2 K loop done",
          12: "gather (tile 2) FwFM done", 7: "tile 1 L3 K loop done", 13: "gather (tile 2) sums done",
          8: "tile 1 end"})
print(f"{a.kernel}: {len(st)} workgroups; cycles since the workgroup's start (median / p10 / p90)")
for slot, nm in sorted(names.items(), key=lambda kv: np.median(rel[:, kv[0]])):
    v = rel[:, slot]
    print(f"  slot {slot:2d} {nm:28s} {np.median(v):9.0f} {np.percentile(v, 10):9.0f} {np.percentile(v, 90):9.0f}")
