"""Per-phase cycle breakdown of the fused backward from in-kernel s_memtime stamps (diagnostic).

    [DFWFM_DIAG=bwd=<bits>] python tools/bwd_stamps.py [--batch 4096] [--iters 5]     (adds stamps=2)

DFWFM_DIAG bwd= (diagnostics, results invalid for 1 and 2): 1 no G_l stores, 2 no mask loads, 4 the generic K loop
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from _diag import diag_set  # noqa: E402
diag_set("stamps", 2)

from xsdeepfwfm_deprecated_amd import DeepFMs, _lib, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda:0")
sizes = synth.CRITEO_FEATURE_SIZES
m = DeepFMs(field_size=39, feature_sizes=sizes, embedding_size=10, use_fwfm=1, use_fm=0, use_deep=1, use_lw=1,
            numerical=13, use_cuda=True)
shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
m.load_state_dict({k: torch.from_numpy(v) for k, v in synth.synth_state(shapes, 39, 10, 400, True, True).items()})
m = m.to(dev).train()
xi, xv = synth.synth_inputs(sizes, 13, a.batch, seed=5)
y = torch.from_numpy(synth.synth_labels(a.batch, seed=5)).float().to(dev)
xi, xv = torch.from_numpy(xi).to(dev), torch.from_numpy(xv).to(dev)
for _ in range(a.iters):
    m.zero_grad()
    F.binary_cross_entropy_with_logits(m(xi, xv), y).backward()
torch.cuda.synchronize()
grid = (a.batch + 15) // 16
buf = (ctypes.c_uint64 * (grid * 16))()
n = _lib.lib().dfwfm_diag_stamps(m._engine.handle, buf, grid * 16,
                                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
st = np.frombuffer(buf, dtype=np.uint64).reshape(grid, 16)[:n].astype(np.int64)
rt0, rt1 = st[:, 10], st[:, 11]
print(f"workgroups {n}; 100 MHz clock: first start -> last start {(rt0.max() - rt0.min()) / 100:.1f} us, "
      f"first start -> last end {(rt1.max() - rt0.min()) / 100:.1f} us, median WG {np.median(rt1 - rt0) / 100:.1f} us")
order = np.argsort(rt0)
print("start offsets (us) by rank:", [(int(q), round((rt0[order[q]] - rt0.min()) / 100, 1)) for q in (0, 63, 127, 191, 255) if q < n])
names = ["P0 stage", "P1 shallow dE (MFMA)", "  . Gram chains (wave 0)", "  . dE pieces (wave 0)",
         "  . reductions, barrier, Gram sums", "P2 G_H init", "layer H", "layer H-1", "layer H-2", "P3 dE store",
         "total"]
slots = [(0, 1), (1, 2), (1, 12), (12, 13), (13, 2), (2, 3), (3, 4), (4, 5), (5, 6), (8, 9), (0, 9)]
for nm, (s0, s1) in zip(names, slots):
    d = st[:, s1] - st[:, s0]
    print(f"{nm:24s} median {np.median(d):10.0f}  p10 {np.percentile(d, 10):10.0f}  p90 {np.percentile(d, 90):10.0f}")
