"""Per-phase cycle breakdown of the fused forward from in-kernel s_memtime stamps (diagnostic).

    [DFWFM_DIAG=r32=1] python tools/phase_stamps.py [--batch 4096] [--iters 20] [--fwfm] [--batches N]

--fwfm: the MLP-free FwFM-only model (fwd_kernel PART 3); --batches N: N distinct resident batches as one batch set
(dfwfm_forward_batches), with the launch's workgroup lifetimes and concurrency from the 100 MHz stamps.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from _diag import diag_get, diag_set  # noqa: E402
diag_set("stamps", 1, overwrite=False)

from xsdeepfwfm_deprecated_amd import DeepFMs, _lib, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--fwlw", action="store_true")
ap.add_argument("--train", action="store_true", help="stamp the training-mode forward (activations saved)")
ap.add_argument("--fwfm", action="store_true", help="the MLP-free FwFM-only model")
ap.add_argument("--batches", type=int, default=1, help="a batch set of this many distinct batches")
a = ap.parse_args()
dev = torch.device("cuda:0")
sizes = synth.CRITEO_FEATURE_SIZES
m = DeepFMs(field_size=39, feature_sizes=sizes, embedding_size=10, use_fwfm=1, use_fm=0, use_deep=0 if a.fwfm else 1,
            use_lw=1,
            use_fwlw=a.fwlw, numerical=13, use_cuda=True)
shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
m.load_state_dict({k: torch.from_numpy(v) for k, v in synth.synth_state(shapes, 39, 10, 400, True, True).items()})
m = m.to(dev).train() if a.train else m.to(dev).eval()
m.strict_index_check = False
data = []
for i in range(a.batches):
    xi, xv = synth.synth_inputs(sizes, 13, a.batch, seed=5 + i)
    data.append((torch.from_numpy(xi).to(dev), torch.from_numpy(xv).to(dev)))
xi, xv = data[0]
outs = [torch.empty(a.batch, device=dev) for _ in data]
if a.train:
    from xsdeepfwfm_deprecated_amd.training import FusedTrainStep
    y = torch.zeros(a.batch, device=dev)
    t = FusedTrainStep(m, a.batch, use_graph=False)
    for _ in range(a.iters):
        t.step(xi, xv, y)
else:
    with torch.no_grad():
        for _ in range(a.iters):
            if a.batches > 1:
                m._sync_inference(dev)  # the tables' serving copy, as bench.py
                m._sync_engine(dev).forward_batches(data, outs)
            else:
                m(xi, xv)
torch.cuda.synchronize()
# fwd32_kernel's 32-sample workgroups: batch sets of the deep model unless r32=0 (r32=1 forces them)
rows = 32 if (diag_get("r32") == "1" or (a.batches > 1 and not a.fwfm and not a.train and diag_get("r32") != "0")) else 16
grid = a.batches * ((a.batch + rows - 1) // rows)
buf = (ctypes.c_uint64 * (grid * 16))()
n = _lib.lib().dfwfm_diag_stamps(m._engine.handle, buf, grid * 16,
                                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
st = np.frombuffer(buf, dtype=np.uint64).reshape(grid, 16)[:n].astype(np.int64)
names = ["stage (params, Xi/Xv)", "gather E + table first order", "shallow (fwlw, FwFM MFMA, sums)",
         "  . fwlw first order", "  . FwFM MFMA (wave 0)", "  . barrier wait", "  . first/second sums",
         "    . sums code (wave 0)", "    . sums end -> MLP start",
         "MLP layer 1", "  . K loop (wave 0)", "  . epilogue (wave 0)", "  . barrier wait", "MLP layer 2",
         "MLP layer 3", "deep reduce + combine"]
slots = [(0, 1), (1, 2), (2, 3), (2, 9), (9, 10), (10, 11), (11, 3), (11, 7), (7, 3), (3, 4), (3, 12), (12, 13),
         (13, 4), (4, 5), (5, 6), (6, 8)]
if int(diag_get("ft", "0")) & 1:  # ftrain_kernel: each wave's HW_ID in slot `wave`
    for w in range(min(4, n)):
        print(f"workgroup {w}: wave -> SIMD", [int((st[w, k] >> 4) & 3) for k in range(12)],
              "CU", [int((st[w, k] >> 8) & 15) for k in range(12)])
    sys.exit(0)
rt0, rt1 = st[:, 14], st[:, 15] & ((1 << 48) - 1)
life = (rt1 - rt0) / 100.0
span = (rt1.max() - rt0.min()) / 100.0
ev = np.concatenate([np.stack([rt0, np.ones_like(rt0)], 1), np.stack([rt1, -np.ones_like(rt1)], 1)])
ev = ev[np.argsort(ev[:, 0], kind="stable")]
conc = np.cumsum(ev[:, 1])
dt = np.diff(ev[:, 0])
mean_conc = float((conc[:-1] * dt).sum() / max(dt.sum(), 1))
print(f"launch span {span:.1f} us on the 100 MHz clock; workgroup lifetime median {np.median(life):.2f} us "
      f"(p10 {np.percentile(life, 10):.2f}, p90 {np.percentile(life, 90):.2f}); workgroups resident: mean "
      f"{mean_conc:.0f}, max {conc.max()}; first 10 % of workgroups start within "
      f"{(np.percentile(rt0, 10) - rt0.min()) / 100:.1f} us, last end - last start {(rt1.max() - rt0.max()) / 100:.1f} us")
tot = st[:, 8] - st[:, 0]
print(f"workgroups {n}; total cycles median {np.median(tot):.0f} (p10 {np.percentile(tot, 10):.0f}, "
      f"p90 {np.percentile(tot, 90):.0f})")
if a.fwfm:  # no MLP: stage, gather, shallow phases, then the combine (slot 8)
    names = ["stage (params, Xi/Xv)", "gather E + table first order", "shallow + combine",
             "  . fwlw first order", "  . FwFM MFMA (wave 0)", "  . barrier wait", "  . sums (wave 0)",
             "  . barrier + logits out"]
    slots = [(0, 1), (1, 2), (2, 8), (2, 9), (9, 10), (10, 11), (11, 7), (7, 8)]
elif a.train and diag_get("ftrain", "1") != "0":  # ftrain_kernel: helper waves beside the MLP
    names = ["stage (params, Xi/Xv)", "gather E (+ X_0) to LDS", "  helpers W0: FwFM pieces", "  helpers W0: fwlw, E / X_0",
             "  helpers W1: sums, fo save, X_1", "  helpers W2: X_2", "MLP layer 1", "  . K loop (wave 0)",
             "  . epilogue (wave 0)", "  . barriers, split tile", "MLP layer 2", "MLP layer 3", "combine"]
    slots = [(0, 1), (1, 2), (2, 10), (10, 9), (4, 11), (5, 7), (3, 4), (3, 12), (12, 13), (13, 4), (4, 5), (5, 6),
             (6, 8)]
elif rows == 32:  # fwd32 has no slot 7
    names = names[:7] + names[9:]
    slots = slots[:7] + slots[9:]
for nm, sl in zip(names, slots):
    if sl is None:
        continue
    d = st[:, sl[1]] - st[:, sl[0]]
    print(f"  {nm:34s} median {np.median(d):8.0f} cycles  ({100 * np.median(d) / np.median(tot):5.1f} %)")
