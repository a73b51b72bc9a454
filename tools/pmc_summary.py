"""Summarise rocprofv3 --pmc passes (tools/pmc.sh over bench.py's own command) per forward-kernel name into
entries of profiles/pmc_traffic.json keyed by (kernel, workload) -- bench.py reads `traffic` from the entry of the
kernel AND workload it runs, nothing else.

traffic (HBM/fabric bytes per launch) = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes): gfx950's FETCH_SIZE counts
64 B per 128-B request of a wide (16 B/lane) read, so it is doubled (MI355X_MICROARCH.md, HBM section); WRITE_SIZE
is exact for wide stores.  FETCH_SIZE counts every L2 miss, Infinity-Cache hits included.  MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE x 1024 SIMDs / 8 XCDs (GRBM counts per XCD).

    python tools/pmc_summary.py TAG [root] [pmc_traffic.json] ["bench args"]
"""
import csv
import glob
import json
import os
import shlex
import statistics as st
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r03"
root = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
dst = sys.argv[3] if len(sys.argv) > 3 else None
bench_args = sys.argv[4] if len(sys.argv) > 4 else ""


def workload_of(args):
    """bench.py's workload_id for these arguments: config/first_order/scaleK/inputs."""
    a = shlex.split(args)

    def opt(name, default):
        return a[a.index(name) + 1] if name in a else default
    m = int(opt('--batch-set', '32'))
    packed = opt('--pack-tables', '1') != '0' and opt('--config', 'deepfwfm') != 'qr'  # the tables' serving copy
    return f"{opt('--config', 'deepfwfm')}/{opt('--first-order', 'lw')}/scale{opt('--table-scale', '1')}/" \
           f"{opt('--inputs', 'uniform')}" + ("/set" if m > 1 else "") + ("/packed" if packed else "")


def batches_per_launch(args):
    """bench.py's batches per forward launch under tools/pmc.sh (64 steps, 64 warmup, two streams)."""
    a = shlex.split(args)
    return int(a[a.index('--batch-set') + 1]) if '--batch-set' in a else 32


vals, durs = {}, {}
for path in glob.glob(os.path.join(root, f"pmc_{tag}_*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if not any(n in k for n in ("fwd_kernel", "fwd32_kernel")):
            continue
        k = k.replace("void ", "").replace(" ", "").split("(")[0]  # bench.py's kernel_name form
        vals.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        durs.setdefault(k, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
wl = workload_of(bench_args)
entries = []
fewest = min((len(d) for d in durs.values()), default=0)
for k, v in vals.items():
    med = {c: st.median(x) for c, x in v.items()}
    # a set run's per-call leg (one batch per launch, thousands of dispatches; tools/pmc.sh now passes
    # --no-per-call) is its own workload
    is_set = "/set" in wl
    kwl = wl.replace("/set", "/call") if is_set and len(durs[k]) > 10 * fewest else wl
    e = {"kernel": k, "workload": kwl, "bench_args": bench_args, "tag": tag,
         "counters_median_per_dispatch": med, "profiled_duration_us_median": st.median(durs[k]) / 1e3,
         "dispatches": len(durs[k])}
    if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
        e["hbm_bytes_per_launch"] = int(2 * med["FETCH_SIZE"] * 1024 + med["WRITE_SIZE"] * 1024)
        if "/set" in kwl:  # a launch is a set of M batches: bench.py scales the per-batch bytes to its sets
            e["batches_per_launch"] = batches_per_launch(bench_args)
            e["hbm_bytes_per_batch"] = e["hbm_bytes_per_launch"] // e["batches_per_launch"]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in med and "GRBM_GUI_ACTIVE" in med:
        e["mfma_busy_frac"] = med["SQ_VALU_MFMA_BUSY_CYCLES"] / (med["GRBM_GUI_ACTIVE"] / 8 * 1024)
    entries.append(e)
print(json.dumps(entries, indent=1))
if dst:
    try:
        d = json.load(open(dst))
    except Exception:
        d = {}
    keep = [e for e in d.get("entries", []) if (e["kernel"], e["workload"]) not in
            {(n["kernel"], n["workload"]) for n in entries}]
    d = {"source": "tools/pmc.sh (rocprofv3 --pmc over bench.py's own command, one counter group per pass; the "
                   "profiler serialises the counted dispatches) + tools/pmc_summary.py",
         "traffic_formula": "2*FETCH_SIZE + WRITE_SIZE (KB); FETCH doubled per the gfx950 calibration",
         "entries": keep + entries}
    open(dst, "w").write(json.dumps(d, indent=1) + "\n")
