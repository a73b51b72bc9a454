"""Summarise rocprofv3 --pmc passes for the forward kernel into profiles/pmc_traffic.json.

traffic (HBM/fabric bytes per launch) = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes): gfx950's
FETCH_SIZE counts 64 B per 128-B request of a wide (16 B/lane) read, so it is doubled
(MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for wide stores.  FETCH_SIZE counts
every L2 miss, Infinity-Cache hits included.
"""
import csv
import glob
import json
import os
import statistics as st
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
root = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
vals = {}
durs = []
for path in glob.glob(os.path.join(root, f"pmc_{tag}_*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        if "fwd_kernel" not in r["Kernel_Name"]:
            continue
        vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
med = {k: st.median(v) for k, v in vals.items()}
out = {"kernel": "dfwfm::fwd_kernel<10,6,1,false>", "counters_median_per_dispatch": med,
       "profiled_duration_us_median": st.median(durs) / 1e3 if durs else None}
if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
    out["hbm_bytes_per_launch"] = int(2 * med["FETCH_SIZE"] * 1024 + med["WRITE_SIZE"] * 1024)
    out["traffic_formula"] = "2*FETCH_SIZE + WRITE_SIZE (KB); FETCH doubled per the gfx950 calibration"
if "SQ_VALU_MFMA_BUSY_CYCLES" in med and "GRBM_GUI_ACTIVE" in med:
    out["mfma_util_pct"] = 100 * med["SQ_VALU_MFMA_BUSY_CYCLES"] / (med["GRBM_GUI_ACTIVE"] / 8 * 1024)
if "TCC_HIT_sum" in med and "TCC_MISS_sum" in med:
    out["l2_hit_pct"] = 100 * med["TCC_HIT_sum"] / (med["TCC_HIT_sum"] + med["TCC_MISS_sum"])
print(json.dumps(out, indent=1))
