"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) per forward-kernel variant into a JSON file.

traffic (HBM/fabric bytes per launch) = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes): gfx950's
FETCH_SIZE counts 64 B per 128-B request of a wide (16 B/lane) read, so it is doubled
(MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for wide stores.  FETCH_SIZE counts
every L2 miss, Infinity-Cache hits included.  MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES over
GRBM_GUI_ACTIVE x 1024 SIMDs / 8 XCDs (GRBM counts per XCD).

    python tools/pmc_summary.py TAG [root] [out.json]
"""
import csv
import glob
import json
import os
import statistics as st
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
root = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
dst = sys.argv[3] if len(sys.argv) > 3 else None
vals, durs = {}, {}
for path in glob.glob(os.path.join(root, f"pmc_{tag}_*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "fwd_kernel" not in k:
            continue
        # bench.py's kernel_name form: "dfwfm::fwd_kernel<10,3,1,false,0,8,25>"
        k = k.replace("void ", "").replace(" ", "").split("(")[0]
        vals.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        durs.setdefault(k, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {}
for k, v in vals.items():
    med = {c: st.median(x) for c, x in v.items()}
    e = {"counters_median_per_dispatch": med, "profiled_duration_us_median": st.median(durs[k]) / 1e3}
    if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
        e["hbm_bytes_per_launch"] = int(2 * med["FETCH_SIZE"] * 1024 + med["WRITE_SIZE"] * 1024)
        e["traffic_formula"] = "2*FETCH_SIZE + WRITE_SIZE (KB); FETCH doubled per the gfx950 calibration"
    if "SQ_VALU_MFMA_BUSY_CYCLES" in med and "GRBM_GUI_ACTIVE" in med:
        e["mfma_busy_frac"] = med["SQ_VALU_MFMA_BUSY_CYCLES"] / (med["GRBM_GUI_ACTIVE"] / 8 * 1024)
    out[k] = e
s = json.dumps({"source": f"tools/pmc.sh (tag {tag}): eager, one stream, rocprofv3 --pmc, one counter group per pass",
                "kernels": out}, indent=1)
print(s)
if dst:
    open(dst, "w").write(s + "\n")
