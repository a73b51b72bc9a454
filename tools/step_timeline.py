"""One training step's kernel timeline from a rocprofv3 kernel trace (between two forward launches):
    python tools/step_timeline.py gpurun_out/<tag>_proftrainx/run_kernel_trace.csv [k-th last step]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("void dfwfm::fwd_kernel")]
i0, i1 = starts[-k], starts[-k + 1]
t0 = int(rows[i0]["Start_Timestamp"])
busy_end = 0.0
idle = 0.0
for r in rows[i0:i1 + 1]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    if r is not rows[i1] and s > busy_end:
        idle += s - busy_end
    busy_end = max(busy_end, e)
    print("%8.1f %8.1f %7.1f q%s %s" % (s, e, e - s, r["Queue_Id"], r["Kernel_Name"][:64]))
print("step %.1f us, GPU idle %.1f us" % ((int(rows[i1]["Start_Timestamp"]) - t0) / 1e3, idle))
