"""Timeline of the sg:: kernels in a rocprofv3 kernel_trace.csv: the last N batch pipelines (a batch starts at
k_prep), each kernel's start / end relative to the first k_prep shown, in µs, to see what overlaps.

    python scripts/timeline.py gpurun_out/prof/<...>_kernel_trace.csv [N]
"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "sg::" in r["Kernel_Name"] or r["Kernel_Name"].startswith(("k_", "void k_"))]
n_show = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
preps = [i for i, r in enumerate(rows) if "k_prep" in r["Kernel_Name"]]
if len(preps) > n_show + 1:
    rows = rows[preps[-n_show - 1]:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sg::", "")
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{name:32s} {s / 1e3:9.1f} {e / 1e3:9.1f}  ({(e - s) / 1e3:7.1f})")
