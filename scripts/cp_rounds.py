"""Per-launch durations of the cparam walkers / combine in a rocprofv3 kernel trace (last batch): which rounds cost what.
    python scripts/cp_rounds.py gpurun_out/cp_prof/cp_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
keep = ("k_cp_", "k_radix", "k_seg", "k_colsum", "k_chunkscan", "k_rescan", "k_lim")
rows = [r for r in rows if any(k in r["Kernel_Name"] for k in keep)]
starts = [i for i, r in enumerate(rows) if "k_cp_recinit" in r["Kernel_Name"]]
rows = rows[starts[-1]:] if starts else rows
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sg::", "")
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{name:28s} {s / 1e3:9.1f} {e / 1e3:9.1f}  ({(e - s) / 1e3:8.1f})")
