"""Timeline of the last C3 step from a rocprofv3 kernel trace: kernel, start and end relative to the step's first
kernel (us)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if "sg::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# steps start at k_prep
starts = [i for i, r in enumerate(rows) if "k_prep" in r["Kernel_Name"]]
step = rows[starts[-2]:starts[-1]]
t0 = int(step[0]["Start_Timestamp"])
for r in step:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sg::", "")
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{n:28s} {s:8.1f} {e:8.1f} {e - s:8.1f}")
