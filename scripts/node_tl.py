"""Timeline of the last `ms` milliseconds of a rocprofv3 kernel_trace.csv: every kernel's start / end (µs, relative
to the window), duration and the queue / stream it ran on — to see how same-device node shards interleave.

    python scripts/node_tl.py <kernel_trace.csv> [ms]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ms = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t_end = max(int(r["End_Timestamp"]) for r in rows)
rows = [r for r in rows if int(r["Start_Timestamp"]) >= t_end - ms * 1e6]
t0 = int(rows[0]["Start_Timestamp"])
qk = "Queue_Id" if "Queue_Id" in rows[0] else None
sk = "Stream_Id" if "Stream_Id" in rows[0] else None
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sg::", "")[:34]
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{name:34s} {s / 1e3:9.1f} {e / 1e3:9.1f} ({(e - s) / 1e3:7.1f}) q{r.get(qk, '') if qk else ''} "
          f"s{r.get(sk, '') if sk else ''} grid {r.get('Grid_Size', r.get('Grid_Size_X', ''))}")
