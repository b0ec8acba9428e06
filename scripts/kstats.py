"""Print the sg:: kernels of a rocprofv3 kernel_stats.csv: calls, average µs, total share."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    name = r["Name"]
    if "sg::" not in name:
        continue
    short = name.split("(")[0].replace("void ", "").replace("sg::", "")
    print(f"{short:28s} calls {int(r['Calls']):4d}  avg {float(r['AverageNs']) / 1e3:9.1f} us")
