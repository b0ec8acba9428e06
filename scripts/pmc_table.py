"""Per-kernel mean of every collected counter over the rocprofv3 --pmc passes in a directory."""
import csv, glob, sys, collections
root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    if not k.startswith("sg::"):
        continue
    vals = {c: sum(v) / len(v) for c, v in acc[k].items()}
    print(k, {c: f"{v:.4g}" for c, v in sorted(vals.items())})
