"""Per-kernel SQ counters from rocprofv3 --pmc passes (counter_collection.csv), per-launch means, with the shares
of wave time spent issuing (SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES) and waiting (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES),
and VALU instructions per decided record when the records per launch are given.

    python scripts/sq_summary.py <out.json> <records_per_launch or 0> <pass_dir> [<pass_dir> ...]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(out, records, dirs):
    per = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"].split("(")[0].strip().split("::")[-1]
                per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        if wc:
            m["issue_share"] = m.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
            m["wait_share"] = m.get("SQ_WAIT_INST_ANY", 0.0) / wc
        if records and "SQ_INSTS_VALU" in m:
            m["valu_wave_insts_per_record"] = m["SQ_INSTS_VALU"] / records
        res[k] = m
    json.dump({"note": "rocprofv3 --pmc SQ counters, per-launch means; issue/wait shares of SQ_WAVE_CYCLES",
               "records_per_launch": records, "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), sys.argv[3:])
