"""Per-kernel HBM traffic from rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; counter_collection.csv).

FETCH_SIZE is doubled (MI355X_MICROARCH.md §HBM: on gfx950 it reports half the bytes of wide coalesced
reads); both are KiB in rocprofv3's derived-counter units. The doubling is calibrated only for wide coalesced
reads, so an optional third pass counts the L2's memory-side read requests by size (TCC_EA0_RDREQ_32B / _64B /
_128B and all of them, TCC_EA0_RDREQ): each kernel's reads are then also given as 32·n32 + 64·n64 + 128·n128
bytes ("sized_fetch_bytes"), and the per-step total uses those (the random gathers of the walkers and hash probes
issue 32- and 64-B requests, which FETCH_SIZE × 2 overstates). Output: {kernel: {launches, fetch_bytes,
write_bytes[, sized_fetch_bytes, req32, req64, req128, req_all]}} per launch, and the per-step sum over the
decision pipeline's kernels.

    python scripts/pmc_summary.py <fetch_dir> <write_dir> <out.json> [<reqsize_dir>]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# every decision-pipeline kernel (k_*) except one-off state setup / readout; steps = launches of the batch's finish kernel
NOT_PIPELINE = ("k_init_state", "k_local_init", "k_ptable_clear", "k_psclear", "k_psread", "k_snapshot", "k_cp_clear",
                "k_local_metrics", "k_hot_sync")
FINISH = ("k_finish", "k_local_finish", "k_pfinish", "k_psfinish", "k_pace_finish", "k_cp_finish_batch")


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].split("<")[0].strip().split("::")[-1]
            per[name].append(float(r["Counter_Value"]) * 1024.0)
    return per


def load_raw(d, counter):
    """Raw counter values (not KiB) per kernel launch."""
    return {k: [v / 1024.0 for v in vals] for k, vals in load(d, counter).items()}


def mean(xs):
    return sum(xs) / max(1, len(xs))


def main(fetch_dir, write_dir, out, size_dir=None):
    f = load(fetch_dir, "FETCH_SIZE")
    w = load(write_dir, "WRITE_SIZE")
    sized = {}
    if size_dir:
        for c, key in (("TCC_EA0_RDREQ_32B_sum", "req32"), ("TCC_EA0_RDREQ_64B_sum", "req64"),
                       ("TCC_EA0_RDREQ_128B_sum", "req128"), ("TCC_EA0_RDREQ_sum", "req_all")):
            for k, vals in load_raw(size_dir, c).items():
                sized.setdefault(k, {})[key] = mean(vals)
    res = {}
    for k in sorted(set(f) | set(w)):
        fb = 2.0 * sum(f.get(k, [])) / max(1, len(f.get(k, [])))
        wb = sum(w.get(k, [])) / max(1, len(w.get(k, [])))
        res[k] = {"launches": max(len(f.get(k, [])), len(w.get(k, []))), "fetch_bytes": fb, "write_bytes": wb}
        if k in sized and {"req32", "req64", "req128"} <= set(sized[k]):
            z = sized[k]
            res[k].update(z)
            res[k]["sized_fetch_bytes"] = 32.0 * z["req32"] + 64.0 * z["req64"] + 128.0 * z["req128"]
    # per step: every pipeline kernel's per-launch traffic × launches per step (launch counts / steps)
    steps = None
    for k in FINISH:
        if k in res:
            steps = res[k]["launches"]
    step_bytes = step_doubled = 0.0
    if steps:
        for k, v in res.items():
            if k.startswith("k_") and k not in NOT_PIPELINE:
                per = v["launches"] / steps
                step_doubled += (v["fetch_bytes"] + v["write_bytes"]) * per
                step_bytes += (v.get("sized_fetch_bytes", v["fetch_bytes"]) + v["write_bytes"]) * per
    note = "FETCH_SIZE x2 (gfx950 correction), KiB→bytes"
    if sized:
        note = ("reads = 32·TCC_EA0_RDREQ_32B + 64·_64B + 128·_128B per kernel (request-size pass); "
                "pipeline_bytes_per_step_fetch_x2 keeps the FETCH_SIZE x2 figure; writes = WRITE_SIZE")
    json.dump({"kernels": res, "pipeline_bytes_per_step": step_bytes, "pipeline_bytes_per_step_fetch_x2": step_doubled,
               "steps_seen": steps, "note": note}, open(out, "w"), indent=1)
    print(json.dumps({"pipeline_bytes_per_step": step_bytes, "fetch_x2": step_doubled, "steps_seen": steps}))


if __name__ == "__main__":
    main(*sys.argv[1:5])
