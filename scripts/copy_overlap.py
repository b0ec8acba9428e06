"""Copy-engine timeline of the end-to-end host path (bench.py end_to_end) from a rocprofv3
--memory-copy-trace --kernel-trace run: H2D copies (SDMA, memory_copy_trace) and D2H copies of the results (ROCclr
blit kernels `__amd_rocclr_copyBuffer`, kernel_trace), each direction's busy time and rate, and how much of the
D2H time overlaps an H2D copy (full duplex on the link).

    python scripts/copy_overlap.py <rocprof_dir> <h2d_bytes> <d2h_bytes> [out.json]
"""
import csv
import glob
import json
import os
import sys


def main(d, h2d_bytes, d2h_bytes, out=None):
    h2d_bytes, d2h_bytes = int(h2d_bytes), int(d2h_bytes)
    mc = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)[0]
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    h = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(mc))
         if r["Direction"].endswith("HOST_TO_DEVICE")]
    k = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(kt))
         if "copyBuffer" in r["Kernel_Name"]]
    # the batches' copies: the largest ones (setup copies are small)
    h = [x for x in h if x[1] - x[0] > 0.5 * max(e - s for s, e in h)]
    k = [x for x in k if x[1] - x[0] > 0.5 * max(e - s for s, e in k)]
    ov = sum(max(0, min(a[1], b[1]) - max(a[0], b[0])) for a in h for b in k)
    hb, kb = sum(e - s for s, e in h), sum(e - s for s, e in k)
    res = {"h2d_copies": len(h), "d2h_copies": len(k), "h2d_busy_ms": hb / 1e6, "d2h_busy_ms": kb / 1e6,
           "h2d_GBps_while_busy": len(h) * h2d_bytes / hb, "d2h_GBps_while_busy": len(k) * d2h_bytes / kb,
           "d2h_time_overlapping_h2d_ms": ov / 1e6, "d2h_overlap_fraction": ov / kb,
           "window_ms": (max(e for _, e in h + k) - min(s for s, _ in h + k)) / 1e6}
    print(json.dumps(res))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:5])
