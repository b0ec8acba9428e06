"""Short-walker timers (SG_DEBUG & 64) on the C3 bench workload: one batch, then per length class the
number of wave groups and the average gather / walk time per group (s_memrealtime, 100 MHz)."""
import os, sys
os.environ["SG_DEBUG"] = str(int(os.environ.get("SG_DEBUG", "0")) | 64 | 2)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import bench
from sentinel_amd import abi
from sentinel_amd.engine import FlowEngine
dev = torch.device("cuda", 0)
n = 16_000_000
wl = bench.ShardWorkload(1_000_000, n, 0, 1, dev)
eng = FlowEngine(device=0, max_batch=n)
ns = np.zeros(1, abi.NS_DTYPE); ns["connected_count"] = 1; ns["max_allowed_qps"] = 30000
eng.set_namespaces(ns); eng.load_rules(wl.rules)
out = torch.empty(n * 12, dtype=torch.uint8, device=dev)
for b in range(2):
    x = wl.batch(b)
    torch.cuda.synchronize()
    eng.decide_device(x.data_ptr(), n, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
c = eng.debug_copy(5, np.uint64, 32).astype(np.uint64)
print(f"total group time {int(c[0]) / 100:.0f} us (summed over waves)")
for cl in range(6):
    g = int(c[1 + cl])
    if not g:
        continue
    gat, wk = int(c[7 + cl]) & 0xFFFFFFFF, int(c[7 + cl]) >> 32
    print(f"class {cl}: groups {g:7d}  gather {gat / g / 100:7.2f} us/group  walk {wk / g / 100:8.2f} us/group")
print(f"all groups: outer trips {int(c[13])}, max-lane records (sum over groups) {int(c[14])}, records {int(c[15])}")
