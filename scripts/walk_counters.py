"""Short-walker cycle counters (SG_DEBUG & 64) on the C3 bench workload: one batch, then the counters."""
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
c = eng.debug_copy(5, np.uint64, 16).astype(np.int64)
g = max(1, c[0])
print(f"groups {c[0]}  scan cyc/group {c[1]/g:.0f}  walk cyc/group {c[2]/g:.0f}  periods opened/lane {c[3]/g/64:.2f}  "
      f"records/lane {c[4]/g/64:.2f}  max len/group {c[5]/g:.1f}")
print("cycles per class (sum over groups):", list(c[6:12]))
