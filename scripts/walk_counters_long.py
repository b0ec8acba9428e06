"""Long-walker timers (SG_DEBUG & 64): per segment length bucket, segments and
average wave time per segment (s_memrealtime, 100 MHz). The short walker's timers are zeroed first by running
it with no short segments... (both walkers share dbg_ctr: run with SG_SHORT_MAX small and read [1..8])."""
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
eng = FlowEngine(device=0, max_batch=n, flags=int(os.environ.get("SG_FLAGS", "0")))
ns = np.zeros(1, abi.NS_DTYPE); ns["connected_count"] = 1; ns["max_allowed_qps"] = 30000
eng.set_namespaces(ns); eng.load_rules(wl.rules)
out = torch.empty(n * 12, dtype=torch.uint8, device=dev)
for b in range(2):
    x = wl.batch(b)
    torch.cuda.synchronize()
    eng.decide_device(x.data_ptr(), n, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
c = eng.debug_copy(5, np.uint64, 32).astype(np.uint64)
for i, name in enumerate(["<=64", "<=256", "<=1024", ">1024"]):
    cnt, t, mx = int(c[16 + 2 * i]), int(c[17 + 2 * i]), int(c[24 + i])
    if cnt:
        print(f"long segments {name:7s}: {cnt:7d}  {t / cnt / 100:8.2f} us/segment  max {mx / 100:8.2f} us")
