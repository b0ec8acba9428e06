"""Bisect a parity failure: run one trace through the oracle and through each walker mode."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle.binding import ClusterTokenService
from sentinel_amd import abi
from sentinel_amd.engine import FlowEngine
from tests.test_flow_gpu import _rules, _trace, _ns

def run(n_keys, n, zipf, prio, S, interval, flags, batches=3):
    rng = np.random.default_rng(n_keys * 1000 + n + S)
    rules = _rules(n_keys, rng, S=S, interval=interval)
    eng = FlowEngine(max_batch=1 << 20, flags=flags); eng.set_namespaces(_ns()); eng.load_rules(rules)
    ora = ClusterTokenService(); ora.set_namespaces(_ns()); ora.load_rules(rules)
    t = 1_700_000_000_017
    for b in range(batches):
        span = int(rng.integers(1, 3 * interval))
        req = _trace(rng, n, n_keys, t, span, zipf=zipf, prio=prio)
        t = int(req["ts_ms"][-1]) + int(rng.integers(0, 2 * interval))
        o, g = ora.decide(req), eng.decide_host(req)
        bad = np.nonzero(o != g)[0]
        if len(bad):
            keys = req["key"] & abi.KEY_INDEX
            print(f"  flags={flags} batch={b} span={span}: {len(bad)} differ; by key:",
                  {int(k): int((keys[bad] == k).sum()) for k in np.unique(keys[bad])})
            for i in bad[:3]:
                k = keys[i]
                same = np.nonzero(keys[:i + 1] == k)[0]
                print(f"    i={i} req={req[i]} ora={o[i]} gpu={g[i]} (#{len(same)-1} of key {k}, thr={rules['count'][k]})")
            return False
    print(f"  flags={flags}: all {batches} batches match")
    return True

for case in [(7, 20_000, 1.2, 0.05, 5, 1000), (100, 50_000, 1.0, 0.01, 10, 1000), (2, 3000, 1.0, 0.0, 10, 1000)]:
    print("case", case)
    for flags in (0, abi.FLAG_SERIAL_ONLY, abi.FLAG_WAVE_ONLY):
        run(*case, flags)

print("intermediates check")
rng = np.random.default_rng(7 * 1000 + 20000 + 5)
rules = _rules(7, rng, S=5, interval=1000)
eng = FlowEngine(max_batch=1 << 20); eng.set_namespaces(_ns()); eng.load_rules(rules)
span = int(rng.integers(1, 3000))
req = _trace(rng, 20000, 7, 1_700_000_000_017, span, zipf=1.2, prio=0.05)
eng.decide_host(req)
n = len(req)
rec = eng.debug_copy(0, np.uint64, n); srt = eng.debug_copy(1, np.uint64, n)
bnd = eng.debug_copy(2, np.uint32, 8 * 65536).reshape(8, 65536); p0 = eng.debug_copy(3, np.int64, 8); npp = eng.debug_copy(4, np.uint32, 8)
kshift, abits = 61, 41
keys = (req["key"] & abi.KEY_INDEX).astype(np.uint64)
print(" rec key field ok:", np.array_equal(rec >> np.uint64(kshift), keys))
print(" rec idx field ok:", np.array_equal((rec >> np.uint64(abits)) & np.uint64((1 << 20) - 1), np.arange(n, dtype=np.uint64)))
want = rec[np.argsort(rec >> np.uint64(kshift), kind="stable")]
print(" sorted ok:", np.array_equal(srt, want), "first diff:", np.nonzero(srt != want)[0][:5])
P = req["ts_ms"] // 200
print(" p0:", p0[0], "want", P[0], " np:", npp[0], "want", P[-1] - P[0] + 1)
wb = [int(np.searchsorted(P, P[0] + q)) for q in range(int(P[-1] - P[0] + 1))]
print(" bnd:", list(bnd[0][:len(wb)]), "\n want", wb)
