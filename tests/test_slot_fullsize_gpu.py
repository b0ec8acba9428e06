"""The whole slot chain at full size in the driver's GPU suite: `bench_configs.py --workload slot`'s trace — 1M
resources with C5's breakers, 10 % of them carrying an origin-limitApp rule, a WarmUp rule or a ParamFlowRule (the
lane and wave cx walkers' work queues, dead chunks, writer-lane hand-off on hot segments of ~200k records), 16M
entries per 1000 ms batch plus the exits of the passed ones from the oracle's client model — decided by
sg_slot_decide_batch; every result of both batches must equal the oracle's sequential replay (slot() raises on the
first difference). The second batch carries the first one's state: open windows, breakers, param token buckets,
origin nodes created a batch earlier."""
import types

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_slot_chain_full_size_equals_oracle():
    import torch

    import bench_configs
    args = types.SimpleNamespace(resources=1_000_000, events=16_000_000, warmup=0, steps=2)
    r = bench_configs.slot(args, torch.device("cuda", 0))
    assert r["extra"]["parity"] == "every batch equal to the oracle"
    assert r["extra"]["cx_among_hottest_1000"] > 0      # hot cx segments: the wave walker's long work items
    assert r["n"] > 16_000_000                          # entries and exits
