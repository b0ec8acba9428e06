"""The sharded local chain on the device: G handles of one GPU standing for G GPUs of a node, each loaded with the
node's rules and fed the events of the resources sg_local_owners gives it (key groups co-located), decide every
event as one sequential replay of the node trace does; the rows of sg_local_metrics_raw merged over the handles
(sentinel_amd/cluster.py merge_metric_rows, the LocalMetricRollup's merge) equal the single chain's metrics.log rows,
Constants.ENTRY_NODE included; sg_local_owners equals the Python restatement (cluster.local_owners)."""
import numpy as np
import pytest

from sentinel_amd import abi
from sentinel_amd.cluster import ENTRY_NODE_RESOURCE, local_owners, merge_metric_rows, split_local_events
from tests.test_local_shard import N_ORIGINS, N_RES, node_setup, node_trace

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("device_rows", ["host", "device", "enqueue", "enqueue_worst"])
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_local_chain_handles_equal_node_replay(world, device_rows):
    """device_rows: sg_local_metrics_raw_device into HBM (or sg_local_metrics_raw_enqueue, ordered on a stream, first
    with a buffer too small: no rows, no side effect; enqueue_worst: a buffer for every possible row, no counting pass)
    and the device rollup's merge (DeviceLocalMetricRollup)."""
    import torch

    from sentinel_amd.cluster import DeviceLocalMetricRollup
    from sentinel_amd.engine import FlowEngine
    base, frules, relate, inbound = node_setup()
    trace = node_trace(base, frules, inbound)
    engs = []
    for _ in range(world):
        e = FlowEngine(device=0, max_batch=1 << 16)
        e.local_load_rules(base, 2, 1000, 500)
        e.local_load_flow_rules(frules, N_ORIGINS, 0)
        e.local_set_entry_types(inbound)
        engs.append(e)
    owners = engs[0].local_owners(world)
    assert np.array_equal(owners.astype(np.int64), local_owners(N_RES, relate, world))
    for e in engs[1:]:
        assert np.array_equal(e.local_owners(world), owners)
    saw_entry = False
    for b, (ev, want, now, rows_want) in enumerate(trace):
        parts = split_local_events(ev, owners, world)
        for r in range(world):
            got = engs[r].local_decide_host(ev[parts[r]])
            assert np.array_equal(got, want[parts[r]]), f"batch {b} shard {r}: {(got != want[parts[r]]).sum()} differ"
        if device_rows == "enqueue_worst":
            st = torch.cuda.current_stream().cuda_stream
            bufs = [torch.empty((59 * N_RES + 60, 8), dtype=torch.int64, device="cuda") for _ in engs]
            cnts = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in engs]
            for e, buf, c in zip(engs, bufs, cnts):
                e.local_metrics_raw_enqueue(now, buf, c, st)
            got_rows = [buf[:int(c.item())] for buf, c in zip(bufs, cnts)]
            m = DeviceLocalMetricRollup.merge(torch.cat(got_rows))
            rows = m.cpu().numpy().copy().view(abi.METRIC_NODE_DTYPE).reshape(-1)
        elif device_rows == "enqueue":
            st = torch.cuda.current_stream().cuda_stream
            bufs = [torch.empty((4 * N_RES + 64, 8), dtype=torch.int64, device="cuda") for _ in engs]
            cnts = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in engs]
            tiny = torch.empty((1, 8), dtype=torch.int64, device="cuda")
            for e, c in zip(engs, cnts):
                e.local_metrics_raw_enqueue(now, tiny, c, st)   # too small: only the count
            need = [int(c.item()) for c in cnts]
            for e, buf, c in zip(engs, bufs, cnts):
                e.local_metrics_raw_enqueue(now, buf, c, st)
            assert [int(c.item()) for c in cnts] == need
            got_rows = [buf[:int(c.item())] for buf, c in zip(bufs, cnts)]
            m = DeviceLocalMetricRollup.merge(torch.cat(got_rows))
            rows = m.cpu().numpy().copy().view(abi.METRIC_NODE_DTYPE).reshape(-1)
        elif device_rows == "device":
            bufs = [torch.empty((4 * N_RES + 64, 8), dtype=torch.int64, device="cuda") for _ in engs]
            got_rows = [buf[:e.local_metrics_raw_device(now, buf)] for e, buf in zip(engs, bufs)]
            m = DeviceLocalMetricRollup.merge(torch.cat(got_rows))
            rows = m.cpu().numpy().copy().view(abi.METRIC_NODE_DTYPE).reshape(-1)
        else:
            rows = merge_metric_rows([e.local_metrics_raw(now) for e in engs])
        assert np.array_equal(rows, rows_want), f"batch {b}: metric rows differ"
        saw_entry |= bool((rows_want["resource"] == ENTRY_NODE_RESOURCE).any())
    assert saw_entry


def test_local_owners_contract():
    from sentinel_amd.engine import EngineError, FlowEngine
    base, frules, relate, inbound = node_setup()
    e = FlowEngine(device=0, max_batch=1 << 12)
    with pytest.raises(EngineError):  # before sg_local_load_rules
        e._check(e._L.sg_local_owners(e.h, 2, None, 0))
    e.local_load_rules(base, 2, 1000, 500)
    e.local_load_flow_rules(frules, N_ORIGINS, 0)
    assert (e.local_owners(1) == 0).all()
    with pytest.raises(EngineError):
        e._check(e._L.sg_local_owners(e.h, 0, None, 0))
