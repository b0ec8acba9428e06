"""Node-level sharding and the metric rollup.

flowIds are owned by GPU `splitmix64(flowIndex) mod G`; each rank decides only its own flows' requests,
so the decision path needs no collective. The one exchange is the metric rollup that feeds
`ClusterMetricNodeGenerator`-style snapshots (srv/flow/statistic/ClusterMetricNodeGenerator.java:39-105):
per-flow {passQps, blockQps} gathered to every rank and the node totals all-reduced. With backend
"nccl" this runs over RCCL/xGMI; the same code runs over gloo on CPU in the tests.
"""
import numpy as np
import torch
import torch.distributed as dist

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser of (x + golden gamma), elementwise on uint64."""
    with np.errstate(over="ignore"):
        z = np.asarray(x, dtype=np.uint64) + _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def owner_of(flow_index: np.ndarray, world: int) -> np.ndarray:
    """GPU that owns each flow (by dense flow index)."""
    return (splitmix64(flow_index) % np.uint64(world)).astype(np.int64)


def shard_flows(n_flows: int, rank: int, world: int) -> np.ndarray:
    """Global flow indices owned by `rank`, ascending (local key i ↔ global flow shard[i])."""
    idx = np.arange(n_flows, dtype=np.uint64)
    return np.nonzero(owner_of(idx, world) == rank)[0].astype(np.int64)


def route_requests(req_keys: np.ndarray, world: int):
    """Host-side partition of a node-level request array by owning GPU (stable, keeps arrival order).
    Returns (order, counts): req_keys[order] grouped by rank, counts per rank."""
    own = owner_of(req_keys.astype(np.uint64), world)
    order = np.argsort(own, kind="stable")
    counts = np.bincount(own, minlength=world)
    return order, counts


class MetricRollup:
    """Per-step node-wide rollup of per-flow {passQps, blockQps} snapshots.

    `snap` is this rank's [K_local, 2] float64 tensor (on the rank's device for nccl, CPU for gloo).
    After `run()`, `totals` holds the node-wide Σ passQps / Σ blockQps and `gathered[r]` rank r's
    snapshot (ranks may own different numbers of flows: snapshots are padded to the largest shard).
    """

    def __init__(self, k_local: int, device, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.device = device
        sizes = torch.tensor([k_local], dtype=torch.int64, device=device)
        if self.world > 1:
            all_sizes = [torch.zeros_like(sizes) for _ in range(self.world)]
            dist.all_gather(all_sizes, sizes, group=group)
            self.sizes = [int(s.item()) for s in all_sizes]
        else:
            self.sizes = [k_local]
        self.k_max = max(self.sizes)
        self.padded = torch.zeros((self.k_max, 2), dtype=torch.float64, device=device)
        self.gathered = [torch.zeros_like(self.padded) for _ in range(self.world)]
        self.totals = torch.zeros(2, dtype=torch.float64, device=device)

    def run(self, snap: torch.Tensor):
        k = snap.shape[0]
        self.padded[:k].copy_(snap)
        torch.sum(snap, 0, out=self.totals)
        if self.world > 1:
            dist.all_reduce(self.totals, group=self.group)
            dist.all_gather(self.gathered, self.padded, group=self.group)
        else:
            self.gathered[0].copy_(self.padded)
        return self.totals

    def node_snapshot(self, shards):
        """Reassemble the node-wide [n_flows, 2] snapshot from gathered shards (shards[r] = global
        flow indices of rank r, as from shard_flows)."""
        n = sum(len(s) for s in shards)
        out = torch.zeros((n, 2), dtype=torch.float64, device=self.device)
        for r, s in enumerate(shards):
            out[torch.as_tensor(s, device=self.device)] = self.gathered[r][: len(s)]
        return out


def node_order(shard_ts):
    """The node's arrival order under the sharded limiter exchange: (ts_ms, shard rank, position in the shard's
    batch). `shard_ts[r]` = rank r's batch timestamps (time-ordered). Returns the permutation that puts the
    concatenation [rank 0's batch, rank 1's, ...] into node order (stable sort by ts)."""
    cat = np.concatenate([np.asarray(t, np.int64) for t in shard_ts]) if shard_ts else np.zeros(0, np.int64)
    return np.argsort(cat, kind="stable")


class LimiterExchange:
    """SURVEY §8(e) exchange step for the namespace QPS limiter (GlobalRequestLimiter.java:46-55): one node-wide
    window per namespace although every GPU sees only its flows' requests.

    Per node batch: all_reduce(MAX) of (-first ts, last ts) → the node's millisecond range; sg_lim_arrivals counts
    this shard's limited requests per (namespace slot, millisecond); all_gather of those counts (n_lim × n_ms × 4
    bytes per rank: 4 KB for one namespace over a 1 s batch); sg_lim_exchange arms the engine's next flow batch.
    The node's arrival order is then (ts, rank, position) — `node_order`. Collectives run on `coll_device` (the
    rank's GPU for RCCL, "cpu" for gloo)."""

    def __init__(self, engine, device, coll_device=None, group=None):
        self.eng = engine
        self.n_lim = engine.lim_slots()  # the layout [world][n_lim][n_ms] is the engine's (re-read by every arm())
        self.device = torch.device(device)
        self.coll = torch.device(coll_device) if coll_device is not None else self.device
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self._gathered = None  # kept alive until the armed batch has been decided

    def time_range(self, t_first, t_last):
        """Node-wide [t_base, t_base + n_ms) from each rank's first / last timestamp (None: empty batch)."""
        big = np.iinfo(np.int64).max
        v = torch.tensor([-(t_first if t_first is not None else big), t_last if t_last is not None else -big],
                         dtype=torch.int64, device=self.coll)
        if self.world > 1:
            dist.all_reduce(v, op=dist.ReduceOp.MAX, group=self.group)
        lo, hi = -int(v[0]), int(v[1])
        if hi < lo:
            return None
        return lo, hi - lo + 1

    def arm(self, req_ptr: int, n: int, t_first, t_last, stream_ptr: int = 0, param: bool = False):
        """Count, exchange and arm for this rank's batch (device records at req_ptr: sg_req, or sg_cparam_req with
        param=True). Every rank calls this for every node batch, with n = 0 when it has no requests; the caller
        then decides its batch (n may be 0) on any flow entry point, or sg_cparam_decide_batch for param=True."""
        self.n_lim = self.eng.lim_slots()  # set_namespaces may have changed the limiter slots since the last batch
        rng = self.time_range(t_first, t_last)
        if rng is None:
            rng = (0, 1)  # no requests anywhere: nothing to count, the windows see no tryPass
        t_base, n_ms = rng
        mine = torch.zeros(max(1, self.n_lim * n_ms), dtype=torch.int32, device=self.device)
        count = self.eng.lim_arrivals_param if param else self.eng.lim_arrivals
        count(req_ptr if n else 0, n, t_base, n_ms, mine.data_ptr(), stream_ptr, counts_words=self.n_lim * n_ms)
        if self.world > 1:
            parts = [torch.zeros_like(mine, device=self.coll) for _ in range(self.world)]
            dist.all_gather(parts, mine.to(self.coll), group=self.group)
            gathered = torch.cat(parts).to(self.device)
        else:
            gathered = mine
        self._gathered = gathered
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        self.eng.lim_exchange(gathered.data_ptr(), t_base, n_ms, gathered_words=self.world * self.n_lim * n_ms)
        return t_base, n_ms


# ---------------------------------------------------------------------------------------- the sharded local chain

ENTRY_NODE_RESOURCE = 0xFFFFFFFF


def local_group_keys(n_res: int, relate_pairs) -> np.ndarray:
    """The smallest resource of each resource's key group (union-find over RELATE references (resource, ref)): the
    resources whose decisions read each other's ClusterNode. The library's sg_local_owners computes the same groups
    from the loaded rules (plus, on an embedded token server, flowId / limited-namespace sharing)."""
    parent = np.arange(n_res, dtype=np.int64)

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for a, b in relate_pairs:
        if 0 <= a < n_res and 0 <= b < n_res:
            x, y = find(int(a)), find(int(b))
            if x != y:
                parent[max(x, y)] = min(x, y)
    return np.array([find(k) for k in range(n_res)], dtype=np.int64)


def local_owners(n_res: int, relate_pairs, world: int) -> np.ndarray:
    """GPU that owns each resource of the local chain: splitmix64(group key) mod world (sg_local_owners)."""
    return owner_of(local_group_keys(n_res, relate_pairs).astype(np.uint64), world)


def split_local_events(events: np.ndarray, owners: np.ndarray, world: int):
    """Per rank, the positions of its events in arrival order: an entry and its exit go to the owner of their
    resource (the key bits only; the prioritized bit is not part of the resource)."""
    res = (events["resource"] & np.uint32(0x7FFFFFFF)).astype(np.int64)
    own = np.asarray(owners)[res]
    return [np.nonzero(own == r)[0] for r in range(world)]


def merge_metric_rows(parts) -> np.ndarray:
    """The node's MetricTimerListener rows from every GPU's sg_local_metrics_raw rows: a resource's rows come from
    its owner alone (rt = Σrt / success when success != 0, ArrayMetric.fromBucket); Constants.ENTRY_NODE's rows of
    one second are the sums over the GPUs (each summed its inbound resources), then the same rt and the
    isValidMetricNode filter on the sums. Sorted by (timestamp, resource) as the listener's TreeMap."""
    from sentinel_amd import abi
    rows = np.concatenate([np.asarray(p, abi.METRIC_NODE_DTYPE) for p in parts]) if parts else \
        np.zeros(0, abi.METRIC_NODE_DTYPE)
    res_rows = rows[rows["resource"] != ENTRY_NODE_RESOURCE].copy()
    succ = res_rows["success_qps"]
    res_rows["rt"] = np.where(succ != 0, res_rows["rt"] // np.where(succ != 0, succ, 1), res_rows["rt"])
    ent = rows[rows["resource"] == ENTRY_NODE_RESOURCE]
    merged = []
    for ts in np.unique(ent["timestamp"]):
        g = ent[ent["timestamp"] == ts]
        r = np.zeros((), abi.METRIC_NODE_DTYPE)
        r["timestamp"] = ts
        for f in ("pass_qps", "block_qps", "success_qps", "exception_qps", "rt"):
            r[f] = g[f].sum()
        s = int(r["success_qps"])
        if s != 0:
            r["rt"] = int(r["rt"]) // s
        r["resource"] = ENTRY_NODE_RESOURCE
        if r["pass_qps"] > 0 or r["block_qps"] > 0 or s > 0 or r["exception_qps"] > 0 or r["rt"] > 0:
            merged.append(r)
    out = np.concatenate([res_rows, np.array(merged, abi.METRIC_NODE_DTYPE)]) if merged else res_rows
    order = np.lexsort((out["resource"], out["timestamp"]))
    return out[order]


class LocalMetricRollup:
    """SURVEY §8(e) for the sharded local chain: every GPU's sg_local_metrics_raw rows gathered to every rank
    (all_gather of the row counts, then of the rows padded to the largest, 64 B each as 8 int64 words) and merged
    by merge_metric_rows — the node's metrics.log lines, ENTRY_NODE included. RCCL on the rank's GPU for "nccl",
    CPU tensors for gloo."""

    def __init__(self, coll_device, group=None):
        self.coll = torch.device(coll_device)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1

    def run(self, rows: np.ndarray) -> np.ndarray:
        from sentinel_amd import abi
        rows = np.ascontiguousarray(rows, abi.METRIC_NODE_DTYPE)
        if self.world == 1:
            return merge_metric_rows([rows])
        n = torch.tensor([len(rows)], dtype=torch.int64, device=self.coll)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(sizes, n, group=self.group)
        sizes = [int(s.item()) for s in sizes]
        m = max(1, max(sizes))
        words = np.zeros((m, 8), np.int64)
        words[:len(rows)] = rows.view(np.int64).reshape(-1, 8)
        mine = torch.from_numpy(words).to(self.coll)
        parts = [torch.zeros_like(mine) for _ in range(self.world)]
        dist.all_gather(parts, mine, group=self.group)
        got = [p.cpu().numpy()[:k].copy().view(abi.METRIC_NODE_DTYPE).reshape(-1) for p, k in zip(parts, sizes)]
        return merge_metric_rows(got)


class DeviceLocalMetricRollup:
    """LocalMetricRollup with the rows kept in HBM: every GPU's sg_local_metrics_raw_device rows (int64 [n, 8], 64 B
    each) all-gathered over RCCL (row counts first, then the rows padded to the largest) and merged on the device —
    resource rows' rt = rt / success when success != 0, Constants.ENTRY_NODE rows of one second summed over the GPUs
    then rt = Σrt / Σsuccess and isValidMetricNode on the sums, every row ordered by (timestamp, resource) — the same
    table as merge_metric_rows, as a device tensor. Collective tensors live on coll_device (the rank's GPU for "nccl",
    the CPU for gloo); the merged table is returned there."""

    def __init__(self, coll_device, group=None):
        self.coll = torch.device(coll_device)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1

    def gather(self, rows: torch.Tensor) -> torch.Tensor:
        rows = rows.to(self.coll)
        if self.world == 1:
            return rows
        n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=self.coll)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(sizes, n, group=self.group)
        sizes = [int(x.item()) for x in sizes]
        m = max(1, max(sizes))
        mine = torch.zeros((m, 8), dtype=torch.int64, device=self.coll)
        mine[:rows.shape[0]] = rows
        parts = [torch.empty_like(mine) for _ in range(self.world)]
        dist.all_gather(parts, mine, group=self.group)
        return torch.cat([p[:k] for p, k in zip(parts, sizes)])

    @staticmethod
    def _entry_rows(er: torch.Tensor) -> torch.Tensor:
        """Constants.ENTRY_NODE rows of every GPU, one per second: sums, rt = Σrt / Σsuccess, isValidMetricNode."""
        ts, inv = torch.unique(er[:, 0], return_inverse=True)
        sums = torch.zeros((ts.shape[0], 8), dtype=torch.int64, device=er.device)
        sums.index_add_(0, inv, er)
        m = torch.zeros_like(sums)
        m[:, 0] = ts
        m[:, 1:6] = sums[:, 1:6]
        s = m[:, 3]
        m[:, 5] = torch.where(s != 0, torch.div(m[:, 5], torch.where(s != 0, s, 1), rounding_mode="floor"), m[:, 5])
        m[:, 7] = ENTRY_NODE_RESOURCE
        keep = (m[:, 1] > 0) | (m[:, 2] > 0) | (s > 0) | (m[:, 4] > 0) | (m[:, 5] > 0)
        return m[keep]

    @staticmethod
    def merge(rows: torch.Tensor) -> torch.Tensor:
        """merge_metric_rows on an int64 [n, 8] tensor (words: timestamp, pass, block, success, exception, rt,
        occupied pass, resource | concurrency << 32). The resource rows are ordered by one sort of the key
        (timestamp - the earliest) << 32 | resource and one gather of the rows; the few ENTRY_NODE rows (one per
        second after the merge, the largest resource id) are spliced in after their second's resource rows."""
        n = rows.shape[0]
        if n == 0:
            return rows.clone()
        res = rows[:, 7] & 0xFFFFFFFF
        ent = res == ENTRY_NODE_RESOURCE
        ts = rows[:, 0]
        t_lo, t_hi, n_e = torch.stack([ts.min(), ts.max(), ent.sum()]).tolist()  # one host round trip
        if t_hi - t_lo >= (1 << 31):  # rows spanning ~24 days: two stable sorts instead of the packed key
            rr = torch.cat([rows[~ent], DeviceLocalMetricRollup._entry_rows(rows[ent])]) if n_e else rows[~ent]
            succ = rr[:, 3]
            is_res = (rr[:, 7] & 0xFFFFFFFF) != ENTRY_NODE_RESOURCE
            rr[:, 5] = torch.where(is_res & (succ != 0),
                                   torch.div(rr[:, 5], torch.where(succ != 0, succ, 1), rounding_mode="floor"), rr[:, 5])
            rr = rr[torch.sort(rr[:, 7] & 0xFFFFFFFF, stable=True).indices]
            return rr[torch.sort(rr[:, 0], stable=True).indices]
        key = torch.where(ent, torch.full_like(ts, (1 << 63) - 1), ((ts - t_lo) << 32) | res)
        skey, order = torch.sort(key)
        n_r = n - n_e
        out = rows.index_select(0, order[:n_r])
        succ = out[:, 3]
        out[:, 5] = torch.where(succ != 0, torch.div(out[:, 5], torch.where(succ != 0, succ, 1), rounding_mode="floor"),
                                out[:, 5])
        if n_e == 0:
            return out
        m = DeviceLocalMetricRollup._entry_rows(rows[ent])
        if m.shape[0] == 0:
            return out
        mkey = ((m[:, 0] - t_lo) << 32) | ENTRY_NODE_RESOURCE
        pos = torch.searchsorted(skey[:n_r], mkey).tolist()  # m is sorted by second (torch.unique)
        parts, prev = [], 0
        for i, p in enumerate(pos):
            parts += [out[prev:p], m[i:i + 1]]
            prev = p
        parts.append(out[prev:])
        return torch.cat(parts)

    def run(self, rows: torch.Tensor) -> torch.Tensor:
        return self.merge(self.gather(rows))
