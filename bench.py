"""Benchmark: flow decisions/sec of the cluster token-server hot path (BASELINE.json north star, C3).

One step = one 1000 ms simulated batch of token requests decided exactly as
DefaultTokenService.requestToken → ClusterFlowChecker would, over the flowIds this rank owns
(flowIds hash-sharded over ranks; weak scaling: every rank decides n_requests per step). Requests
are synthetic (Zipf(1.0) flowIds, U{1..32} thresholds, 1 % prioritized), generated on the GPU before
the timed region and resident in HBM. With N > 1 ranks each step also runs the node-wide metric
rollup over RCCL (all-reduce of pass/block totals, all-gather of per-flowId QPS snapshots).

Prints one JSON line (rank 0). See DESIGN.md §Measurement for the roofline bytes.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from sentinel_amd import abi  # noqa: E402
from sentinel_amd.cluster import MetricRollup, shard_flows  # noqa: E402
from sentinel_amd.engine import FlowEngine  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
REQ_B, RES_B = 16, 12          # sg_req / sg_result bytes
STATE_B = 2 * 640 + 2 * 64      # bucket ring 10×64 B read+write, occupy read+write
RULE_B = 16


class ShardWorkload:
    """This rank's share of the C3 node workload, generated on the GPU."""

    def __init__(self, n_flows, n_requests, rank, world, device, seed=3, zipf_s=1.0, span_ms=1000,
                 prio_frac=0.01, multi_frac=0.10, sample_count=10, interval_ms=1000, t0=1_700_000_000_000):
        self.dev = device
        self.n_requests = n_requests
        self.span_ms = span_ms
        self.t0 = t0
        self.prio_frac, self.multi_frac = prio_frac, multi_frac
        rng = np.random.default_rng(seed)
        perm = rng.permutation(n_flows)                       # global popularity rank → flow index
        rank_of = np.empty(n_flows, np.int64)
        rank_of[perm] = np.arange(n_flows)
        self.flows = shard_flows(n_flows, rank, world)        # local key i ↔ global flow self.flows[i]
        self.K = len(self.flows)
        w = 1.0 / np.power(rank_of[self.flows].astype(np.float64) + 1.0, zipf_s)
        cdf = np.cumsum(w)
        self.cdf = torch.from_numpy(cdf / cdf[-1]).to(device)
        counts = rng.integers(1, 33, n_flows).astype(np.float64)
        self.rules = np.zeros(self.K, abi.RULE_DTYPE)
        self.rules["flow_id"] = self.flows.astype(np.int64) + 10_000_001
        self.rules["count"] = counts[self.flows]
        self.rules["threshold_type"] = abi.THRESHOLD_GLOBAL
        self.rules["sample_count"] = sample_count
        self.rules["window_interval_ms"] = interval_ms
        self.gen = torch.Generator(device=device).manual_seed(seed * 1000 + rank)

    def batch(self, b):
        """Requests of simulated second b as a uint8 tensor of n × 16 B (sg_req layout) on the GPU."""
        n, dev, g = self.n_requests, self.dev, self.gen
        ts = torch.randint(0, self.span_ms, (n,), generator=g, device=dev, dtype=torch.int64)
        ts = torch.sort(ts).values + (self.t0 + b * self.span_ms)
        u = torch.rand(n, generator=g, device=dev, dtype=torch.float64)
        key = torch.searchsorted(self.cdf, u, right=True).clamp_(max=self.K - 1)
        acq = torch.ones(n, dtype=torch.int64, device=dev)
        multi = torch.rand(n, generator=g, device=dev) < self.multi_frac
        acq = torch.where(multi, torch.randint(2, 5, (n,), generator=g, device=dev), acq)
        prio = (torch.rand(n, generator=g, device=dev) < self.prio_frac).to(torch.int64) << 31
        words = torch.empty((n, 2), dtype=torch.int64, device=dev)
        words[:, 0] = ts
        words[:, 1] = (acq << 32) | key | prio
        return words.view(torch.uint8).reshape(-1)


PMC_SUMMARY = os.path.join(ROOT, "profiles", "r06_c3_pmc_summary.json")


def pmc_traffic():
    """HBM bytes per step of the decision pipeline's kernels from the committed rocprofv3 FETCH_SIZE /
    WRITE_SIZE passes of this same command (scripts/gpu_round.sh pmc, summarised by scripts/pmc_summary.py;
    FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM). None when no summary is committed."""
    try:
        with open(PMC_SUMMARY) as f:
            return float(json.load(f)["pipeline_bytes_per_step"])
    except (OSError, KeyError, ValueError):
        return None


def cpu_threads():
    """Host threads for the CPU baseline: the box's CPU share (16 per GPU), at most os.cpu_count()."""
    return max(1, min(int(os.environ.get("SG_CPU_THREADS", "16")), os.cpu_count() or 1))


def cpu_baseline(n_flows, n_requests, seconds_budget=25.0, threads=None):
    """The oracle (sequential C restatement) on the same C3 workload, sharded by flowId over `threads` host
    threads ("OpenMP-sharded by key on all host cores"): flowIds are independent with the
    namespace limiter off, so shard t replays, in arrival order, the requests of the flowIds with
    key % threads == t on its own ClusterTokenService (ctypes drops the GIL inside or_cts_decide). Whole
    1000 ms batches until ~10 s of decide time or the budget is spent; the per-batch split into shards
    (numpy, before the clock starts) is the request router's work and is not timed. A single-thread pass
    over the first batch is reported beside it."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle.binding import ClusterTokenService
    from sentinel_amd.workload import ClusterWorkload
    T = threads or cpu_threads()
    wl = ClusterWorkload(n_flows=n_flows, n_requests=n_requests)
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ns["max_allowed_qps"] = 30000
    rules = wl.rules()

    def service():
        s = ClusterTokenService()
        s.set_namespaces(ns)
        s.load_rules(rules)
        return s

    # single thread, first batch
    s1 = service()
    req0 = wl.requests(0)
    t = time.perf_counter()
    s1.decide(req0)
    single = len(req0) / (time.perf_counter() - t)
    del s1
    services = [service() for _ in range(T)]
    pool = ThreadPoolExecutor(max_workers=T)
    t_start = time.time()
    done, decide_s, batches = 0, 0.0, 0
    while decide_s < 10.0 and time.time() - t_start < seconds_budget:
        req = req0 if batches == 0 else wl.requests(batches)
        shard = (req["key"] & abi.KEY_INDEX) % T
        parts = [np.ascontiguousarray(req[shard == i]) for i in range(T)]
        t = time.perf_counter()
        list(pool.map(lambda i: services[i].decide(parts[i]), range(T)))
        decide_s += time.perf_counter() - t
        done += len(req)
        batches += 1
    pool.shutdown()
    return {"value": done / decide_s, "unit": "decisions/s", "cores": T, "kind": "port",
            "single_thread_value": single,
            "sample": f"{batches} consecutive 1000 ms C3 batches ({done} requests, {n_flows} flowIds) through "
                      f"oracle/liboracle.so (sequential C restatement of DefaultTokenService/ClusterFlowChecker), "
                      f"flowIds sharded by key % {T} over {T} threads, {decide_s:.1f} s of decide time "
                      f"(shard split not timed); single thread on batch 0: {single / 1e6:.2f} M decisions/s"}


def end_to_end(eng, wl, first_b, n_batches, n_req, n_out=4):
    """Decisions/s with the requests in HOST memory (what a JVM token server hands over through JNI): pinned
    buffers → sg_flow_submit (H2D and D2H on the copy engines, overlapping each other and the decisions, 3 batches
    in flight) → sg_flow_wait, n_batches back to back in steady state. Every batch has its own pinned
    request buffer (time-ordered batches, generated before the clock starts); the outputs cycle through n_out
    buffers, as a caller reusing its result buffers would."""
    ins = [eng.host_array(n_req, abi.REQ_DTYPE) for _ in range(n_batches)]
    outs = [eng.host_array(n_req, abi.RES_DTYPE) for _ in range(n_out)]
    for i in range(n_batches):
        ins[i][:] = wl.batch(first_b + i).cpu().numpy().view(abi.REQ_DTYPE)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tickets = []
    for i in range(n_batches):
        if len(tickets) >= n_out:  # the output buffer about to be reused has been collected
            eng.wait(tickets[i - n_out])
        tickets.append(eng.submit(ins[i], outs[i % n_out]))
    for t in tickets[max(0, n_batches - n_out):]:
        eng.wait(t)
    el = time.perf_counter() - t0
    ok = int((outs[(n_batches - 1) % n_out]["status"] == abi.OK).sum())
    for a in ins + outs:
        eng.free_host(a)
    h2d, d2h = n_req * REQ_B, n_req * RES_B
    return {"value": n_batches * n_req / el, "unit": "decisions/s", "batches": n_batches,
            "ms_per_batch": el * 1000.0 / n_batches, "h2d_bytes_per_batch": h2d, "d2h_bytes_per_batch": d2h,
            "h2d_GBps": h2d * n_batches / el / 1e9, "d2h_GBps": d2h * n_batches / el / 1e9, "ok_last_batch": ok,
            "d2h_path": "shader copy (k_copy_out)" if os.environ.get("SG_D2H") == "1" else "copy engine",
            "path": "pinned host buffers -> sg_flow_submit (H2D / decide / D2H overlapped, 3 in flight) -> sg_flow_wait"}


def node_main(args):
    """--node: the node handle (sg_node_*) as a token server over N devices in ONE process — the front on device 0
    validates and runs the namespace limiters over each node batch in caller order, routes the requests by owner
    (splitmix64(flowId) mod N) and every shard decides its slice on its device (the records path and the node
    pipeline, sg_node_flow_enqueue, when all shards share device 0; peer copies of the slices over xGMI otherwise).
    Weak scaling: N x --requests per node batch over N x --flows flowIds. Not the driver's launch (that one is
    torch.distributed.run with one rank per GPU and no routing); this line prices the routing."""
    from sentinel_amd.engine import NodeEngine
    N = args.gpus
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n_req = args.requests * N
    wl = ShardWorkload(args.flows * N, n_req, 0, 1, dev)
    nd = NodeEngine(list(range(N)), max_batch=n_req)
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ns["max_allowed_qps"] = args.limiter_qps if args.limiter_qps > 0 else 30000
    ns["limiter_enabled"] = 1 if args.limiter_qps > 0 else 0
    nd.set_namespaces(ns)
    nd.load_rules(wl.rules)
    total_steps = args.warmup + args.steps
    batches = [wl.batch(b) for b in range(total_steps)]
    outs = [torch.empty(n_req * RES_B, dtype=torch.uint8, device=dev) for _ in range(2)]
    torch.cuda.synchronize()

    def run_steps(b0, b1):
        tickets = []
        for b in range(b0, b1):
            if len(tickets) >= 2:
                nd.wait(tickets.pop(0))
            tickets.append(nd.enqueue_device(batches[b].data_ptr(), n_req, outs[b % 2].data_ptr()))
        for t in tickets:
            nd.wait(t)

    run_steps(0, args.warmup)
    for d in range(N):
        torch.cuda.synchronize(d)
    t0 = time.perf_counter()
    run_steps(args.warmup, total_steps)
    for d in range(N):
        torch.cuda.synchronize(d)
    elapsed = time.perf_counter() - t0
    last = batches[-1].view(torch.int64).reshape(-1, 2)[:, 1] & 0x7FFFFFFF
    touched = int(torch.unique(last).numel())
    ms_per_step = elapsed * 1000.0 / args.steps
    b_alg = n_req * (REQ_B + RES_B) + touched * (STATE_B + RULE_B)
    step_gbs = b_alg / (ms_per_step / 1000.0) / 1e9
    peak = HBM_PEAK_GBS * N
    print(json.dumps({
        "metric": "flow decisions/sec (node) at 1M flowIds, 1/2/4/8 GPU; HBM GB/s vs peak",
        "value": n_req / (elapsed / args.steps), "unit": "decisions/s", "n_gpus": N, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (GPU-generated, seeded): Zipf(1.0) flowIds, counts U{1..32}, 10% acquire U{2..4}, 1% prioritized",
        "config": {"workload": "C3 cluster token server through the node handle (sg_node, routing inside)",
                   "flow_ids": args.flows * N, "requests_per_step": n_req, "simulated_ms_per_step": wl.span_ms,
                   "parallelism": f"sg_node over {N} device(s), one process",
                   "namespace_limiter": (f"on, maxAllowedQps {args.limiter_qps:g}" if args.limiter_qps > 0 else "off")},
        "roofline": {"bound": "hbm", "kernel": "whole node batch (front prep + routing + shard sort + walk), step time",
                     "achieved": step_gbs, "peak": peak, "unit": "GB/s", "frac": step_gbs / peak, "traffic": None,
                     "algorithmic_bytes_per_step": b_alg, "touched_flow_ids": touched},
    }), flush=True)


C5_PMC_SUMMARY = os.path.join(ROOT, "profiles", "r06_c5_node_pmc_summary.json")


def c5_rules(K):
    """BASELINE configs[4]: every resource a QPS FlowRule (count U{1..64}) + an RT breaker (100 ms, slow ratio 0.5)
    + an exception-ratio breaker (0.5), statIntervalMs 1000, minRequestAmount 5, timeWindow 10 s (bench_configs c5)."""
    from oracle.binding import degrade_rule
    rng = np.random.default_rng(5)
    rules = np.zeros(K, abi.LOCAL_RULE_DTYPE)
    rules["flow_count"] = rng.integers(1, 65, K).astype(np.float64)
    rules["flow_grade"] = abi.FLOW_GRADE_QPS
    rules["n_breakers"] = 2
    b = np.zeros(2, abi.DEGRADE_RULE_DTYPE)
    b[0] = degrade_rule(abi.DEGRADE_RT, 100, 10, 5, 1000, 0.5)
    b[1] = degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.5, 10, 5, 1000)
    rules["breakers"] = b
    return rules


def c5_trace(rules, own, n, n_batches, rank, check, t0=1_700_000_000_000):
    """This rank's share of the node's C5 trace: the entries of the resources it owns (Zipf(1.0) popularity over the
    node's resources, restricted to `own` — the node trace split by owner, since resources share no state) and the
    exits of the passed ones, produced by the oracle's client model over the owned resources (oracle.binding
    LocalTraceGen: the exits depend on the decisions). Returns per batch (events with node resource ids, the
    oracle's decisions, the oracle's raw metric rows at the batch's end with node ids — check only) and the oracle's
    replay seconds (the cpu_baseline)."""
    from oracle.binding import LocalChain, LocalTraceGen
    K = len(rules)
    perm = np.random.default_rng(5).permutation(K)             # popularity rank -> resource
    rank_of = np.empty(K, np.int64)
    rank_of[perm] = np.arange(K)
    w = 1.0 / (rank_of[own].astype(np.float64) + 1.0)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    ora = LocalChain(2, 1000, 500)
    ora.load_rules(rules[own])
    ora.set_entry_types(np.ones(len(own), np.uint8))
    gen = LocalTraceGen(ora)
    rng = np.random.default_rng(5 + 1000 * rank)
    out, gen_s = [], 0.0
    for bt in range(n_batches):
        ent = np.zeros(n, abi.LOCAL_EVENT_DTYPE)
        ent["ts_ms"] = t0 + 1000 * bt + np.sort(rng.integers(0, 1000, n))
        ent["resource"] = np.minimum(np.searchsorted(cdf, rng.random(n), side="right"), len(own) - 1)
        ent["count"] = 1
        rt = np.minimum(np.round(np.exp(rng.normal(2.5, 0.8, n))), 10_000).astype(np.int32)
        err = (rng.random(n) < 0.05).astype(np.uint8)
        t = time.perf_counter()
        ev, res = gen.run(ent, rt, err, t0 + 1000 * (bt + 1))
        gen_s += time.perf_counter() - t
        rows = ora.metrics(t0 + 1000 * (bt + 1), raw=True) if check else None
        ev["resource"] = own[ev["resource"]].astype(np.uint32)
        if rows is not None:
            m = rows["resource"] != abi.ENTRY_NODE_RESOURCE
            rows["resource"][m] = own[rows["resource"][m]].astype(np.uint32)
        out.append((ev, res, rows))
    return out, gen_s


def c5_main(args, rank, world, dev, coll, one_dev):
    """--workload c5: BASELINE configs[4] (1M resources, QPS FlowRule + RT + exception-ratio breakers, minute window)
    over the node's GPUs, one rank per GPU. Every rank loads the node's rules (all resources EntryType.IN) and decides
    the entries and exits of the resources sg_local_owners gives it (weak scaling: --requests entries per rank per
    1000 ms step plus the exits of the passed ones); after each batch the node's MetricTimerListener rows of that
    second are rolled up on the devices (sg_local_metrics_raw_enqueue behind the batch's walkers, then
    DeviceLocalMetricRollup while the next batch runs: RCCL all_gather of the rows, ENTRY_NODE sums and the
    (timestamp, resource) order on the GPU). The event stream depends on the
    decisions, so each rank's share is produced by the oracle's client model before the timed region. With --check
    (on by default in the SG_BENCH_ONE_DEVICE rehearsal) every decision and every merged row is compared with the
    oracle's node replay after the timed region."""
    from sentinel_amd.cluster import DeviceLocalMetricRollup, merge_metric_rows
    check = args.check or one_dev
    K, n = args.resources, args.requests
    rules = c5_rules(K)
    eng = FlowEngine(device=dev.index, max_batch=1)
    eng.local_load_rules(rules, 2, 1000, 500)
    eng.local_set_entry_types(np.ones(K, np.uint8))
    owners = eng.local_owners(world)                         # sg_local_owners: the routing of the node's events
    own = np.nonzero(owners == rank)[0]
    total_steps = args.warmup + args.steps
    t_gen = time.time()
    trace, gen_s = c5_trace(rules, own, n, total_steps, rank, check)
    print(f"# c5 rank {rank}: {len(own)} resources, {sum(len(e) for e, _, _ in trace)} events from the oracle client "
          f"model in {time.time() - t_gen:.1f} s", file=sys.stderr, flush=True)
    sizes = [len(e) for e, _, _ in trace]
    eng.close()
    eng = FlowEngine(device=dev.index, max_batch=max(sizes))
    eng.local_load_rules(rules, 2, 1000, 500)
    eng.local_set_entry_types(np.ones(K, np.uint8))
    batches = [torch.from_numpy(e.view(np.uint8).copy()).to(dev) for e, _, _ in trace]
    outs = [torch.empty(sz * abi.LOCAL_RES_DTYPE.itemsize, dtype=torch.uint8, device=dev) for sz in sizes]
    # room for every row the listener could return (59 per resource + 60): the metric pass skips its counting pass
    rows_buf = [torch.empty((59 * K + 60, 8), dtype=torch.int64, device=dev) for _ in range(2)]
    rows_cnt = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(2)]
    rollup = DeviceLocalMetricRollup(coll)
    merged = [None] * total_steps
    t0 = 1_700_000_000_000
    # the rollups on streams of their own (torch's default stream is the null stream, which would also wait for the
    # pipeline's walkers), one per row buffer: second b's stream waits for second b's metric pass only
    sides = [torch.cuda.Stream(dev) for _ in range(2)]
    tickets = []
    torch.cuda.synchronize()

    def roll(b):  # second b's rows
        with torch.cuda.stream(sides[b % 2]):
            merged[b] = rollup.run(rows_buf[b % 2][:int(rows_cnt[b % 2].item())])

    def step(b):
        """Batch b on the local pipeline, the rollup of second b - 1 while it runs, then second b's metric pass
        enqueued behind its walkers (sg_local_metrics_raw_enqueue: no pipeline drain; after the rollup that last
        read the same row buffer)."""
        if len(tickets) >= 2:
            eng.local_wait(tickets.pop(0))
        tickets.append(eng.local_enqueue(batches[b].data_ptr(), sizes[b], outs[b].data_ptr()))
        if b > 0:  # (second b - 1 first: enqueueing b's metric pass before it measured 3.30 against 3.00-3.12 ms)
            roll(b - 1)
        eng.local_metrics_raw_enqueue(t0 + 1000 * (b + 1), rows_buf[b % 2], rows_cnt[b % 2], sides[b % 2].cuda_stream)

    def drain(b_last):
        roll(b_last)
        while tickets:
            eng.local_wait(tickets.pop(0))

    for b in range(args.warmup):
        step(b)
    drain(args.warmup - 1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for b in range(args.warmup, total_steps):
        step(b)
    drain(total_steps - 1)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    stats = torch.tensor([elapsed, float(sum(sizes[args.warmup:]))], dtype=torch.float64, device=coll)
    if world > 1:
        t_max = stats[:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        tot = stats[1:].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed, decided = float(t_max.item()), float(tot.item())
    else:
        elapsed, decided = elapsed, float(stats[1].item())

    parity = None
    if check:  # every decision of this rank, then the merged rows of every second against the node replay
        bad = 0
        for b in range(total_steps):
            got = outs[b].cpu().numpy().view(abi.LOCAL_RES_DTYPE)
            bad += int((got != trace[b][1]).sum())
        rows_ok = True
        for b in range(total_steps):
            parts = [trace[b][2]]
            if world > 1:
                allp = [None] * world
                dist.all_gather_object(allp, trace[b][2])
                parts = allp
            want = merge_metric_rows(parts)
            got = merged[b].cpu().numpy().copy().view(abi.METRIC_NODE_DTYPE).reshape(-1)
            rows_ok &= bool(np.array_equal(got, want))
        flags = torch.tensor([bad, 0 if rows_ok else 1], dtype=torch.int64, device=coll)
        if world > 1:
            dist.all_reduce(flags)
        parity = {"decisions_differing": int(flags[0].item()), "metric_steps_differing": int(flags[1].item()),
                  "checked": f"all {total_steps} batches on every rank against the oracle's node replay; merged "
                             f"metric rows (ENTRY_NODE included) of every second against merge_metric_rows"}

    touched = int(np.unique(trace[-1][0]["resource"] & 0x7FFFFFFF).size)
    ms_per_step = elapsed * 1000.0 / args.steps
    # per event 32 B in + 8 B out; per touched resource: second window 2x128 B, two minute buckets 2x2x64 B, head
    # (threads + two breakers) 2x128 B, rule 80 B (bench_configs c5); per rank and step
    b_alg = sizes[-1] * (32 + 8) + touched * (2 * 128 + 2 * 2 * 64 + 2 * 128 + 80)
    step_gbs = b_alg / (ms_per_step / 1000.0) / 1e9
    traffic = None
    if os.path.exists(C5_PMC_SUMMARY):
        traffic = json.load(open(C5_PMC_SUMMARY)).get("pipeline_bytes_per_step")
    result = {
        "metric": "local flow + circuit-breaker decisions/sec (entries + exits), 1M resources, 1/2/4/8 GPU",
        "value": decided / elapsed, "unit": "decisions/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (seeded): Zipf(1.0) resources, rt lognormal(2.5, 0.8) ms, 5% errors; exits generated by "
                "the oracle client model",
        "config": {"workload": "C5: 1M resources x (QPS FlowRule + RT breaker + exception-ratio breaker), minute "
                               "window, --requests entries per GPU per 1000 ms step + exits of passed entries, "
                               "resources sharded by sg_local_owners, per-step device metric rollup",
                   "resources": K, "resources_per_gpu": len(own), "entries_per_step_per_gpu": n,
                   "events_last_step_per_gpu": sizes[-1],
                   "parallelism": f"resources sharded by sg_local_owners x{world}" + (" (one-device rehearsal)" if one_dev else ""),
                   "rollup": ("DeviceLocalMetricRollup per step (RCCL all_gather of raw rows, merge on device)"
                              if world > 1 and not one_dev else
                              "DeviceLocalMetricRollup per step (gloo rehearsal)" if world > 1 else
                              "DeviceLocalMetricRollup per step (merge on device, 1 GPU)")},
        "roofline": {"bound": "hbm", "kernel": "whole step (local pipeline + metric rows + rollup), step time",
                     "achieved": step_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": step_gbs / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": os.path.relpath(C5_PMC_SUMMARY, ROOT) if traffic else None,
                     "algorithmic_bytes_per_step": b_alg, "touched_resources": touched},
    }
    if parity is not None:
        result["parity"] = parity
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = {"value": sum(sizes) / gen_s, "unit": "decisions/s", "cores": 1, "kind": "port",
                                  "sample": f"the oracle (oracle/liboracle.so LocalChain) replaying all {sum(sizes)} "
                                            f"events of this rank while generating them (client model, 1 thread), "
                                            f"{gen_s:.1f} s"}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def launch_ranks(n):
    """Run this script as n ranks of one node (the driver's own launch line), as a child process."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--flows", type=int, default=1_000_000)
    ap.add_argument("--requests", type=int, default=16_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e-batches", type=int, default=16, help="host-buffer batches for the end-to-end figure (0: skip)")
    ap.add_argument("--limiter-qps", type=float, default=0.0,
                    help="namespace GlobalRequestLimiter maxAllowedQps (SURVEY §8d C3's second run: 1e12 exercises the "
                         "pre-pass without rejecting); 0: limiter off, the headline configuration")
    ap.add_argument("--workload", choices=["c3", "c5"], default="c3",
                    help="c3: the headline cluster token server (default); c5: BASELINE configs[4], the local chain "
                         "with breakers over --resources resources, sharded by sg_local_owners, per-step metric rollup")
    ap.add_argument("--resources", type=int, default=1_000_000, help="c5: the node's resources")
    ap.add_argument("--check", action="store_true",
                    help="c5: compare every decision and merged metric row with the oracle's node replay (untimed; "
                         "on by default under SG_BENCH_ONE_DEVICE=1)")
    ap.add_argument("--node", action="store_true",
                    help="one process, one sg_node over --gpus N devices: node-order batches of N x --requests over "
                         "N x --flows flowIds, routing inside the library and inside the timed region")
    args = ap.parse_args()
    if args.node:
        return node_main(args)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` outside a launcher: start N ranks (one process per GPU) through torch.distributed.run
        # and exit with its status. Nothing in this parent has touched the GPU (torch.cuda is not initialised).
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch with --nproc-per-node {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # SG_BENCH_ONE_DEVICE=1: rehearsal of the N-rank path on a one-GPU box (every rank on device 0, gloo on CPU
    # tensors instead of RCCL); never the measured configuration
    one_dev = os.environ.get("SG_BENCH_ONE_DEVICE") == "1"
    if one_dev:
        local_rank = 0
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local_rank)
        if one_dev:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    coll = torch.device("cpu") if one_dev else dev  # where the collectives' tensors live
    torch.cuda.set_device(dev)
    if args.workload == "c5":
        return c5_main(args, rank, world, dev, coll, one_dev)

    wl = ShardWorkload(args.flows, args.requests, rank, world, dev)
    eng = FlowEngine(device=local_rank, max_batch=args.requests)
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ns["max_allowed_qps"] = args.limiter_qps if args.limiter_qps > 0 else 30000
    ns["limiter_enabled"] = 1 if args.limiter_qps > 0 else 0
    eng.set_namespaces(ns)
    eng.load_rules(wl.rules)

    total_steps = args.warmup + args.steps
    n_phase = 2  # extra batches through the synchronous path for the per-phase device times
    batches = [wl.batch(b) for b in range(total_steps + n_phase)]
    # one output buffer per batch in flight (the pipeline keeps up to 4 batches enqueued)
    outs = [torch.empty(args.requests * RES_B, dtype=torch.uint8, device=dev) for _ in range(4)]
    snaps = [torch.empty((wl.K, 2), dtype=torch.float64, device=dev) for _ in range(2)]
    rollup = MetricRollup(wl.K, coll) if world > 1 else None
    torch.cuda.synchronize()

    def run_steps(b0, b1):
        """Batches b0..b1-1 back to back on the pipelined path (sg_flow_enqueue: each batch's sort beside the
        previous batch's walkers). With N > 1 ranks, the node-wide metric rollup of each simulated second runs
        over RCCL while the next second is being decided (its snapshot is ordered after the batch)."""
        tickets, pend = [], None
        for b in range(b0, b1):
            tickets.append(eng.enqueue_device(batches[b].data_ptr(), args.requests, outs[b % 4].data_ptr()))
            if rollup is not None:
                now = wl.t0 + (b + 1) * wl.span_ms
                t_snap = eng.snapshot_enqueue(now, snaps[b % 2].data_ptr(), wl.K)
                if pend is not None:
                    eng.wait(pend[0])
                    rollup.run(snaps[pend[1] % 2].to(coll))
                pend = (t_snap, b)
        for t in tickets:
            eng.wait(t)
        if pend is not None:
            eng.wait(pend[0])
            rollup.run(snaps[pend[1] % 2].to(coll))

    run_steps(0, args.warmup)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(args.warmup, total_steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t_max = torch.tensor([elapsed], dtype=torch.float64, device=coll)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    elapsed = float(t_max.item())

    # per-phase device time of one batch on its own (synchronous path, HIP events on the call's stream; untimed)
    eng.enable_stats(True)
    phase = {"sort_ms": 0.0, "walk_ms": 0.0, "total_ms": 0.0}
    stream = torch.cuda.current_stream(dev)
    for b in range(total_steps, total_steps + n_phase):
        eng.decide_device(batches[b].data_ptr(), args.requests, outs[0].data_ptr(), stream.cuda_stream)
        st = eng.stats()
        for k in phase:
            phase[k] += st[k] / n_phase
        long_segments = st["long_segments"]
    eng.enable_stats(False)

    # touched flowIds of the last batch (for the algorithmic byte count)
    last = batches[-1].view(torch.int64).reshape(-1, 2)[:, 1] & 0x7FFFFFFF
    touched = int(torch.unique(last).numel())
    ms_per_step = elapsed * 1000.0 / args.steps
    value = args.requests * world / (elapsed / args.steps)
    b_alg = args.requests * (REQ_B + RES_B) + touched * (STATE_B + RULE_B)
    walk_ms = phase["walk_ms"]
    total_ms = phase["total_ms"]
    step_gbs = b_alg / (ms_per_step / 1000.0) / 1e9  # pipelined: algorithmic bytes per batch over the step time
    result = {
        "metric": "flow decisions/sec (node) at 1M flowIds, 1/2/4/8 GPU; HBM GB/s vs peak",
        "value": value,
        "unit": "decisions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (GPU-generated, seeded): Zipf(1.0) flowIds, counts U{1..32}, 10% acquire U{2..4}, 1% prioritized",
        "config": {"workload": "C3 cluster token server: ClusterFlowChecker, FLOW_THRESHOLD_GLOBAL, S=10/1000 ms",
                   "flow_ids": args.flows, "flow_ids_per_gpu": wl.K, "requests_per_step_per_gpu": args.requests,
                   "simulated_ms_per_step": wl.span_ms, "parallelism": f"hash-sharded flowIds x{world}" + (" (one-device rehearsal)" if one_dev else ""),
                   "rollup": "RCCL all_reduce + all_gather per step" if world > 1 else "none (1 GPU)",
                   "namespace_limiter": (f"on, maxAllowedQps {args.limiter_qps:g}" if args.limiter_qps > 0 else "off")},
        "roofline": {"bound": "hbm", "kernel": "whole batch pipeline (prep + sort + walk), step time with batches "
                                               "pipelined (sort of batch i+1 beside the walkers of batch i)",
                     "achieved": step_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": step_gbs / HBM_PEAK_GBS,
                     "traffic": pmc_traffic(), "traffic_source": os.path.relpath(PMC_SUMMARY, ROOT),
                     "algorithmic_bytes_per_step": b_alg, "touched_flow_ids": touched},
        "phases_ms": {"device_total_one_batch_unpipelined": total_ms, "sort": phase["sort_ms"], "walk": walk_ms,
                      "long_segments": long_segments},
    }
    if world == 1 and args.e2e_batches > 0:
        result["end_to_end"] = end_to_end(eng, wl, total_steps + n_phase, args.e2e_batches, args.requests)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.flows, args.requests)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
