"""Secondary benchmarks: the other BASELINE.json configurations, on one GPU, with the same JSON contract as
bench.py (which measures the headline C3 workload).

  --workload c2  10k resources, QPS FlowRule each (count U{1..64}), DefaultController over each resource's
                 StatisticNode (second window S=2/1000 ms + minute window), 16M entries per 1000 ms batch,
                 Zipf(1.0) resources, acquire 1 (10 % U{2..4}), no prioritized requests, no exits.
  --workload c4  one ParamFlowRule (count 5, durationInSec 1, DEFAULT token bucket) over 10M distinct u64
                 values, Zipf(1.1), 16M requests per 1000 ms batch, exact HBM table (2^25 slots).
  --workload c5  1M resources, each a QPS FlowRule + RT breaker (100 ms, slow ratio 0.5) + exception-ratio
                 breaker (0.5); statIntervalMs 1000, minRequestAmount 5, timeWindow 10 s; 16M entries per
                 1000 ms batch plus the exits of the passed ones (rt ~ lognormal, median 12 ms; 5 % errors).
                 The event stream depends on the decisions (only passed entries exit), so it is produced by
                 the CPU oracle's client model (oracle.binding.LocalTraceGen) before the timed region.
  --workload cparam  cluster hot-parameter tokens: 1000 ClusterParamFlowRules, 50k values each Zipf(1.1), 16M
                 requests per batch, 10 % with 2-3 values (the fixed-point path).
  --workload slot  the whole slot chain at C5 size with 10 % of the resources carrying an origin-limitApp rule, a
                 WarmUp rule or a ParamFlowRule (the cx walker's share); every batch checked against the oracle.
  --workload node  the C3 workload through the node handle (G same-device shards, --shards), pipelined.
  --workload pace  1M resources, each a FlowRule with CONTROL_BEHAVIOR_RATE_LIMITER (RateLimiterController,
                 count U{1..64}, maxQueueingTimeMs 500), 16M canPass calls per 1000 ms batch, Zipf(1.0),
                 acquire 1 (10 % U{2..4}).

Inputs are resident in HBM before the timed region; one step = one batch. cpu_baseline = the oracle
(sequential C restatement, 1 thread) on the first batch of the same workload.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from sentinel_amd import abi  # noqa: E402
from sentinel_amd.engine import FlowEngine  # noqa: E402

HBM_PEAK_GBS = 8000.0
T0 = 1_700_000_000_000


def zipf_cdf(n, s, seed):
    rng = np.random.default_rng(seed)
    perm = rng.permutation(n)
    w = 1.0 / np.power(np.arange(1, n + 1, dtype=np.float64), s)
    cdf = np.cumsum(w)
    return cdf / cdf[-1], perm


def gpu_keys(cdf_t, perm_t, n, gen):
    u = torch.rand(n, generator=gen, device=cdf_t.device, dtype=torch.float64)
    r = torch.searchsorted(cdf_t, u, right=True).clamp_(max=len(cdf_t) - 1)
    return perm_t[r]


def timed(step, warmup, steps):
    for b in range(warmup):
        step(b)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in range(warmup, warmup + steps):
        step(b)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def local_timed(eng, batches, sizes, args, dev, stream):
    """C2 / C5 steps through sg_local_enqueue (the pipelined local path: a batch's front half — validation, sort by
    resource, segment and exit lists — beside the previous batch's walkers): at most two batches in flight (the two
    workspaces), each ticket collected two batches later, two out buffers alternating. --local-sync: the synchronous
    sg_local_decide_batch, one batch at a time."""
    outs = [torch.empty(max(sizes) * 8, dtype=torch.uint8, device=dev) for _ in range(2)]
    if args.local_sync:
        return timed(lambda b: eng.local_decide_device(batches[b].data_ptr(), sizes[b], outs[0].data_ptr(), stream),
                     args.warmup, args.steps)
    tickets = []

    def step(b):
        if len(tickets) >= 2:
            eng.local_wait(tickets.pop(0))
        tickets.append(eng.local_enqueue(batches[b].data_ptr(), sizes[b], outs[b % 2].data_ptr()))

    torch.cuda.synchronize()  # the batches were generated on torch's stream
    el = timed(step, args.warmup, args.steps)
    for t in tickets:
        eng.local_wait(t)
    return el


def c2(args, dev):
    K, n = 10_000, args.events
    rng = np.random.default_rng(2)
    rules = np.zeros(K, abi.LOCAL_RULE_DTYPE)
    rules["flow_count"] = rng.integers(1, 65, K).astype(np.float64)
    rules["flow_grade"] = abi.FLOW_GRADE_QPS
    cdf, perm = zipf_cdf(K, 1.0, 2)
    cdf_t, perm_t = torch.from_numpy(cdf).to(dev), torch.from_numpy(perm.astype(np.int64)).to(dev)
    gen = torch.Generator(device=dev).manual_seed(2)

    def batch(b):
        w = torch.zeros((n, 4), dtype=torch.int64, device=dev)
        w[:, 0] = torch.sort(torch.randint(0, 1000, (n,), generator=gen, device=dev)).values + T0 + 1000 * b
        cnt = torch.where(torch.rand(n, generator=gen, device=dev) < 0.1,
                          torch.randint(2, 5, (n,), generator=gen, device=dev), torch.ones(n, dtype=torch.int64, device=dev))
        w[:, 2] = gpu_keys(cdf_t, perm_t, n, gen) | (cnt << 32)   # resource | count << 32; kind = 0 (entry)
        return w.view(torch.uint8).reshape(-1)

    eng = FlowEngine(device=0, max_batch=n)
    eng.local_load_rules(rules, 2, 1000, 500)
    batches = [batch(b) for b in range(args.warmup + args.steps)]
    stream = torch.cuda.current_stream(dev).cuda_stream
    el = local_timed(eng, batches, [n] * len(batches), args, dev, stream)
    touched = int(torch.unique(batches[-1].view(torch.int64).reshape(-1, 4)[:, 2] & 0xFFFFFFFF).numel())
    # per event: 32 B sg_local_event in + 8 B result out; per touched resource: second window 2x64 B read +
    # write, one minute bucket read + write, curThreadNum/breaker head 2x16 B, rule 16 B
    b_alg = n * (32 + 8) + touched * (2 * 128 + 2 * 64 + 2 * 16 + 16)
    base = None
    if not args.no_cpu_baseline:
        from oracle.binding import LocalChain
        ev = batches[0].view(torch.int64).reshape(-1, 4)[: args.cpu_events].cpu().numpy().copy().view(abi.LOCAL_EVENT_DTYPE).reshape(-1)
        ora = LocalChain(2, 1000, 500)
        ora.load_rules(rules)
        t = time.perf_counter()
        ora.decide(ev)
        dt = time.perf_counter() - t
        base = {"value": len(ev) / dt, "unit": "decisions/s", "cores": 1, "kind": "port",
                "sample": f"first {len(ev)} events of batch 0 through oracle LocalChain (1 thread), {dt:.1f} s"}
    return {"metric": "local flow decisions/sec (DefaultController over StatisticNode), 10k resources",
            "workload": "C2: 10k resources x QPS FlowRule, S=2/1000 ms second window + minute window, 16M entries/batch",
            "value": n * args.steps / el, "el": el, "n": n, "b_alg": b_alg, "touched": touched, "cpu": base,
            "data": "synthetic (GPU-generated, seeded): Zipf(1.0) resources, counts U{1..64}, 10% acquire U{2..4}"}


def c4(args, dev):
    n, V = args.events, 10_000_000
    rules = np.zeros(1, abi.PARAM_RULE_DTYPE)
    rules["count"], rules["duration_sec"], rules["behavior"], rules["capacity_log2"] = 5, 1, abi.BEHAVIOR_DEFAULT, 25
    cdf, perm = zipf_cdf(V, 1.1, 4)
    cdf_t, perm_t = torch.from_numpy(cdf).to(dev), torch.from_numpy(perm.astype(np.int64)).to(dev)
    gen = torch.Generator(device=dev).manual_seed(4)

    def batch(b):
        w = torch.zeros((n, 3), dtype=torch.int64, device=dev)
        w[:, 0] = torch.sort(torch.randint(0, 1000, (n,), generator=gen, device=dev)).values + T0 + 1000 * b
        w[:, 1] = gpu_keys(cdf_t, perm_t, n, gen) * 0x9E3779B1 + 17     # distinct u64 values
        w[:, 2] = 1 << 32                                                # rule 0, acquireCount 1
        return w.view(torch.uint8).reshape(-1)

    eng = FlowEngine(device=0, max_batch=n)
    eng.param_load_rules(rules)
    batches = [batch(b) for b in range(args.warmup + args.steps)]
    out = torch.empty(n * 4, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    el = timed(lambda b: eng.param_decide_device(batches[b].data_ptr(), n, out.data_ptr(), stream), args.warmup, args.steps)
    touched = int(torch.unique(batches[-1].view(torch.int64).reshape(-1, 3)[:, 1]).numel())
    b_alg = n * (24 + 4) + touched * (2 * 32)   # request in, pass bit out; per value slot 32 B read + write
    base = None
    if not args.no_cpu_baseline:
        from oracle.binding import ParamFlowChecker
        req = batches[0].view(torch.int64).reshape(-1, 3)[: args.cpu_events].cpu().numpy().copy().view(abi.PARAM_REQ_DTYPE).reshape(-1)
        ora = ParamFlowChecker()
        ora.load_rules(rules)
        t = time.perf_counter()
        ora.decide(req)
        dt = time.perf_counter() - t
        base = {"value": len(req) / dt, "unit": "decisions/s", "cores": 1, "kind": "port",
                "sample": f"first {len(req)} requests of batch 0 through oracle ParamFlowChecker (1 thread), {dt:.1f} s"}
    return {"metric": "hot-parameter decisions/sec (ParamFlowChecker token bucket), 10M values",
            "workload": "C4: 1 ParamFlowRule count=5/1 s, 10M distinct values Zipf(1.1), 16M requests/batch",
            "value": n * args.steps / el, "el": el, "n": n, "b_alg": b_alg, "touched": touched, "cpu": base,
            "data": "synthetic (GPU-generated, seeded)"}


def c5(args, dev):
    from oracle.binding import LocalChain, LocalTraceGen, degrade_rule, local_rule
    K, n = args.resources, args.events
    rng = np.random.default_rng(5)
    rules = np.zeros(K, abi.LOCAL_RULE_DTYPE)
    rules["flow_count"] = rng.integers(1, 65, K).astype(np.float64)
    rules["flow_grade"] = abi.FLOW_GRADE_QPS
    rules["n_breakers"] = 2
    b = np.zeros(2, abi.DEGRADE_RULE_DTYPE)
    b[0] = degrade_rule(abi.DEGRADE_RT, 100, 10, 5, 1000, 0.5)
    b[1] = degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.5, 10, 5, 1000)
    rules["breakers"] = b
    cdf, perm = zipf_cdf(K, 1.0, 5)
    ora = LocalChain(2, 1000, 500)
    ora.load_rules(rules)
    gen = LocalTraceGen(ora)
    t_gen = time.time()
    host = []
    gen_s = 0.0
    for bt in range(args.warmup + args.steps):
        ent = np.zeros(n, abi.LOCAL_EVENT_DTYPE)
        ent["ts_ms"] = T0 + 1000 * bt + np.sort(rng.integers(0, 1000, n))
        ent["resource"] = perm[np.minimum(np.searchsorted(cdf, rng.random(n), side="right"), K - 1)]
        ent["count"] = 1
        rt = np.minimum(np.round(np.exp(rng.normal(2.5, 0.8, n))), 10_000).astype(np.int32)
        err = (rng.random(n) < 0.05).astype(np.uint8)
        t = time.perf_counter()
        ev, _ = gen.run(ent, rt, err, T0 + 1000 * (bt + 1))
        gen_s += time.perf_counter() - t
        host.append(ev)
    print(f"# c5 trace: {sum(len(e) for e in host)} events generated by the oracle client model in "
          f"{time.time() - t_gen:.1f} s", file=sys.stderr)
    eng = FlowEngine(device=0, max_batch=max(len(e) for e in host))
    eng.local_load_rules(rules, 2, 1000, 500)
    batches = [torch.from_numpy(e.view(np.uint8).copy()).to(dev) for e in host]
    stream = torch.cuda.current_stream(dev).cuda_stream
    sizes = [len(e) for e in host]
    el = local_timed(eng, batches, sizes, args, dev, stream)
    decided = sum(sizes[args.warmup:])
    touched = int(np.unique(host[-1]["resource"] & 0x7FFFFFFF).size)
    # per event 32 B in + 8 B out; per touched resource: second window 2x128 B, two minute buckets 2x2x64 B,
    # head (threads + two breakers) 2x128 B, rule 80 B
    b_alg = sizes[-1] * (32 + 8) + touched * (2 * 128 + 2 * 2 * 64 + 2 * 128 + 80)
    base = {"value": sum(sizes) / gen_s, "unit": "decisions/s", "cores": 1, "kind": "port",
            "sample": f"the oracle replaying all {sum(sizes)} events while generating them (client model, 1 thread), "
                      f"{gen_s:.1f} s"}
    return {"metric": "local flow + circuit-breaker decisions/sec (entries + exits), 1M resources",
            "workload": "C5: 1M resources x (QPS FlowRule + RT breaker + exception-ratio breaker), minute window, "
                        "16M entries/batch + exits of passed entries",
            "value": decided / el, "el": el, "n": decided // args.steps, "b_alg": b_alg, "touched": touched,
            "cpu": base, "data": "synthetic (seeded): Zipf(1.0) resources, rt lognormal(2.5, 0.8) ms, 5% errors; "
                                 "exits generated by the oracle client model"}


def slot(args, dev):
    """The whole slot chain at C5 size (sg_slot_decide_batch: ParamFlowSlot -> FlowSlot -> DegradeSlot inside
    StatisticSlot), with 10 % of the 1M resources off the fast walkers' single-DefaultController shape: a third carry an
    origin-limitApp rule beside their default rule (their callers pass an origin: 70 % of their entries, U{1..4}), a
    third a WarmUp rule (warmUpPeriodSec 10, coldFactor 3), a third a ParamFlowRule on argument 0 (QPS, count U{5..20},
    1 s; the argument one of 1000 values, Zipf 1.1). Every resource keeps C5's RT and exception-ratio breakers. Those
    resources go through the cx walker (k_lwalk_cx); with Zipf(1.0) popularity some of the hottest are among them.
    Entries + the exits of passed entries (the oracle's client model, as C5); the batches are synchronous (origin
    nodes are created with a host round trip). Every timed batch's results are checked against the oracle."""
    from oracle.binding import LocalChain, LocalTraceGen, ParamFlowSlot, degrade_rule
    K, n = args.resources, args.events
    rng = np.random.default_rng(7)
    base = np.zeros(K, abi.LOCAL_RULE_DTYPE)
    base["flow_grade"] = abi.FLOW_GRADE_NONE
    base["n_breakers"] = 2
    b = np.zeros(2, abi.DEGRADE_RULE_DTYPE)
    b[0] = degrade_rule(abi.DEGRADE_RT, 100, 10, 5, 1000, 0.5)
    b[1] = degrade_rule(abi.DEGRADE_EXCEPTION_RATIO, 0.5, 10, 5, 1000)
    base["breakers"] = b
    kind = np.zeros(K, np.int64)  # 0 plain, 1 origin-limitApp, 2 WarmUp, 3 param rule
    cx = rng.random(K) < 0.10
    kind[cx] = rng.integers(1, 4, int(cx.sum()))
    n_org = int((kind == 1).sum())
    fr = np.zeros(K + n_org, abi.LOCAL_FLOW_RULE_DTYPE)
    fr["resource"][:K] = np.arange(K)
    fr["grade"] = abi.FLOW_GRADE_QPS
    fr["count"][:K] = rng.integers(1, 65, K)
    fr["control_behavior"][:K] = np.where(kind == 2, abi.CONTROL_WARM_UP, abi.CONTROL_DEFAULT)
    fr["limit_app"] = abi.LIMIT_APP_DEFAULT
    fr["strategy"] = abi.STRATEGY_DIRECT
    fr["warm_up_period_sec"] = 10
    fr["max_queueing_ms"] = 500
    fr["ref_resource"] = -1
    fr["cluster_key"] = abi.KEY_NO_RULE
    org_res = np.nonzero(kind == 1)[0]
    fr["resource"][K:] = org_res
    fr["count"][K:] = rng.integers(1, 17, n_org)
    fr["limit_app"][K:] = rng.integers(1, 5, n_org)
    par_res = np.nonzero(kind == 3)[0]
    params = np.zeros(len(par_res), abi.PSLOT_RULE_DTYPE)
    params["resource"] = par_res
    params["param_idx"] = 0
    params["grade"] = abi.FLOW_GRADE_QPS
    params["rule"]["count"] = rng.integers(5, 21, len(par_res))
    params["rule"]["duration_sec"] = 1
    params["rule"]["capacity_log2"] = 11  # exact value table of 2048 slots per rule (1000 values)
    n_vals = 1000
    pargs = np.zeros(n_vals, abi.PSLOT_ARG_DTYPE)
    pargs["value_begin"] = np.arange(n_vals)
    pargs["value_count"] = 1
    pargs["kind"] = abi.ARG_VALUE
    values = np.arange(1, n_vals + 1, dtype=np.uint64)
    vcdf, _ = zipf_cdf(n_vals, 1.1, 8)
    cdf, perm = zipf_cdf(K, 1.0, 7)
    ora = LocalChain(2, 1000, 500)
    ora.load_rules(base)
    kept = ora.load_flow_rules(fr, 4, 0)
    ps = ParamFlowSlot(params, n_resources=K)
    ora.attach_params(ps)
    gen = LocalTraceGen(ora)
    host, wants = [], []
    gen_s = 0.0
    for bt in range(args.warmup + args.steps):
        ent = np.zeros(n, abi.LOCAL_EVENT_DTYPE)
        ent["ts_ms"] = T0 + 1000 * bt + np.sort(rng.integers(0, 1000, n))
        res = perm[np.minimum(np.searchsorted(cdf, rng.random(n), side="right"), K - 1)]
        ent["resource"] = res
        ent["count"] = 1
        og = rng.integers(1, 5, n).astype(np.int32)
        og[(kind[res] != 1) | (rng.random(n) < 0.3)] = 0
        ent["origin"] = og
        ext = np.zeros(n, abi.SLOT_EXT_DTYPE)
        ext["args_null"] = (kind[res] != 3).astype(np.int32)
        ext["arg_begin"] = np.minimum(np.searchsorted(vcdf, rng.random(n), side="right"), n_vals - 1)
        ext["arg_count"] = 1
        rt = np.minimum(np.round(np.exp(rng.normal(2.5, 0.8, n))), 10_000).astype(np.int32)
        err = (rng.random(n) < 0.05).astype(np.uint8)
        t = time.perf_counter()
        ev, xo, want = gen.run_ext(ent, ext, rt, err, T0 + 1000 * (bt + 1), pargs, values)
        gen_s += time.perf_counter() - t
        host.append((ev, xo))
        wants.append(want)
        print(f"# slot trace batch {bt}: {len(ev)} events, {gen_s:.1f} s so far", file=sys.stderr, flush=True)
    print(f"# slot trace: {sum(len(e) for e, _ in host)} events generated by the oracle client model in {gen_s:.1f} s",
          file=sys.stderr)
    eng = FlowEngine(device=0, max_batch=max(len(e) for e, _ in host))
    eng.local_load_rules(base, 2, 1000, 500)
    assert eng.local_load_flow_rules(fr, 4, 0) == kept
    eng.pslot_load_rules(params, n_resources=K)
    d_args = torch.from_numpy(pargs.view(np.uint8).copy()).to(dev)
    d_vals = torch.from_numpy(values.view(np.uint8).copy()).to(dev)
    evs = [torch.from_numpy(e.view(np.uint8).copy()).to(dev) for e, _ in host]
    exs = [torch.from_numpy(x.view(np.uint8).copy()).to(dev) for _, x in host]
    sizes = [len(e) for e, _ in host]
    outs = [torch.empty(sz * 8, dtype=torch.uint8, device=dev) for sz in sizes]
    stream = torch.cuda.current_stream(dev).cuda_stream
    el = timed(lambda i: eng.slot_decide_device(evs[i].data_ptr(), exs[i].data_ptr(), sizes[i], d_args.data_ptr(),
                                                n_vals, d_vals.data_ptr(), n_vals, outs[i].data_ptr(), stream),
               args.warmup, args.steps)
    if int(os.environ.get("SG_DEBUG", "0")) & 64:  # the cx wave walker's counters (local.hip cx_wave), per batch
        d = eng.debug_copy(5, np.uint64, 128).astype(np.int64)
        nb = len(sizes)
        print("# cxw per batch: segments %.0f, wave-ms sum %.2f max %.2f, dead chunks %.0f, general chunks %.0f, "
              "serial entries %.0f exits %.0f, dead-chunk ms %.2f, serial ms %.2f" % (
                  d[20] / nb, d[21] / nb / 1e5, d[22] / 1e5, d[23] / nb, d[24] / nb, d[25] / nb, d[26] / nb,
                  d[27] / nb / 1e5, d[28] / nb / 1e5), file=sys.stderr, flush=True)
        print("# cxw dead-chunk head ms per batch: %.2f" % (d[17] / nb / 1e5), file=sys.stderr, flush=True)
        print("# cxw param dead loop phases ms per batch: prefetch+fixup %.2f, chains %.2f, stores %.2f" % (
            d[12] / nb / 1e5, d[13] / nb / 1e5, d[14] / nb / 1e5), file=sys.stderr, flush=True)
        print("# cxw segments over 5 ms per batch: %.1f; their serial steps %.0f (%.2f ms), dead chunks %.0f" % (
            d[19] / nb, d[29] / nb, d[30] / nb / 1e5, d[31] / nb), file=sys.stderr, flush=True)
        for sl in range(min(12, int(d[18]))):
            o = d[32 + 8 * sl: 40 + 8 * sl]
            print("#   segment: resource %d records %d wave-ms %.2f dead-ms %.2f dead chunks %d serial %d (%.2f ms) "
                  "param rule %d" % (o[0], o[1], o[2] / 1e5, o[3] / 1e5, o[4], o[5], o[6] / 1e5, o[7]),
                  file=sys.stderr, flush=True)
    for i in range(len(sizes)):  # full-size parity of every batch
        got = outs[i].cpu().numpy().view(abi.LOCAL_RES_DTYPE)
        if not np.array_equal(got, wants[i]):
            bad = np.nonzero(got != wants[i])[0]
            raise AssertionError(f"slot batch {i}: {len(bad)} results differ from the oracle (first at {bad[0]})")
    decided = sum(sizes[args.warmup:])
    last = host[-1][0]
    touched = int(np.unique(last["resource"] & 0x7FFFFFFF).size)
    hot = perm[:1000]
    b_alg = sizes[-1] * (32 + 16 + 8) + touched * (2 * 128 + 2 * 2 * 64 + 2 * 128 + 80)  # C5's bytes + the ext
    base_cpu = {"value": sum(sizes) / gen_s, "unit": "decisions/s", "cores": 1, "kind": "port",
                "sample": f"the oracle replaying all {sum(sizes)} events while generating them (client model, 1 thread), "
                          f"{gen_s:.1f} s"}
    return {"metric": "slot-chain decisions/sec (entries + exits), 1M resources, 10 % origin / WarmUp / param rules",
            "workload": "slot: C5 (1M resources, QPS FlowRule + RT + exception-ratio breakers, 16M entries/batch + exits) "
                        "with 10 % of resources carrying an origin-limitApp rule, a WarmUp rule or a ParamFlowRule",
            "value": decided / el, "el": el, "n": decided // args.steps, "b_alg": b_alg, "touched": touched,
            "cpu": base_cpu,
            "extra": {"cx_resources": int(cx.sum()), "cx_among_hottest_1000": int(cx[hot].sum()),
                      "cx_share_of_entries": float(np.isin(last["resource"] & 0x7FFFFFFF,
                                                            np.nonzero(cx)[0])[last["kind"] == 0].mean()),
                      "parity": "every batch equal to the oracle"},
            "data": "synthetic (seeded): Zipf(1.0) resources, rt lognormal(2.5, 0.8) ms, 5% errors; exits generated by "
                    "the oracle client model"}


def codec(args, dev):
    """Token-server step from the wire: 16M MSG_TYPE_FLOW frames (the C3 traffic, 1M flowIds, Zipf 1.0)
    → sg_codec_decode_flow → sg_flow_decide_batch → sg_codec_encode_flow, all resident in HBM."""
    import bench
    from sentinel_amd.engine import FlowEngine
    n = args.events
    wl = bench.ShardWorkload(args.resources, n, 0, 1, dev)
    fid_t = torch.from_numpy(wl.rules["flow_id"].astype(np.int64)).to(dev)
    FB = 18  # [i32 xid][u8 type][i64 flowId][i32 count][bool prio]

    def be(x, nbytes):  # int64 tensor → big-endian bytes [n, nbytes]
        return torch.stack([(x >> (8 * (nbytes - 1 - j))) & 0xFF for j in range(nbytes)], dim=1).to(torch.uint8)

    def frames(b):
        req = wl.batch(b).view(torch.int64).reshape(-1, 2)
        ts, kw = req[:, 0].contiguous(), req[:, 1]
        key, acq = kw & 0x7FFFFFFF, (kw >> 32) & 0xFFFFFFFF
        prio = (kw >> 31) & 1
        xid = torch.arange(n, device=dev, dtype=torch.int64) + b * n
        pay = torch.cat([be(xid, 4), torch.ones((n, 1), dtype=torch.uint8, device=dev), be(fid_t[key], 8),
                         be(acq, 4), prio.to(torch.uint8).reshape(-1, 1)], dim=1).reshape(-1).contiguous()
        return pay, ts

    eng = FlowEngine(device=0, max_batch=n)
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    ns["max_allowed_qps"] = 30000
    eng.set_namespaces(ns)
    eng.load_rules(wl.rules)
    batches = [frames(b) for b in range(args.warmup + args.steps)]
    offsets = (torch.arange(n + 1, device=dev, dtype=torch.int64) * FB).to(torch.int32)
    req = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    xid = torch.empty(n * 4, dtype=torch.uint8, device=dev)
    kind = torch.empty(n, dtype=torch.uint8, device=dev)
    res = torch.empty(n * 12, dtype=torch.uint8, device=dev)
    out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    s = stream.cuda_stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    t_codec = [0.0, 0.0]

    def step(b, timed_codec=False):
        pay, ts = batches[b]
        ev[0].record(stream)
        eng.codec_decode(pay.data_ptr(), offsets.data_ptr(), ts.data_ptr(), n, req.data_ptr(), xid.data_ptr(),
                         kind.data_ptr(), s)
        ev[1].record(stream)
        eng.decide_device(req.data_ptr(), n, res.data_ptr(), s)
        ev[2].record(stream)
        eng.codec_encode(xid.data_ptr(), kind.data_ptr(), res.data_ptr(), n, out.data_ptr(), s)
        ev[3].record(stream)
        if timed_codec:
            ev[3].synchronize()
            t_codec[0] += ev[0].elapsed_time(ev[1])
            t_codec[1] += ev[2].elapsed_time(ev[3])

    el = timed(lambda b: step(b, b >= args.warmup), args.warmup, args.steps)
    dec_ms, enc_ms = t_codec[0] / args.steps, t_codec[1] / args.steps
    dec_b, enc_b = n * (FB + 4 + 8 + 16 + 4 + 1), n * (4 + 1 + 12 + 16)
    touched = int(torch.unique(batches[-1][0].reshape(-1, FB)[:, 5:13].contiguous().view(torch.int64)).numel())
    b_alg = n * (FB + 4 + 16) + touched * (bench.STATE_B + bench.RULE_B)  # frames in/out + the C3 state
    base = None
    if not args.no_cpu_baseline:
        from oracle import binding
        from oracle.binding import ClusterTokenService
        m = min(args.cpu_events, n)
        pay, ts = batches[0]
        pay_h = pay[: m * FB].cpu().numpy()
        off_h = np.arange(m + 1, dtype=np.uint32) * FB
        ts_h = ts[:m].cpu().numpy()
        ora = ClusterTokenService()
        ora.set_namespaces(ns)
        ora.load_rules(wl.rules)
        t = time.perf_counter()
        r_h, x_h, k_h = binding.codec_decode_flow(pay_h, off_h, ts_h, wl.rules["flow_id"])
        binding.codec_encode_flow(x_h, k_h, ora.decide(r_h))
        dt = time.perf_counter() - t
        base = {"value": m / dt, "unit": "frames/s", "cores": 1, "kind": "port",
                "sample": f"first {m} frames of batch 0 through the oracle codec + ClusterTokenService (1 thread), {dt:.1f} s"}
    return {"metric": "token-server frames/sec (decode + decide + encode), 1M flowIds",
            "workload": "C3 traffic as MSG_TYPE_FLOW frames: sg_codec_decode_flow -> sg_flow_decide_batch -> "
                        "sg_codec_encode_flow, 16M frames per 1000 ms batch",
            "value": n * args.steps / el, "el": el, "n": n, "b_alg": b_alg, "touched": touched, "cpu": base,
            "unit": "frames/s", "dtype": "u8",
            "extra": {"codec_kernels": {"decode_ms": dec_ms, "encode_ms": enc_ms,
                                        "decode_gbs": dec_b / dec_ms / 1e6, "encode_gbs": enc_b / enc_ms / 1e6,
                                        "decode_frac": dec_b / dec_ms / 1e6 / HBM_PEAK_GBS,
                                        "encode_frac": enc_b / enc_ms / 1e6 / HBM_PEAK_GBS,
                                        "bytes_per_frame": {"decode": dec_b // n, "encode": enc_b // n}}},
            "data": "synthetic (GPU-generated, seeded): the bench.py C3 trace encoded as big-endian flow frames"}


def pace(args, dev):
    K, n = args.resources, args.events
    rng = np.random.default_rng(6)
    rules = np.zeros(K, abi.PACE_RULE_DTYPE)
    rules["count"] = rng.integers(1, 65, K).astype(np.float64)
    rules["max_queueing_ms"] = 500
    cdf, perm = zipf_cdf(K, 1.0, 6)
    cdf_t, perm_t = torch.from_numpy(cdf).to(dev), torch.from_numpy(perm.astype(np.int64)).to(dev)
    gen = torch.Generator(device=dev).manual_seed(6)

    def batch(b):
        w = torch.zeros((n, 2), dtype=torch.int64, device=dev)
        w[:, 0] = torch.sort(torch.randint(0, 1000, (n,), generator=gen, device=dev)).values + T0 + 1000 * b
        acq = torch.where(torch.rand(n, generator=gen, device=dev) < 0.1,
                          torch.randint(2, 5, (n,), generator=gen, device=dev), torch.ones(n, dtype=torch.int64, device=dev))
        w[:, 1] = gpu_keys(cdf_t, perm_t, n, gen) | (acq << 32)       # rule | acquireCount << 32
        return w.view(torch.uint8).reshape(-1)

    eng = FlowEngine(device=0, max_batch=n)
    eng.pace_load_rules(rules)
    batches = [batch(b) for b in range(args.warmup + args.steps)]
    out = torch.empty(n * 4, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    el = timed(lambda b: eng.pace_decide_device(batches[b].data_ptr(), n, out.data_ptr(), stream), args.warmup, args.steps)
    touched = int(torch.unique(batches[-1].view(torch.int64).reshape(-1, 2)[:, 1] & 0xFFFFFFFF).numel())
    b_alg = n * (16 + 4) + touched * (16 + 2 * 8)   # request in, wait out; per rule: rule 16 B, latest read + write
    base = None
    if not args.no_cpu_baseline:
        from oracle.binding import RateLimiterController
        req = batches[0].view(torch.int64).reshape(-1, 2)[: args.cpu_events].cpu().numpy().copy().view(abi.PACE_REQ_DTYPE).reshape(-1)
        ora = RateLimiterController(rules)
        t = time.perf_counter()
        ora.decide(req)
        dt = time.perf_counter() - t
        base = {"value": len(req) / dt, "unit": "decisions/s", "cores": 1, "kind": "port",
                "sample": f"first {len(req)} requests of batch 0 through oracle RateLimiterController (1 thread), {dt:.1f} s"}
    return {"metric": "pace decisions/sec (RateLimiterController.canPass), 1M rate-limited resources",
            "workload": "pace: 1M RATE_LIMITER FlowRules count U{1..64} maxQueueing 500 ms, 16M canPass/batch",
            "value": n * args.steps / el, "el": el, "n": n, "b_alg": b_alg, "touched": touched, "cpu": base,
            "data": "synthetic (GPU-generated, seeded): Zipf(1.0) resources, 10% acquire U{2..4}"}


def cparam(args, dev):
    """Cluster hot-parameter tokens: 1000 ClusterParamFlowRules (GLOBAL, count U{1..40}, S=10 / 1000 ms), rules
    Zipf(1.0), each rule's values Zipf(1.1) over 50k distinct u64, 16M requests per 1000 ms batch, 10 % of them
    carrying 2-3 values (all-or-nothing)."""
    R, n, V = 1000, args.events, 50_000
    rng = np.random.default_rng(7)
    rules = np.zeros(R, abi.CPARAM_RULE_DTYPE)
    rules["flow_id"] = np.arange(R) + 1
    rules["count"] = rng.integers(1, 41, R)
    rules["threshold_type"] = abi.THRESHOLD_GLOBAL
    rules["sample_count"], rules["window_interval_ms"] = 10, 1000
    if args.chain:
        rules["count"][0] = 1
    rcdf, rperm = zipf_cdf(R, 1.0, 7)
    vcdf, vperm = zipf_cdf(V, 1.1, 8)
    rcdf_t, rperm_t = torch.from_numpy(rcdf).to(dev), torch.from_numpy(rperm.astype(np.int64)).to(dev)
    vcdf_t, vperm_t = torch.from_numpy(vcdf).to(dev), torch.from_numpy(vperm.astype(np.int64)).to(dev)
    gen = torch.Generator(device=dev).manual_seed(7)

    def batch(b):
        w = torch.zeros((n, 3), dtype=torch.int64, device=dev)
        w[:, 0] = torch.sort(torch.randint(0, 1000, (n,), generator=gen, device=dev)).values + T0 + 1000 * b
        key = gpu_keys(rcdf_t, rperm_t, n, gen)
        cnt = torch.where(torch.rand(n, generator=gen, device=dev) < 0.1,
                          torch.randint(2, 4, (n,), generator=gen, device=dev), torch.ones(n, dtype=torch.int64, device=dev))
        if args.chain:  # chain link k at request k * n / L: rule 0 (threshold 1), values (c_k, c_k+1)
            ci = torch.arange(args.chain, device=dev) * (n // args.chain)
            key[ci] = 0
            cnt[ci] = 2
        begin = torch.cumsum(cnt, 0) - cnt
        w[:, 1] = key | (1 << 32)                     # key, acquireCount 1
        w[:, 2] = begin | (cnt << 32)                 # value_begin, value_count
        nv = int(cnt.sum())
        owner = torch.repeat_interleave(key, cnt)
        vals = gpu_keys(vcdf_t, vperm_t, nv, gen) * 0x9E3779B1 + owner * 0x85EBCA77 + 11
        if args.chain:
            c = (0x5C4A << 48) + b * (args.chain + 1) + torch.arange(args.chain + 1, device=dev)
            vals[begin[ci]] = c[:-1]
            vals[begin[ci] + 1] = c[1:]
        return w.view(torch.uint8).reshape(-1), vals, nv

    batches = [batch(b) for b in range(args.warmup + args.steps)]
    max_nv = max(x[2] for x in batches)
    G = args.shards  # --shards G: the node handle's sharded param path (sg_node_cparam_*), G shards on this GPU
    if G:
        from sentinel_amd.engine import NodeEngine
        eng = NodeEngine([0] * G, max_batch=max(n, max_nv))
    else:
        eng = FlowEngine(device=0, max_batch=max(n, max_nv))
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    eng.set_namespaces(ns)
    eng.cparam_load_rules(rules, None, 17)
    out = torch.empty(n * 12, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    rounds = []

    def step(b):
        req, vals, nv = batches[b]
        eng.cparam_decide_device(req.data_ptr(), n, vals.data_ptr(), nv, out.data_ptr(), stream)
        if not G:
            rounds.append(eng.cparam_last_rounds())

    el = timed(step, args.warmup, args.steps)
    req_l, vals_l, nv_l = batches[-1]
    keys_l = torch.repeat_interleave(req_l.view(torch.int64).reshape(-1, 3)[:, 1] & 0xFFFFFFFF,
                                     (req_l.view(torch.int64).reshape(-1, 3)[:, 2] >> 32))
    touched = int(torch.unique(keys_l * 1_000_003 + vals_l).numel())
    # per request 24 B in + 12 B out; per value 8 B; per touched (rule, value) slot: key 8 B + ring S x 16 B read
    # and written once
    b_alg = n * (24 + 12) + nv_l * 8 + touched * (8 + 2 * 10 * 16)
    base = None
    if not args.no_cpu_baseline:
        from oracle.binding import ClusterTokenService
        m = min(args.cpu_events, n)
        req0, vals0, _ = batches[0]
        req_h = req0.view(torch.int64).reshape(-1, 3)[:m].cpu().numpy().copy().view(abi.CPARAM_REQ_DTYPE).reshape(-1)
        end = int(req_h["value_begin"][-1]) + int(req_h["value_count"][-1])
        vals_h = vals0[:end].cpu().numpy().astype(np.uint64)
        ora = ClusterTokenService()
        ora.set_namespaces(ns)
        ora.load_param_rules(rules)
        t = time.perf_counter()
        ora.decide_param(req_h, vals_h)
        dt = time.perf_counter() - t
        base = {"value": m / dt, "unit": "decisions/s", "cores": 1, "kind": "port",
                "sample": f"first {m} requests of batch 0 through oracle ClusterTokenService.decide_param (1 thread), "
                          f"{dt:.1f} s"}
    return {"metric": "cluster hot-parameter token decisions/sec (ClusterParamFlowChecker), 1000 param rules"
                      + (f", node handle with {G} shards on one GPU (routing inside)" if G else ""),
            "workload": "cparam: 1000 ClusterParamFlowRules x 50k values Zipf(1.1), 16M requests/batch, 10% multi-value"
                        + (f", a {args.chain}-deep two-value dependency chain per batch (rule 0, threshold 1)" if args.chain else "")
                        + (f", sg_node_cparam_decide_batch over {G} same-device shards" if G else ""),
            "value": n * args.steps / el, "el": el, "n": n, "b_alg": b_alg, "touched": touched, "cpu": base,
            "extra": {"fixed_point_rounds": rounds[args.warmup:], "values_per_step": nv_l, "shards": G},
            "data": "synthetic (GPU-generated, seeded): rules Zipf(1.0), values Zipf(1.1) per rule, 10% 2-3 values"}


def node(args, dev):
    """The node handle (sg_node_*) on one GPU: the C3 workload (1M flowIds, 16M requests per 1000 ms batch) decided
    by G same-device shard handles with the routing inside the library — validation and the namespace limiters on the
    front handle, the stable multisplit by splitmix64(flowId) mod G, every shard's sort and walkers — through the node
    pipeline (sg_node_flow_enqueue: the front's part of batch i+1 and the shards' sorts beside the shards' walkers of
    batch i, at most two batches in flight), against one handle's pipeline (sg_flow_enqueue) on the same batches;
    --local-sync: both synchronous (sg_node_flow_decide_batch / sg_flow_decide_batch)."""
    import bench
    from sentinel_amd.engine import NodeEngine
    G = args.shards or 2
    wl = bench.ShardWorkload(1_000_000, args.events, 0, 1, dev)
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    nd = NodeEngine([0] * G, max_batch=args.events)
    nd.set_namespaces(ns)
    nd.load_rules(wl.rules)
    one = FlowEngine(device=0, max_batch=args.events)
    one.set_namespaces(ns)
    one.load_rules(wl.rules)
    batches = [wl.batch(b) for b in range(args.warmup + args.steps)]
    outs = [torch.empty(args.events * 12, dtype=torch.uint8, device=dev) for _ in range(2)]
    stream = torch.cuda.current_stream(dev).cuda_stream

    def run(eng, bs, sync):
        if sync:
            return timed(lambda b: eng.decide_device(bs[b].data_ptr(), args.events, outs[0].data_ptr(), stream),
                         args.warmup, args.steps)
        tickets = []

        def step(b):
            if len(tickets) >= 2:
                eng.wait(tickets.pop(0))
            tickets.append(eng.enqueue_device(bs[b].data_ptr(), args.events, outs[b % 2].data_ptr()))
        torch.cuda.synchronize()
        el = timed(step, args.warmup, args.steps)
        for t in tickets:
            eng.wait(t)
        return el

    el = run(nd, batches, args.local_sync)
    # the single handle on the same batches, later in time (each batch shifted past the node's last)
    later = [b.clone() for b in batches]
    for x in later:
        x.view(torch.int64).view(-1, 2)[:, 0] += 1000 * (args.warmup + args.steps)
    el1 = run(one, later, args.local_sync)
    n = args.events
    keys = batches[-1].view(torch.int64).view(-1, 2)[:, 1] & 0x7FFFFFFF
    touched = int(torch.unique(keys).numel())
    b_alg = n * (bench.REQ_B + bench.RES_B) + touched * (bench.STATE_B + bench.RULE_B)  # bench.py's C3 bytes
    mode = "synchronous" if args.local_sync else "pipelined"
    return {"metric": f"flow decisions/sec through the node handle, {G} shards on one GPU (routing inside)",
            "workload": f"C3 workload (1M flowIds, 16M requests/batch, Zipf 1.0) on sg_node with {G} same-device "
                        f"shards, {mode} node batches",
            "value": n * args.steps / el, "el": el, "n": n, "b_alg": b_alg, "touched": touched, "cpu": None,
            "extra": {"shards": G, "mode": mode, "single_handle_ms_per_step": el1 / args.steps * 1e3,
                      "single_handle_decisions_per_s": n * args.steps / el1,
                      "node_over_single": el / el1},
            "data": "synthetic (GPU-generated, seeded): bench.py's C3 batches"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["c2", "c4", "c5", "codec", "pace", "cparam", "node", "slot"], default="c2")
    ap.add_argument("--shards", type=int, default=0,
                    help="node: shard handles on the one GPU (default 2); cparam: decide through the node handle "
                         "with this many shards (default: one handle)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--events", type=int, default=16_000_000)
    ap.add_argument("--resources", type=int, default=1_000_000)
    ap.add_argument("--cpu-events", type=int, default=4_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--local-sync", action="store_true",
                    help="c2 / c5: time the synchronous sg_local_decide_batch instead of the sg_local_enqueue pipeline")
    ap.add_argument("--chain", type=int, default=0,
                    help="cparam: embed a chain of this many two-value requests per batch, each sharing a value with "
                         "the next under a threshold of one (adversarial: one link per fixed-point round)")
    ap.add_argument("--pmc-summary", default=None,
                    help="scripts/pmc_summary.py output of this workload's FETCH_SIZE / WRITE_SIZE passes (roofline traffic)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    r = {"c2": c2, "c4": c4, "c5": c5, "codec": codec, "pace": pace, "cparam": cparam, "node": node,
         "slot": slot}[args.workload](args, dev)
    ms = r["el"] * 1000.0 / args.steps
    gbs = r["b_alg"] / (ms / 1000.0) / 1e9
    res = {"metric": r["metric"], "value": r["value"], "unit": r.get("unit", "decisions/s"), "n_gpus": 1,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": r.get("dtype", "int64"), "data": r["data"],
           "config": {"workload": r["workload"], "decisions_per_step": r["n"], "touched_keys": r["touched"]},
           "roofline": {"bound": "hbm", "kernel": "whole batch pipeline, wall time per step", "achieved": gbs,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "traffic": None,
                        "algorithmic_bytes_per_step": r["b_alg"]}}
    if args.pmc_summary and os.path.exists(args.pmc_summary):
        res["roofline"]["traffic"] = json.load(open(args.pmc_summary)).get("pipeline_bytes_per_step")
        res["roofline"]["traffic_source"] = args.pmc_summary
    res.update(r.get("extra", {}))
    if r["cpu"] is not None:
        res["cpu_baseline"] = r["cpu"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
