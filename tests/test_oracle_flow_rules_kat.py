"""Known-answer tests of the local chain's flow-rule layer in the oracle: several rules per resource,
limitApp node selection, rule order and the warm-up / rate-limiter controllers. Each restates a test the
reference holds:

  WarmUpControllerTest.testWarmUp            sentinel-core/src/test/.../flow/controller/WarmUpControllerTest.java:33-63
  WarmUpRateLimiterControllerTest.{testPace, testPaceCanNotPass}   …/controller/WarmUpRateLimiterControllerTest.java:33-66
  FlowRuleCheckerTest (limitApp selection)   sentinel-core/src/test/.../flow/FlowRuleCheckerTest.java:40-175
  FlowRuleComparatorTest.testFlowRuleComparator                    …/flow/FlowRuleComparatorTest.java:33-52
  FlowPartialIntegrationTest.{testQPSGrade, testThreadGrade, testOriginFlowRule, testFlowRule_other, testStrategy}
                                             sentinel-core/src/test/.../flow/FlowPartialIntegrationTest.java:48-215

The controller tests mock the node (passQps / previousPassQps) and the clock (AbstractTimeBasedTest, or real
sleeps for testPace): here the controller is driven with explicit values and an explicit clock that advances by
the sleep canPass asks for. Origins are dense ids (appA = 1, appB = 2, …).
"""
import numpy as np
import pytest

from oracle.binding import Controller, LocalChain, local_flow_rule, local_rule, select_node
from sentinel_amd import abi

T0S = [1_700_000_000_000, 1_700_000_000_437, 1_650_000_123_999, 86_400_000 * 365 + 17]


@pytest.mark.parametrize("t0", T0S)
def test_warm_up_controller(t0):
    c = Controller(10, 10, 3)
    assert (c.warning_token, c.max_token) == (50, 100)
    t = t0
    assert not c.warm_can_pass(t, 8, 1)          # passQps 8, previousPassQps 1
    assert c.warm_can_pass(t, 1, 1)
    for _ in range(100):                          # previousPassQps 10, 100 x sleep(100)
        t += 100
        c.warm_can_pass(t, 1, 10)
    assert c.warm_can_pass(t, 8, 10)
    assert not c.warm_can_pass(t, 10, 10)


@pytest.mark.parametrize("t0", T0S)
def test_warm_up_rate_limiter_pace(t0):
    c = Controller(10, 10, 3, behavior=abi.CONTROL_WARM_UP_RATE_LIMITER, max_queueing_ms=1000)
    t = t0
    ok, w = c.warm_rl_can_pass(t, 100)
    assert ok
    t += w
    start = t
    for _ in range(10):
        ok, w = c.warm_rl_can_pass(t, 100)
        assert ok
        t += w                                   # Thread.sleep(waitTime) inside canPass
    cost = (t - start) / 10
    assert abs(cost - 100) < 10


@pytest.mark.parametrize("t0", T0S)
def test_warm_up_rate_limiter_cannot_pass(t0):
    c = Controller(10, 10, 3, behavior=abi.CONTROL_WARM_UP_RATE_LIMITER, max_queueing_ms=10)
    assert c.warm_rl_can_pass(t0, 100)[0]
    assert not c.warm_rl_can_pass(t0, 100)[0]


def test_warm_up_token_arithmetic():
    """The constructor's int arithmetic and the cold-factor branch of coolDownTokens (:161-175)."""
    c = Controller(7.5, 3, 4)
    assert c.warning_token == int(3 * 7.5) // 3
    assert c.max_token == c.warning_token + int(2 * 3 * 7.5 / 5.0)
    t = 1_700_000_000_000
    c.warm_can_pass(t, 0, 0)                     # first sync fills to maxToken
    assert c.state()[0] == c.max_token and c.state()[1] == t
    c.warm_can_pass(t + 1000, 0, 1)              # stored > warning and not (1 < (int)7.5 / 4): no refill, - 1
    assert c.state()[0] == c.max_token - 1


def test_select_node_default():
    rules = np.array([local_flow_rule(count=1)])
    assert select_node(rules, 0, 0) == 0
    assert select_node(rules, 0, 3) == 0


def test_select_node_custom_origin():
    appA, appB = 1, 2
    rules = np.array([local_flow_rule(count=1, limit_app=appA)])
    assert select_node(rules, 0, appA) == 1      # origin matches: the origin node
    rules = np.array([local_flow_rule(count=1, limit_app=appB)])
    assert select_node(rules, 0, appA) is None   # mismatch: no node


def test_select_node_other_origin():
    appA, appB = 1, 2
    rules = np.array([local_flow_rule(count=1, limit_app=appA), local_flow_rule(count=2, limit_app=abi.LIMIT_APP_OTHER)])
    assert select_node(rules, 1, appB) == 1      # appB is "other"
    assert select_node(rules, 1, appA) is None   # appA has its own rule
    assert select_node(rules, 1, 0) is None      # no origin: isOtherOrigin("") is false


def test_pass_check_select_empty_node_success():
    ch = LocalChain()
    ch.load_rules(np.array([local_rule()]))
    abc, defo = 1, 2
    assert ch.load_flow_rules(np.array([local_flow_rule(count=1, limit_app=abc)]), n_origins=2) == 1
    t = 1_700_000_000_000
    for i in range(5):
        assert ch.entry(t + i, origin=defo)[0] == abi.LOCAL_PASS


def test_select_node_for_empty_reference():
    """testSelectNodeForEmptyReference: a CHAIN rule without refResource selects no node."""
    rules = np.array([local_flow_rule(count=1, strategy=abi.STRATEGY_CHAIN, ref=-1)])
    assert select_node(rules, 0, 0, context=0) is None


def test_select_node_for_relate_reference():
    """testSelectNodeForRelateReference: RELATE reads refResource's ClusterNode when ClusterBuilderSlot created it
    (the test puts it into the map); without it, no node."""
    rules = np.array([local_flow_rule(count=1, strategy=abi.STRATEGY_RELATE, ref=1)])
    assert select_node(rules, 0, 0, ref_exists=True) == 3
    assert select_node(rules, 0, 0, ref_exists=False) is None


def test_select_reference_node_for_context_entrance():
    """testSelectReferenceNodeForContextEntrance: CHAIN selects the DefaultNode only in the named context."""
    good, other = 5, 6
    rules = np.array([local_flow_rule(count=1, strategy=abi.STRATEGY_CHAIN, ref=good)])
    assert select_node(rules, 0, 0, context=good) == 2
    assert select_node(rules, 0, 0, context=other) is None


def test_select_reference_node_for_origin_rules():
    """A limitApp origin / "other" rule with a reference strategy: the origin match decides whether the reference
    node is looked at at all (selectNodeByRequesterAndStrategy :122-141)."""
    appA, appB, ctx = 1, 2, 3
    rules = np.array([local_flow_rule(count=1, limit_app=appA, strategy=abi.STRATEGY_CHAIN, ref=ctx),
                      local_flow_rule(count=1, limit_app=abi.LIMIT_APP_OTHER, strategy=abi.STRATEGY_RELATE, ref=0)])
    assert select_node(rules, 0, appA, context=ctx) == 2
    assert select_node(rules, 0, appB, context=ctx) is None
    assert select_node(rules, 1, appB) == 3
    assert select_node(rules, 1, appA) is None    # appA has its own rule: not "other"


@pytest.mark.parametrize("t0", T0S)
def test_partial_integration_strategy(t0):
    """FlowPartialIntegrationTest.testStrategy: a DIRECT count-0 rule blocks inside a named context; then the rule is
    replaced by a CHAIN rule of another resource without refResource (invalid, ignored): the entry passes."""
    ch = LocalChain()
    ch.load_rules(np.array([local_rule(), local_rule()]))
    assert ch.load_flow_rules(np.array([local_flow_rule(0, count=0)]), n_contexts=3) == 1
    x = np.zeros(1, abi.SLOT_EXT_DTYPE)
    x["context"], x["args_null"] = 1, 1                           # ContextUtil.enter("testStrategy")
    ev = np.zeros(1, abi.LOCAL_EVENT_DTYPE)
    ev["ts_ms"], ev["count"] = t0, 1
    assert ch.decide_ext(ev, x, [], [])[0]["status"] == abi.LOCAL_BLOCK_FLOW
    assert ch.load_flow_rules(np.array([local_flow_rule(1, count=0, strategy=abi.STRATEGY_CHAIN)]), n_contexts=3) == 0
    x["context"] = 2                                              # ContextUtil.enter("entry1")
    assert ch.decide_ext(ev, x, [], [])[0]["status"] == abi.LOCAL_PASS


@pytest.mark.parametrize("t0", T0S)
def test_chain_rule_reads_the_context_default_node(t0):
    """A CHAIN rule limits the resource's entries through one context only; the DefaultNode of that context counts
    that context's traffic, while the ClusterNode counts every context's."""
    ch = LocalChain()
    ch.load_rules(np.array([local_rule()]))
    assert ch.load_flow_rules(np.array([local_flow_rule(0, count=2, strategy=abi.STRATEGY_CHAIN, ref=1)]),
                              n_contexts=2) == 1
    ev = np.zeros(6, abi.LOCAL_EVENT_DTYPE)
    ev["ts_ms"], ev["count"] = t0, 1
    x = np.zeros(6, abi.SLOT_EXT_DTYPE)
    x["args_null"] = 1
    x["context"] = [1, 0, 1, 0, 1, 0]
    st = ch.decide_ext(ev, x, [], [])["status"].tolist()
    assert st == [abi.LOCAL_PASS, abi.LOCAL_PASS, abi.LOCAL_PASS, abi.LOCAL_PASS, abi.LOCAL_BLOCK_FLOW, abi.LOCAL_PASS]
    assert ch.second_sum(0, t0, 0) == 5 and ch.second_sum(0, t0, 1) == 1
    d1 = ch.context_dump(0, 1)
    assert d1[4] and d1[0][:, 1].sum() == 2 and d1[0][:, 2].sum() == 1 and d1[3] == 2
    d0 = ch.context_dump(0, 0)
    assert d0[0][:, 1].sum() == 3 and d0[3] == 3


@pytest.mark.parametrize("t0", T0S)
def test_relate_rule_reads_the_referenced_cluster_node(t0):
    """A RELATE rule on resource 0 limits it by resource 1's pass QPS; before resource 1's first entry there is no
    ClusterNode (ClusterBuilderSlot), so the rule passes even at count 0."""
    ch = LocalChain()
    ch.load_rules(np.array([local_rule(), local_rule()]))
    assert ch.load_flow_rules(np.array([local_flow_rule(0, count=0, strategy=abi.STRATEGY_RELATE, ref=1)])) == 1
    assert ch.entry(t0, res=0)[0] == abi.LOCAL_PASS          # no ClusterNode of resource 1 yet
    ch.load_flow_rules(np.array([local_flow_rule(0, count=2, strategy=abi.STRATEGY_RELATE, ref=1)]))
    for _ in range(2):
        assert ch.entry(t0, res=1)[0] == abi.LOCAL_PASS      # resource 1: no rule
    assert ch.entry(t0, res=0)[0] == abi.LOCAL_BLOCK_FLOW    # 2 + 1 > 2 on resource 1's node
    assert ch.second_sum(1, t0, 0) == 2 and ch.second_sum(0, t0, 1) == 1
    assert ch.entry(t0 + 1000, res=0)[0] == abi.LOCAL_PASS   # resource 1's second is over


@pytest.mark.parametrize("t0", T0S)
def test_cluster_mode_rules_without_a_token_service(t0):
    """FlowRuleChecker.passClusterCheck on a node that is neither token client nor server: fallbackToLocalOrPass —
    with fallbackToLocalWhenFail the rule is checked locally, without it the rule passes; cluster rules sort after
    local ones (FlowRuleComparator :31-37)."""
    ch = LocalChain()
    ch.load_rules(np.array([local_rule(), local_rule()]))
    rules = np.array([local_flow_rule(0, count=0, cluster_mode=abi.CLUSTER_MODE_NO_FALLBACK, cluster_config=7),
                      local_flow_rule(1, count=1, cluster_mode=abi.CLUSTER_MODE_FALLBACK, cluster_config=8),
                      local_flow_rule(1, count=5),
                      local_flow_rule(0, count=1, cluster_mode=abi.CLUSTER_MODE_INVALID)])
    assert ch.load_flow_rules(rules) == 3
    assert ch.rule_order(1) == [2, 1]
    assert ch.entry(t0, res=0)[0] == abi.LOCAL_PASS          # not activated
    assert ch.entry(t0, res=1)[0] == abi.LOCAL_PASS
    assert ch.entry(t0, res=1)[0] == abi.LOCAL_BLOCK_FLOW    # the fallback's local check (count 1)


def test_flow_rule_comparator_order():
    ch = LocalChain()
    ch.load_rules(np.array([local_rule()]))
    A = local_flow_rule(count=10)
    B = local_flow_rule(limit_app=1)
    C_ = local_flow_rule(limit_app=2)
    D = local_flow_rule(limit_app=abi.LIMIT_APP_OTHER)
    E = local_flow_rule(count=20)
    assert ch.load_flow_rules(np.array([A, B, C_, D, E]), n_origins=2) == 5
    assert ch.rule_order(0) == [1, 2, 3, 0, 4]   # B, C, D, A, E


def test_invalid_and_duplicate_rules_are_ignored():
    ch = LocalChain()
    ch.load_rules(np.array([local_rule(), local_rule()]))
    rules = np.array([local_flow_rule(count=-1),                                       # count < 0
                      local_flow_rule(count=5, behavior=abi.CONTROL_WARM_UP, warm_up_sec=0),
                      local_flow_rule(count=5, behavior=abi.CONTROL_RATE_LIMITER, max_queueing_ms=0),
                      local_flow_rule(count=5),
                      local_flow_rule(count=5),                                        # duplicate (HashSet)
                      local_flow_rule(resource=1, count=3, grade=abi.FLOW_GRADE_THREAD, behavior=7)])
    assert ch.load_flow_rules(rules) == 2
    assert ch.rule_order(0) == [3] and ch.rule_order(1) == [5]
    assert ch.controller(0) is None and ch.controller(4) is None


def _chain(rules, n_res=1, n_origins=0):
    ch = LocalChain()
    ch.load_rules(np.array([local_rule() for _ in range(n_res)]))
    ch.load_flow_rules(np.array(rules), n_origins=n_origins)
    return ch


@pytest.mark.parametrize("t0", T0S)
def test_partial_integration_qps_grade(t0):
    ch = _chain([local_flow_rule(count=1)])
    assert ch.entry(t0)[0] == abi.LOCAL_PASS
    ch.exit(t0, t0)
    assert ch.entry(t0)[0] == abi.LOCAL_BLOCK_FLOW


@pytest.mark.parametrize("t0", T0S)
def test_partial_integration_thread_grade(t0):
    ch = _chain([local_flow_rule(count=1, grade=abi.FLOW_GRADE_THREAD)])
    assert ch.entry(t0)[0] == abi.LOCAL_PASS         # the other thread holds its entry for 100 ms
    assert ch.entry(t0 + 1)[0] == abi.LOCAL_BLOCK_FLOW
    ch.exit(t0 + 100, t0)
    assert ch.entry(t0 + 101)[0] == abi.LOCAL_PASS


@pytest.mark.parametrize("t0", T0S)
def test_partial_integration_origin_flow_rule(t0):
    app1, app2 = 1, 2
    ch = _chain([local_flow_rule(count=0, limit_app=abi.LIMIT_APP_OTHER), local_flow_rule(count=1, limit_app=app2)],
                n_origins=2)
    assert ch.entry(t0, origin=app1)[0] == abi.LOCAL_BLOCK_FLOW
    assert ch.entry(t0, origin=app2)[0] == abi.LOCAL_PASS
    ch.exit(t0, t0, origin=app2)
    # the origin nodes saw their own traffic: app1 one block, app2 one pass and its exit
    s1 = ch.origin_dump(0, app1)
    s2 = ch.origin_dump(0, app2)
    assert s1[4] and s2[4]
    assert s1[0][:, 2].sum() == 1 and s1[0][:, 1].sum() == 0
    assert s2[0][:, 1].sum() == 1 and s2[0][:, 4].sum() == 1 and s2[3] == 0


@pytest.mark.parametrize("t0", T0S)
def test_partial_integration_other_without_origin(t0):
    ch = _chain([local_flow_rule(count=0, limit_app=abi.LIMIT_APP_OTHER)])
    assert ch.entry(t0)[0] == abi.LOCAL_PASS          # no origin: the "other" rule selects no node
    ch.exit(t0, t0)


@pytest.mark.parametrize("t0", T0S)
def test_partial_integration_strategy_direct(t0):
    ch = _chain([local_flow_rule(count=0)])
    assert ch.entry(t0)[0] == abi.LOCAL_BLOCK_FLOW


@pytest.mark.parametrize("t0", T0S)
def test_chain_rate_limiter_records_statistics(t0):
    """A RATE_LIMITER rule inside the chain: its passes (after the returned sleep) reach the StatisticNode."""
    ch = _chain([local_flow_rule(count=10, behavior=abi.CONTROL_RATE_LIMITER, max_queueing_ms=250)])
    waits = [ch.entry(t0)[1] for _ in range(4)]
    assert waits == [0, 100, 200, 0] or waits[:3] == [0, 100, 200]
    st = [ch.entry(t0)[0] for _ in range(2)]
    assert st == [abi.LOCAL_BLOCK_FLOW] * 2
    assert ch.second_sum(0, t0, 0) == 3 and ch.second_sum(0, t0, 1) == 3 and ch.threads(0) == 3


@pytest.mark.parametrize("t0", T0S)
def test_chain_two_rules_first_failure_wins(t0):
    """A rate limiter before a default rule: the limiter's latestPassedTime moves even when the next rule
    blocks (each rule's canPass runs in order until one fails)."""
    ch = _chain([local_flow_rule(count=1, limit_app=1),
                 local_flow_rule(count=1000, behavior=abi.CONTROL_RATE_LIMITER, max_queueing_ms=500)], n_origins=1)
    assert ch.rule_order(0) == [0, 1]
    assert ch.entry(t0, origin=1) == (abi.LOCAL_PASS, 0)
    assert ch.entry(t0 + 5, origin=1)[0] == abi.LOCAL_BLOCK_FLOW   # the origin rule (count 1) blocks first
    assert ch.controller(1)[2] == t0                                  # the limiter did not run
    assert ch.entry(t0 + 5)[0] == abi.LOCAL_PASS                      # no origin: only the limiter
    assert ch.controller(1)[2] == t0 + 5


@pytest.mark.parametrize("t0", T0S)
def test_nodes_created_on_first_entry_whatever_the_rules(t0):
    """ClusterBuilderSlot.entry (ClusterBuilderSlot.java:99-102) gets or creates the origin node of every entry with
    an origin, and NodeSelectorSlot.entry (NodeSelectorSlot.java:156-170) the DefaultNode of every entry's context,
    whether or not a rule reads them; StatisticSlot (StatisticSlot.java:62-69) counts the entry on both. A rule set
    naming no origin and no context still grows them; context tracking cannot start after a batch."""
    ch = LocalChain(2, 1000, 500)
    ch.load_rules(np.array([local_rule(), local_rule()]))
    assert ch.load_flow_rules(np.array([local_flow_rule(0, 100.0)]), n_origins=2, n_contexts=2) == 1
    ev = np.zeros(3, abi.LOCAL_EVENT_DTYPE)
    ev["ts_ms"], ev["resource"], ev["count"], ev["origin"] = t0, [0, 0, 1], [1, 2, 1], [1, 1, 0]
    ext = np.zeros(3, abi.SLOT_EXT_DTYPE)
    ext["context"], ext["args_null"] = [1, 1, 0], 1
    out = ch.decide_ext(ev, ext, np.zeros(1, abi.PSLOT_ARG_DTYPE), np.zeros(1, np.uint64))
    assert out["status"].tolist() == [abi.LOCAL_PASS] * 3
    sec, _, mnt, th, exists = ch.origin_dump(0, 1)
    assert exists and th == 2 and sec[:, 1].sum() == 3 and mnt[:, 1].sum() == 3
    assert not ch.origin_dump(0, 2)[4] and not ch.origin_dump(1, 1)[4]      # resource 1's entry had no origin
    sec, _, _, th, exists = ch.context_dump(0, 1)
    assert exists and th == 2 and sec[:, 1].sum() == 3
    assert not ch.context_dump(0, 0)[4] and ch.context_dump(1, 0)[4]
    ch2 = LocalChain(2, 1000, 500)
    ch2.load_rules(np.array([local_rule()]))
    ch2.load_flow_rules(np.array([local_flow_rule(0, 100.0)]))
    ch2.decide(np.array([(t0, 0, 0, 1, abi.LOCAL_ENTRY, 0)], abi.LOCAL_EVENT_DTYPE))
    with pytest.raises(ValueError, match=str(abi.SG_E_UNSUPPORTED)):
        ch2.load_flow_rules(np.array([local_flow_rule(0, 100.0)]), n_contexts=1)
    assert ch2.load_flow_rules(np.array([local_flow_rule(0, 100.0, limit_app=1)]), n_origins=1) == 1


def _server(count, ns_qps=None, S=2, prio_ratio=1.0):
    from oracle.binding import ClusterTokenService
    cts = ClusterTokenService(1.0, prio_ratio)
    ns = np.zeros(1, abi.NS_DTYPE)
    ns["connected_count"] = 1
    if ns_qps is not None:
        ns["limiter_enabled"], ns["max_allowed_qps"] = 1, ns_qps
    cts.set_namespaces(ns)
    r = np.zeros(1, abi.RULE_DTYPE)
    r["flow_id"], r["count"], r["threshold_type"] = 77, count, abi.THRESHOLD_GLOBAL
    r["sample_count"], r["window_interval_ms"], r["namespace_id"] = S, 1000, 0
    cts.load_rules(r)
    return cts


def _entries(t0, offsets, prio=()):
    ev = np.zeros(len(offsets), abi.LOCAL_EVENT_DTYPE)
    ev["ts_ms"], ev["count"], ev["kind"] = [t0 + o for o in offsets], 1, abi.LOCAL_ENTRY
    for i in prio:
        ev["resource"][i] |= abi.KEY_PRIO
    return ev


@pytest.mark.parametrize("t0", T0S)
def test_embedded_server_token_results(t0):
    """FlowRuleChecker.passClusterCheck on an embedded token server (FlowRuleChecker.java:147-209, pickClusterService →
    EmbeddedClusterTokenServerProvider, DefaultEmbeddedTokenServer.requestToken → DefaultTokenService.requestToken): a
    cluster rule with a global threshold of 2 per second admits the first two entries of a second (OK), blocks the
    third (BLOCKED → FlowException, the local count of 100 is never consulted), and the server's ClusterMetric holds
    the passes and the block; a prioritized entry that can occupy the next bucket passes after SHOULD_WAIT's 500 ms
    (1000 / sampleCount, ClusterMetric.java:86)."""
    t0 = t0 - t0 % 1000 + 100
    cts = _server(2.0)
    ch = LocalChain(2, 1000, 500)
    ch.load_rules(np.array([local_rule()]))
    rule = local_flow_rule(0, 100.0, cluster_mode=abi.CLUSTER_MODE_FALLBACK, cluster_config=1, cluster_key=0)
    assert ch.load_flow_rules(np.array([rule])) == 1
    ch.attach_cluster(cts, abi.CLUSTER_SERVER)
    out = ch.decide(_entries(t0, [0, 1, 2]))
    assert out["status"].tolist() == [abi.LOCAL_PASS, abi.LOCAL_PASS, abi.LOCAL_BLOCK_FLOW]
    starts, c, occ = cts.read_state(0)
    assert c[:, abi.EV_PASS].sum() == 2 and c[:, abi.EV_BLOCK].sum() == 1
    # t0 + 600: the bucket of t0 + 100 is the window's head (PASS 2); occupying the next bucket fits
    out = ch.decide(_entries(t0, [600], prio=[0]))
    assert (out["status"][0], out["wait_ms"][0]) == (abi.LOCAL_PASS, 500)
    assert cts.read_state(0)[2].tolist() == [1, 1]          # occupied PASS, PASS_REQUEST


@pytest.mark.parametrize("t0", T0S)
def test_embedded_server_fallbacks(t0):
    """applyTokenResult (:186-209): NO_RULE_EXISTS (the flowId has no cluster rule on the server), BAD_REQUEST
    (acquireCount 0) and TOO_MANY_REQUEST (the namespace's GlobalRequestLimiter) fall back to the local check when
    fallbackToLocalWhenFail, else the rule passes; NOT_STARTED (no token service) always falls back."""
    t0 = t0 - t0 % 1000 + 100
    ch = LocalChain(2, 1000, 500)
    ch.load_rules(np.array([local_rule(), local_rule(), local_rule()]))
    rules = [local_flow_rule(0, 1.0, cluster_mode=abi.CLUSTER_MODE_FALLBACK, cluster_config=1),          # no rule
             local_flow_rule(1, 1.0, cluster_mode=abi.CLUSTER_MODE_NO_FALLBACK, cluster_config=2),       # no rule
             local_flow_rule(2, 1.0, cluster_mode=abi.CLUSTER_MODE_FALLBACK, cluster_config=3, cluster_key=0)]
    assert ch.load_flow_rules(np.array(rules)) == 3
    cts = _server(10.0, ns_qps=1.0)           # the namespace admits one token request per second
    ch.attach_cluster(cts, abi.CLUSTER_SERVER)
    ev = _entries(t0, [0, 1, 2, 3, 4, 5, 6])
    ev["resource"] = [0, 0, 1, 1, 2, 2, 2]
    out = ch.decide(ev)
    # resource 0: local count 1 → pass, block; resource 1: not activated; resource 2: the token passes, then
    # TOO_MANY_REQUEST twice → the local check (count 1, one pass in the window) blocks
    assert out["status"].tolist() == [abi.LOCAL_PASS, abi.LOCAL_BLOCK_FLOW, abi.LOCAL_PASS, abi.LOCAL_PASS,
                                      abi.LOCAL_PASS, abi.LOCAL_BLOCK_FLOW, abi.LOCAL_BLOCK_FLOW]
    ch.attach_cluster(None, abi.CLUSTER_NOT_STARTED)
    ev2 = _entries(t0 + 2000, [0, 1])
    ev2["resource"] = 2
    assert ch.decide(ev2)["status"].tolist() == [abi.LOCAL_PASS, abi.LOCAL_BLOCK_FLOW]
    with pytest.raises(ValueError):
        ch.attach_cluster(cts, abi.CLUSTER_CLIENT)
