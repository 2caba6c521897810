"""Local rule graph: FlowRuleChecker with every limitApp and strategy over the
ClusterNode / origin node / DefaultNode graph the slot chain builds.

Oracle KATs (CPU) restate the reference's own FlowRuleCheckerTest (selectNodeByRequesterAndStrategy /
selectReferenceNode / canPassCheck, FlowRuleCheckerTest.java:41-180) and FlowRuleComparatorTest
(FlowRuleComparatorTest.java:19-37) as observable admissions: which node a rule reads shows in which
entries it blocks.  The GPU path (k_lgraph_*) is checked against the oracle on seeded traces with
RELATE cycles, CHAIN contexts, origins, prioritized entries and exits."""
import numpy as np
import pytest

from sentinel_amd import trace as T

DEFAULT, OTHER = 0, 1
DIRECT, RELATE, CHAIN = 0, 1, 2
THREAD, QPS = 0, 1
CLUSTER, ORIGIN, DNODE = 0, 1, 2
PRIO, EXIT, ERROR = 1, 2, 4
APP_A, APP_B, APP_C = 2, 3, 4


def rule(res, count, grade=QPS, strategy=DIRECT, limit_app=DEFAULT, ref=-1):
    return (res, grade, float(count), strategy, limit_app, ref, 0)


class Graph:
    """The oracle graph with a dense numbering of (resource, origin) and (context, resource) nodes,
    as the caller of the C ABI keeps it."""

    def __init__(self, oracle_mod, rules, n_res, origins=(-1, 0, 1, APP_A, APP_B, APP_C), contexts=(0, 1, 2)):
        self.onode = {(r, o): i for i, (r, o) in enumerate((r, o) for r in range(n_res) for o in origins if o >= 0)}
        self.dnode = {(c, r): i for i, (c, r) in enumerate((c, r) for c in contexts for r in range(n_res))}
        self.g = oracle_mod.LocalGraph(rules, n_res, len(self.onode), len(self.dnode))
        self.t = T.T0_ALIGNED

    def ctx(self, res, origin=-1, context=0):
        return (origin, self.onode.get((res, origin), 0), context, self.dnode[(context, res)])

    def entry(self, res, origin=-1, context=0, acquire=1, prio=False, dt=1):
        self.t += dt
        st, w = self.g.replay([res], [acquire], [self.t], [self.ctx(res, origin, context)], [PRIO if prio else 0])
        return int(st[0]) == 0

    def node(self, kind, idx):
        return self.g.node_metrics(kind, idx, self.t)


def test_default_limit_app_selects_cluster_node(oracle_mod):
    """testDefaultLimitAppFlowSelectNode: limitApp "default" + DIRECT -> the ClusterNode, shared by
    every context's DefaultNode of the resource."""
    G = Graph(oracle_mod, [rule(0, 1)], 1)
    assert G.entry(0, context=0)
    assert not G.entry(0, context=1)                 # another DefaultNode, same ClusterNode (passQps 1)
    assert G.node(CLUSTER, 0)[0] == 1 and G.node(CLUSTER, 0)[1] == 1


def test_custom_origin_selects_origin_node(oracle_mod):
    """testCustomOriginFlowSelectNode: limitApp == origin -> the origin node; a mismatching limitApp
    selects no node (pass)."""
    G = Graph(oracle_mod, [rule(0, 1, limit_app=APP_A)], 1)
    assert G.entry(0, origin=APP_A)
    assert not G.entry(0, origin=APP_A)              # origin node (0, appA) holds one pass
    assert G.entry(0, origin=APP_B) and G.entry(0, origin=APP_B)   # limitApp appA != appB: no node
    assert G.node(ORIGIN, G.onode[(0, APP_A)])[0] == 1
    G2 = Graph(oracle_mod, [rule(0, 0, limit_app=APP_B)], 1)
    assert all(G2.entry(0, origin=APP_A) for _ in range(3))


def test_other_origin(oracle_mod):
    """testOtherOriginFlowSelectNode: ruleA limitApp appA (count 1), ruleB limitApp "other" (count 2):
    origin appB is an "other" origin (ruleB on its origin node); origin appA is named by ruleA, so
    ruleB selects nothing for it."""
    G = Graph(oracle_mod, [rule(0, 1, limit_app=APP_A), rule(0, 2, limit_app=OTHER)], 1)
    assert G.entry(0, origin=APP_B) and G.entry(0, origin=APP_B)
    assert not G.entry(0, origin=APP_B)              # ruleB: 2 + 1 > 2 on node (0, appB)
    assert G.entry(0, origin=APP_A)
    assert not G.entry(0, origin=APP_A)              # ruleA on node (0, appA); ruleB not applicable
    assert all(G.entry(0) for _ in range(4))         # no origin: neither rule selects a node


def test_empty_reference(oracle_mod):
    """testSelectNodeForEmptyReference: CHAIN with a blank refResource selects no node.  A QPS rule like
    that is invalid (FlowRuleUtil.checkStrategyField) and dropped; a THREAD one loads and passes."""
    G = Graph(oracle_mod, [rule(0, 0, strategy=CHAIN), rule(1, 0, grade=THREAD, strategy=CHAIN)], 2)
    assert G.g.n_rules(0) == 0 and G.g.n_rules(1) == 1
    assert all(G.entry(1) for _ in range(3))


def test_relate_reference(oracle_mod):
    """testSelectNodeForRelateReference: RELATE reads the refResource's ClusterNode -- none before its
    first entry (ClusterBuilderSlot creates it), then its passQps."""
    G = Graph(oracle_mod, [rule(0, 1, strategy=RELATE, ref=1)], 2)
    assert all(G.entry(0) for _ in range(3))         # resource 1 never entered: no node -> pass
    assert G.entry(1)                                # creates ClusterNode(1), passQps 1
    assert not G.entry(0)                            # 1 + 1 > 1
    assert G.node(CLUSTER, 0)[1] == 1


def test_chain_context_entrance(oracle_mod):
    """testSelectReferenceNodeForContextEntrance: CHAIN refResource == the context name -> this
    DefaultNode, another context -> no node."""
    G = Graph(oracle_mod, [rule(0, 1, strategy=CHAIN, ref=1)], 1)
    assert G.entry(0, context=1)
    assert not G.entry(0, context=1)
    assert all(G.entry(0, context=2) for _ in range(3))
    assert G.node(DNODE, G.dnode[(1, 0)])[0] == 1 and G.node(DNODE, G.dnode[(2, 0)])[0] == 3


def test_pass_check_select_empty_node(oracle_mod):
    """testPassCheckSelectEmptyNodeSuccess: limitApp "abc", origin "def" -> no node -> pass."""
    G = Graph(oracle_mod, [rule(0, 0, limit_app=7)], 1, origins=(-1, 8))
    assert all(G.entry(0, origin=8) for _ in range(3))


def test_comparator_order_decides_the_occupying_node(oracle_mod):
    """FlowRuleComparatorTest: non-"default" limitApps sort before "default" ones (stable).  Given
    [default rule X, appA rule Y] both failing for a prioritized entry, Y is checked first, so its
    node (the origin node) takes the occupied pass (DefaultController.canPass: tryOccupyNext on the
    selected node, then PriorityWaitException ends the check)."""
    G = Graph(oracle_mod, [rule(0, 1), rule(0, 1, limit_app=APP_A)], 1)
    G.t = T.T0_ALIGNED + 100
    assert G.entry(0, origin=APP_A)                  # passQps 1 on both nodes
    # next bucket: tryOccupyNext finds the first bucket's pass leaving the window within 400 ms
    assert G.entry(0, origin=APP_A, prio=True, dt=500)
    o = G.node(ORIGIN, G.onode[(0, APP_A)])
    c = G.node(CLUSTER, 0)
    assert o[8] == 1 and c[8] == 0                   # minute OCCUPIED_PASS on the origin node only
    assert o[13] == 2 and c[13] == 2                 # both entries hold a thread on every node


def test_duplicates_and_invalid_rules(oracle_mod):
    """buildFlowRuleMap: identical rules collapse (HashSet); count < 0 / an unknown grade dropped."""
    G = Graph(oracle_mod, [rule(0, 3), rule(0, 3), rule(0, -1), (0, 7, 1.0, 0, 0, -1, 0), rule(0, 3, limit_app=-1)], 1)
    assert G.g.n_rules(0) == 1                       # a blank limitApp is "default": a duplicate too


# ---------------------------------------------------------------- GPU vs oracle

def graph_rules():
    return [
        rule(0, 5),
        rule(1, 8, strategy=RELATE, ref=0), rule(1, 2, limit_app=APP_A),
        rule(2, 3, strategy=CHAIN, ref=1), rule(2, 4, limit_app=OTHER), rule(2, 2, grade=THREAD, limit_app=APP_B),
        rule(3, 3, grade=THREAD), rule(3, 6, strategy=RELATE, ref=4),
        rule(4, 5, strategy=RELATE, ref=3),                                       # RELATE cycle 3 <-> 4
        rule(6, 4), rule(6, 4), rule(6, -1), rule(6, 0, strategy=CHAIN), rule(6, 0, grade=THREAD, strategy=RELATE),
        rule(7, 2, limit_app=APP_A, strategy=RELATE, ref=8), rule(7, 10),
        rule(8, 4), rule(8, 1, grade=THREAD, limit_app=OTHER),
        rule(9, 7, limit_app=OTHER, strategy=RELATE, ref=9), rule(9, 12),
    ]


def make_trace(G, rng, n, R, t0, exit_frac=0.3, prio_frac=0.1):
    """Online trace: each step either exits a live passed entry (same context / origin / acquire,
    rt = now - its entry time) or makes a new entry; the oracle decides as it goes, so its
    outcomes are the expected verdicts."""
    res = np.zeros(n, np.int32)
    acq = np.zeros(n, np.int32)
    ts = np.zeros(n, np.int64)
    ctx = np.zeros(n, dtype=G.g.CTX_DTYPE)
    fl = np.zeros(n, np.uint8)
    rt = np.zeros(n, np.int64)
    live = []
    t = t0
    origins = (-1, -1, 0, 1, APP_A, APP_B, APP_C)
    for i in range(n):
        t += int(rng.integers(0, 12))
        if rng.random() < 0.01:
            t -= int(rng.integers(1, 40))                # the clock went back
        if live and rng.random() < exit_frac:
            k = int(rng.integers(len(live)))
            r, a, c, te = live.pop(k)
            res[i], acq[i], ctx[i], ts[i] = r, a, c, t
            fl[i] = EXIT | (ERROR if rng.random() < 0.2 else 0)
            rt[i] = t - te
        else:
            r = int(rng.integers(R))
            c = G.ctx(r, int(origins[rng.integers(len(origins))]), int(rng.integers(3)))
            res[i], acq[i], ctx[i], ts[i] = r, int(rng.integers(1, 3)), c, t
            fl[i] = PRIO if rng.random() < prio_frac else 0
        st, _ = G.g.replay(res[i:i + 1], acq[i:i + 1], ts[i:i + 1], ctx[i:i + 1], fl[i:i + 1], rt[i:i + 1])
        if not (fl[i] & EXIT) and st[0] == 0:
            live.append((int(res[i]), int(acq[i]), ctx[i].copy(), int(ts[i])))
    return res, acq, ts, ctx, fl, rt, t


def test_online_trace_generator_is_replayable(oracle_mod):
    """CPU check of the harness: replaying the generated trace on a fresh oracle graph gives the
    verdicts the online run saw (the GPU test compares against exactly this)."""
    rng = np.random.default_rng(5)
    R = 10
    G = Graph(oracle_mod, graph_rules(), R)
    res, acq, ts, ctx, fl, rt, _ = make_trace(G, rng, 600, R, T.T0_ALIGNED)
    G2 = Graph(oracle_mod, graph_rules(), R)
    st, _ = G2.g.replay(res, acq, ts, ctx, fl, rt)
    G3 = Graph(oracle_mod, graph_rules(), R)
    st3, _ = G3.g.replay(res, acq, ts, ctx, fl, rt)
    assert (st == st3).all()
    assert (st == 1).sum() > 20 and (st == 0).sum() > 100


@pytest.mark.gpu
def test_local_graph_vs_oracle(oracle_mod):
    import sentinel_amd as sa
    rng = np.random.default_rng(71)
    R = 10
    G = Graph(oracle_mod, graph_rules(), R)
    ref = Graph(oracle_mod, graph_rules(), R)
    svc = sa.GpuTokenService(0)
    svc.load_local_rules(graph_rules(), R, len(G.onode), len(G.dnode), sample_count=2, interval_ms=1000)
    t = T.T0_ALIGNED + 137
    for b in range(6):
        n = int(rng.integers(200, 1500))
        res, acq, ts, ctx, fl, rt, t = make_trace(G, rng, n, R, t)
        want, wwait = ref.g.replay(res, acq, ts, ctx, fl, rt)
        got, gwait = svc.submit_local_graph_batch_host(res, acq, ts, ctx, fl, rt)
        assert (got == want).all(), (b, np.nonzero(got != want)[0][:10])
        assert (gwait == wwait).all(), b
    for kind, cnt in ((CLUSTER, R), (ORIGIN, len(G.onode)), (DNODE, len(G.dnode))):
        for i in range(cnt):
            np.testing.assert_array_equal(svc.local_graph_node_metrics(kind, i, t), ref.g.node_metrics(kind, i, t),
                                          err_msg=f"node {kind}/{i}")
    # validation: bad node index -> NO_RULE_EXISTS, t < 0 -> FAIL; the single-rule API refuses the graph
    bad = np.zeros(2, dtype=sa._lib.LOCAL_CTX_DTYPE)
    bad[0] = (-1, 0, 0, 10 ** 6)
    bad[1] = G.ctx(0)
    st, _ = svc.submit_local_graph_batch_host([0, 0], [1, 1], [t, -5], bad)
    assert list(st) == [3, -1]
    with pytest.raises(sa.SentinelError):
        svc.submit_local_batch_host([0], [1], [t])
    svc.close()
