"""Rule reloads: ClusterFlowRuleManager.applyClusterFlowRule / ClusterParamFlowRuleManager
.applyClusterParamRules semantics (putMetricIfAbsent, removal, emptied-namespace orphans) and the
server-window reset (ClusterMetricStatistics.resetFlowMetrics).

Reference (sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/alibaba/csp/sentinel/cluster/):
  flow/rule/ClusterFlowRuleManager.java:325-372 (putMetricIfAbsent at :361-362), :268-301
  flow/rule/ClusterParamFlowRuleManager.java:318-360
  flow/statistic/ClusterMetricStatistics.java:44-66, server/config/ClusterServerConfigManager.java:333-343
No reference test exercises a reload (parity of this behaviour is pinned by the restated code only);
the CPU tests below pin the oracle's restatement, the GPU tests compare the engine with it.
"""
import numpy as np
import pytest

from sentinel_amd import trace as T


def _rules(specs):
    """specs: (flow_id, count, sample_count, interval_ms, namespace_idx)"""
    return [dict(flow_id=f, count=c, threshold_type=1, sample_count=n, window_interval_ms=iv, namespace_idx=ns)
            for f, c, n, iv, ns in specs]


NS2 = [dict(connected_count=1), dict(connected_count=1)]

PLAN_A = _rules([(1, 30, 2, 1000, 0), (2, 20, 2, 1000, 0), (3, 25, 5, 500, 0), (4, 40, 10, 1000, 1),
                 (5, 15, 4, 400, 1), (6, 50, 1, 1000, 0)])
# flow 1 unchanged, flow 2 with a new window (keeps the old one), flow 3 removed, flow 7 twice (first
# window wins, last count wins), namespace 1's list emptied (flows 4, 5 orphaned), flow 6 new count
PLAN_B = _rules([(1, 30, 2, 1000, 0), (2, 35, 5, 500, 0), (7, 10, 4, 400, 0), (6, 5, 1, 1000, 0),
                 (7, 60, 2, 1000, 0)])
# flow 4 comes back (revived orphan: old window and counters), flow 5 stays orphaned, flow 2 removed
PLAN_C = _rules([(1, 30, 2, 1000, 0), (4, 44, 2, 1000, 1), (7, 60, 2, 1000, 0), (6, 5, 1, 1000, 0), (8, 9, 5, 1000, 0)])


def test_oracle_reload_semantics(oracle_mod):
    orc = oracle_mod.TokenServiceOracle(PLAN_A, namespaces=NS2)
    rng = np.random.default_rng(5)
    t0 = T.T0_ALIGNED + 17
    ts = t0 + np.sort(rng.integers(0, 900, size=400))
    orc.replay(rng.integers(0, 6, size=400).astype(np.int32), np.ones(400, np.int32), ts)
    before = {f: orc.dump_flow(i) for i, f in enumerate([1, 2, 3, 4, 5, 6])}
    assert orc.metric_count() == 6
    assert orc.reload_flow_rules(PLAN_B) == 4                        # 1, 2, 7, 6 (7 deduplicated)
    assert orc.flow_window(0) == (2, 1000)
    assert orc.flow_window(1) == (2, 1000)                          # flow 2 keeps its old window
    assert orc.flow_window(2) == (4, 400)                           # flow 7: its first occurrence
    assert np.array_equal(orc.dump_flow(0), before[1]) and np.array_equal(orc.dump_flow(1), before[2])
    assert np.array_equal(orc.dump_flow(3), before[6])
    assert orc.metric_count() == 6                                  # 1, 2, 6, 7 + orphans 4, 5 (3 removed)
    # flow 7 decides with its last rule's count (60) on the first occurrence's window
    st, rem, _ = orc.replay(np.array([2], np.int32), np.array([1], np.int32), np.array([t0 + 950]))
    assert st[0] == 0 and rem[0] == 59
    assert orc.reload_flow_rules(PLAN_C) == 5
    assert orc.flow_window(1) == (10, 1000)                         # flow 4 revived with its old window
    assert np.array_equal(orc.dump_flow(1), before[4])
    assert orc.metric_count() == 6                                  # 1, 4, 7, 6, 8 + orphan 5 (2 removed)
    assert orc.reset_metrics(3, 300) == 0                           # server window change
    assert all(orc.flow_window(i) == (3, 300) for i in range(5))
    assert (orc.dump_flow(0)[:24].reshape(3, 8)[:, 0] == -1).all()


def _gpu_engine(rules, namespaces):
    import sentinel_amd as sa
    from sentinel_amd.token_service import ServerNamespace
    svc = sa.GpuTokenService(0)
    svc.set_namespaces([ServerNamespace(**n) for n in namespaces])
    _gpu_load(svc, rules)
    return svc


def _gpu_load(svc, rules):
    import sentinel_amd as sa
    svc.load_flow_rules([sa.FlowRule(count=r["count"], namespace=r["namespace_idx"], cluster_config=sa.ClusterFlowConfig(
        flow_id=r["flow_id"], threshold_type=1, sample_count=r["sample_count"],
        window_interval_ms=r["window_interval_ms"])) for r in rules])


def _check(svc, orc, F, idx, acq, ts):
    st_g, rem_g, w_g = svc.submit_flow_batch_host(idx, acq, ts)
    st_o, rem_o, w_o = orc.replay(idx, acq, ts)
    bad = np.nonzero((st_g != st_o) | (rem_g != rem_o))[0]
    assert len(bad) == 0, (len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]], rem_g[bad[:5]], rem_o[bad[:5]])
    for f in range(F):
        assert svc.flow_window(f) == orc.flow_window(f), f
        assert np.array_equal(svc.dump_flow(f), orc.dump_flow(f)), (f, svc.dump_flow(f), orc.dump_flow(f))


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["sorted", "partition", "small"])
def test_gpu_reload_matches_oracle(oracle_mod, path):
    """Batches -> reload (survivors keep old windows and counters, removals, a changed window, a
    duplicate flowId, an emptied namespace) -> batches -> reload (an orphan comes back) -> server
    window reset -> batches: verdicts, windows and full dumps equal the oracle's."""
    svc = _gpu_engine(PLAN_A, NS2)
    svc.set_flow_path(path)
    orc = oracle_mod.TokenServiceOracle(PLAN_A, namespaces=NS2)
    rng = np.random.default_rng(9)
    t = T.T0_ALIGNED + 29
    for plan, F in ((PLAN_A, 6), (PLAN_B, 4), (PLAN_C, 5), ("reset", 5)):
        if plan == "reset":
            svc.reset_metrics(4, 800)
            orc.reset_metrics(4, 800)
        elif plan is not PLAN_A:
            _gpu_load(svc, plan)
            assert orc.reload_flow_rules(plan) == F
            assert svc.flow_count() == F
        assert svc.metric_count() == orc.metric_count()
        for _ in range(3):
            m = 3000
            ts = np.sort(t + rng.integers(0, 700, size=m)).astype(np.int64)
            idx = rng.integers(0, F, size=m).astype(np.int32)
            acq = np.where(rng.random(m) < 0.1, 2, 1).astype(np.int32)
            _check(svc, orc, F, idx, acq, ts)
            t = int(ts[-1]) + 1


@pytest.mark.gpu
def test_gpu_reload_large_table_device_side(oracle_mod):
    """200k flows: a reload that keeps every flow but changes half the windows and adds 50k flows is
    done on the device (no window state crosses PCIe) and keeps every surviving window bit for bit."""
    import time
    rng = np.random.default_rng(3)
    F = 200_000
    rules = T.make_rules(F, rng, sample_count=10, window_interval_ms=1000)
    import sentinel_amd as sa
    svc = sa.GpuTokenService(0)
    svc.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count,
                         rules.window_interval_ms, rules.namespace, rules.checker)
    orc = oracle_mod.TokenServiceOracle.from_arrays(rules.flow_id, rules.count, rules.threshold_type,
                                                    rules.sample_count, rules.window_interval_ms,
                                                    rules.namespace, rules.checker)
    n = 1_000_000
    idx = rng.integers(0, F, n).astype(np.int32)
    ts = T.timestamps(n, 2.0 * float(rules.count.sum()), T.T0_ALIGNED)
    _ = svc.submit_flow_batch_host(idx, np.ones(n, np.int32), ts)
    orc.replay(idx, np.ones(n, np.int32), ts)
    sample = rng.choice(F, 200, replace=False)
    before = {int(f): svc.dump_flow(int(f)) for f in sample}
    r2 = T.make_rules(F + 50_000, np.random.default_rng(4), sample_count=10, window_interval_ms=1000)
    r2.sample_count[::2] = 5                     # a new window: survivors keep theirs (putMetricIfAbsent)
    r2.window_interval_ms[::2] = 500
    t0 = time.perf_counter()
    svc.load_rules_array(r2.flow_id, r2.count, r2.threshold_type, r2.sample_count, r2.window_interval_ms,
                         r2.namespace, r2.checker)
    reload_ms = (time.perf_counter() - t0) * 1000
    orc.reload_flow_rules([dict(flow_id=int(r2.flow_id[i]), count=float(r2.count[i]), threshold_type=1,
                                sample_count=int(r2.sample_count[i]), window_interval_ms=int(r2.window_interval_ms[i]),
                                namespace_idx=0) for i in range(len(r2))])
    for f in sample:
        assert np.array_equal(svc.dump_flow(int(f)), before[int(f)])
        assert svc.flow_window(int(f)) == (10, 1000)
    assert svc.flow_window(F + 10) == (5, 500) and svc.flow_window(F + 11) == (10, 1000)
    idx = rng.integers(0, F + 50_000, n).astype(np.int32)
    ts = ts[-1] + 1 + T.timestamps(n, 2.0 * float(r2.count.sum()), 0)
    st_g, rem_g, _ = svc.submit_flow_batch_host(idx, np.ones(n, np.int32), ts)
    st_o, rem_o, _ = orc.replay(idx, np.ones(n, np.int32), ts)
    assert np.array_equal(st_g, st_o) and np.array_equal(rem_g, rem_o)
    print(f"reload of {F} -> {F + 50_000} flows: {reload_ms:.1f} ms")


def _param_rules(specs):
    """specs: (flow_id, count, sample_count, interval_ms, namespace_idx)"""
    return [dict(flow_id=f, count=c, threshold_type=1, sample_count=n, window_interval_ms=iv, namespace_idx=ns)
            for f, c, n, iv, ns in specs]


P_A = _param_rules([(11, 8, 2, 1000, 0), (12, 5, 5, 500, 0), (13, 6, 2, 1000, 1), (14, 9, 4, 400, 0)])
P_B = _param_rules([(11, 8, 2, 1000, 0), (12, 7, 2, 1000, 0), (15, 4, 2, 1000, 0), (14, 3, 1, 1000, 0)])
P_C = _param_rules([(11, 8, 2, 1000, 0), (13, 6, 5, 500, 1), (15, 4, 2, 1000, 0)])


def _gpu_param_load(svc, rules):
    import sentinel_amd as sa
    svc.load_param_rules([sa.ParamFlowRule(count=r["count"], namespace=r["namespace_idx"], cluster_config=sa.ClusterFlowConfig(
        flow_id=r["flow_id"], threshold_type=1, sample_count=r["sample_count"],
        window_interval_ms=r["window_interval_ms"])) for r in rules])


@pytest.mark.gpu
def test_gpu_param_reload_matches_oracle(oracle_mod):
    """Param rule reloads: surviving rules keep their per-value counters and old windows, removed rules
    lose them, an emptied namespace's rule comes back with its counters; top values agree."""
    import sentinel_amd as sa
    from sentinel_amd.token_service import ServerNamespace
    svc = sa.GpuTokenService(0)
    svc.set_namespaces([ServerNamespace(**n) for n in NS2])
    _gpu_param_load(svc, P_A)
    orc = oracle_mod.TokenServiceOracle([], namespaces=NS2, param_rules=P_A)
    rng = np.random.default_rng(21)
    t = T.T0_ALIGNED + 3
    for plan, R in ((P_A, 4), (P_B, 4), (P_C, 3)):
        if plan is not P_A:
            _gpu_param_load(svc, plan)
            orc.load_param_rules(plan, {})
        assert svc.param_count() == R
        for _ in range(3):
            m = 4000
            ts = np.sort(t + rng.integers(0, 600, size=m)).astype(np.int64)
            ridx = rng.integers(0, R, size=m).astype(np.int32)
            vals = T.zipf_indices(40, 1.1, m, rng, permute=False)
            # keys identify (rule flowId, value): the flowId, not the dense index, is encoded
            fids = np.array([r["flow_id"] for r in plan], dtype=np.uint64)[ridx]
            keys = (fids << np.uint64(20)) | vals.astype(np.uint64)
            acq = np.ones(m, np.int32)
            st_g, rem_g = svc.submit_param_batch_host(ridx, acq, keys, ts)
            st_o, rem_o = orc.param_replay(ridx, acq, keys, ts)
            bad = np.nonzero((st_g != st_o) | (rem_g != rem_o))[0]
            assert len(bad) == 0, (len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]])
            t = int(ts[-1]) + 1
        top = svc.param_top_values(t)
        for r in range(R):
            assert top[r] == orc.param_top_values(r, t), (r, top[r], orc.param_top_values(r, t))
