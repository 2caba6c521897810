"""Local SphU.entry admission (DefaultController over the ClusterNode's StatisticNode): BASELINE
config 1 (FlowQpsDemo) and randomized multi-resource traces on the GPU against the oracle."""
import json
import os

import numpy as np
import pytest

from sentinel_amd import trace as T

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _oracle_replay(oracle_mod, counts, ridx, acq, ts, sample_count=2, interval_ms=1000):
    """Per resource, the sequential StatisticSlot + DefaultController replay (resources are independent)."""
    ok = np.zeros(len(ts), dtype=bool)
    nodes = {}
    for r in np.unique(ridx):
        sel = np.nonzero(ridx == r)[0]
        node = oracle_mod.StatisticNode(sample_count, interval_ms)
        c = counts[r] if counts[r] is not None else float("inf")
        ok[sel] = node.replay(c, acq[sel], ts[sel]).astype(bool)
        nodes[int(r)] = node
    return ok, nodes


def test_config1_trace_shape():
    ts = T.config1(duration_ms=5_000)
    assert (np.diff(ts) >= 0).all() and len(ts) > 32 * 100


@pytest.mark.gpu
def test_flow_partial_integration_kat():
    """FlowPartialIntegrationTest.java:50-72: QPS 1 -> first entry passes, the second blocks."""
    import sentinel_amd as sa
    kat = json.load(open(os.path.join(GOLDEN, "kat_default_controller.json")))
    for case in kat["integration"]:
        for t0 in case["t0"]:
            svc = sa.GpuTokenService(0)
            svc.load_local_resources([case["count"]])
            ts = t0 + np.cumsum(case["dts"])
            st = svc.submit_local_entry_batch_host(np.zeros(len(ts)), case["acquire"], ts)
            assert list(st == 0) == case["expect"], case["name"]


@pytest.mark.gpu
@pytest.mark.parametrize("t0", [T.T0_ALIGNED, T.T0_ALIGNED + 137])
def test_config1_flowqpsdemo(oracle_mod, t0):
    """BASELINE config 1: FlowQpsDemo (1 resource "abc", QPS 20, 32 threads, 100 s)."""
    import sentinel_amd as sa
    ts = T.config1(seed=1, t0=t0)
    n = len(ts)
    svc = sa.GpuTokenService(0)
    svc.load_local_resources([20.0])
    ok_o, nodes = _oracle_replay(oracle_mod, [20.0], np.zeros(n, np.int32), np.ones(n, np.int32), ts)
    got = np.concatenate([svc.submit_local_entry_batch_host(np.zeros(b - a), np.ones(b - a), ts[a:b])
                          for a, b in [(0, n // 3), (n // 3, n)]])
    assert np.array_equal(got == 0, ok_o)
    # passes per sliding 2-bucket window never exceed the QPS threshold
    assert ok_o.sum() <= 20 * 101 and ok_o.sum() > 15 * 100
    t = int(ts[-1])
    st = svc.local_node_stats(0, t)
    node = nodes[0]
    assert st[0] == node.pass_sum(t) and st[1] == node.block_sum(t)
    assert st[2] == node.total_pass(t) and st[3] == node.minute_block(t)
    assert st[4] == 0 and st[5] == 0


@pytest.mark.gpu
def test_local_entries_multi_resource(oracle_mod):
    import sentinel_amd as sa
    rng = np.random.default_rng(81)
    R = 300
    counts = [None if r % 11 == 0 else float(rng.integers(1, 60)) + (0.5 if r % 7 == 0 else 0.0) for r in range(R)]
    n = 150_000
    ridx = T.zipf_indices(R, 1.0, n, rng)
    acq = np.ones(n, np.int32)
    acq[rng.random(n) < 0.05] = 3
    ts = T.timestamps(n, 20_000.0, T.T0_ALIGNED + 29)
    ts = ts + np.where(rng.random(n) < 0.002, -rng.integers(0, 700, size=n), 0)
    ts = ts.astype(np.int64)
    for sc, iv in [(2, 1000), (3, 1500)]:
        svc = sa.GpuTokenService(0)
        svc.load_local_resources(counts, sample_count=sc, interval_ms=iv)
        ok_o, nodes = _oracle_replay(oracle_mod, counts, ridx, acq, ts, sc, iv)
        got = np.concatenate([svc.submit_local_entry_batch_host(ridx[a:b], acq[a:b], ts[a:b])
                              for a, b in [(0, 50_000), (50_000, 150_000)]])
        bad = np.nonzero((got == 0) != ok_o)[0]
        assert len(bad) == 0, (sc, len(bad), bad[:5])
        t = int(ts.max())
        for r in range(0, R, 13):
            if r in nodes:
                st = svc.local_node_stats(r, t)
                assert list(st[:4]) == [nodes[r].pass_sum(t), nodes[r].block_sum(t), nodes[r].total_pass(t),
                                        nodes[r].minute_block(t)], (sc, r)
    assert set(np.unique(svc.submit_local_entry_batch_host([R + 1], [1], [t]))) == {3}


# Prioritized entries (SphU.entryWithPriority): DefaultController.java:52-64 -> StatisticNode.tryOccupyNext
# (StatisticNode.java:288-320), the borrow array seeding the next window (OccupiableBucketLeapArray.java:40-64).
# No reference test covers tryOccupyNext; this trace is derived by hand from the code (count 5, node 2 x 500 ms):
# five passes in [T-500, T), then at T+100 five prioritized entries borrow from [T+500, T+1000) with a
# 400 ms wait (the [T-500, T) window leaves the interval by then) and the sixth finds the borrow at
# maxCount (-> timeout -> block); at T+500 the new bucket starts with the 5 borrowed PASS, so a plain
# entry blocks, at T+1000 too, and at T+1500 the window is free again.
PRIO_T = 1_600_000_000_000
PRIO_TRACE = [(PRIO_T - 300, 0)] * 5 + [(PRIO_T + 100, 1)] * 6 + [(PRIO_T + 500, 0), (PRIO_T + 1000, 0), (PRIO_T + 1500, 0)]
PRIO_EXPECT = [(True, 0)] * 5 + [(True, 400)] * 5 + [(False, 0)] * 3 + [(True, 0)]


def test_prioritized_entry_oracle_trace(oracle_mod):
    node = oracle_mod.StatisticNode(2, 1000)
    got = [node.entry(5.0, 1, t, bool(p)) for t, p in PRIO_TRACE]
    assert got == PRIO_EXPECT
    t = PRIO_TRACE[-1][0]
    assert node.minute_occupied(t) == 5 and node.total_pass(t) == 11


def test_prioritized_entry_timeout_property(oracle_mod):
    """OccupyTimeoutProperty.updateTimeout: a 300 ms timeout refuses the 400 ms wait; > INTERVAL is ignored."""
    node = oracle_mod.StatisticNode(2, 1000)
    node.set_occupy_timeout(300)
    got = [node.entry(5.0, 1, t, bool(p)) for t, p in PRIO_TRACE[:7]]
    assert got == [(True, 0)] * 5 + [(False, 0)] * 2
    node = oracle_mod.StatisticNode(2, 1000)
    node.set_occupy_timeout(5000)
    assert [node.entry(5.0, 1, t, bool(p)) for t, p in PRIO_TRACE] == PRIO_EXPECT


def _oracle_replay_prio(oracle_mod, counts, ridx, acq, ts, prio, sample_count=2, interval_ms=1000):
    ok = np.zeros(len(ts), dtype=bool)
    wait = np.zeros(len(ts), dtype=np.int64)
    nodes = {}
    for r in np.unique(ridx):
        sel = np.nonzero(ridx == r)[0]
        node = oracle_mod.StatisticNode(sample_count, interval_ms)
        c = counts[r] if counts[r] is not None else float("inf")
        o, w = node.replay_prio(c, acq[sel], ts[sel], prio[sel])
        ok[sel] = o.astype(bool)
        wait[sel] = w
        nodes[int(r)] = node
    return ok, wait, nodes


@pytest.mark.gpu
def test_prioritized_entry_gpu_trace():
    import sentinel_amd as sa
    svc = sa.GpuTokenService(0)
    svc.load_local_resources([5.0])
    ts = np.array([t for t, _ in PRIO_TRACE], np.int64)
    pr = np.array([p for _, p in PRIO_TRACE], np.uint8)
    st, wait = svc.submit_local_entry_batch_host(np.zeros(len(ts)), np.ones(len(ts)), ts, pr, with_wait=True)
    assert [(bool(s == 0), int(w)) for s, w in zip(st, wait)] == PRIO_EXPECT
    stats = svc.local_node_stats(0, int(ts[-1]))
    assert stats[2] == 11 and stats[4] == 5
    svc = sa.GpuTokenService(0)                              # OccupyTimeoutProperty.updateTimeout(300)
    svc.load_local_resources([5.0])
    svc.set_occupy_timeout(300)
    st, wait = svc.submit_local_entry_batch_host(np.zeros(7), np.ones(7), ts[:7], pr[:7], with_wait=True)
    assert [(bool(s == 0), int(w)) for s, w in zip(st, wait)] == [(True, 0)] * 5 + [(False, 0)] * 2


@pytest.mark.gpu
@pytest.mark.parametrize("sc,iv", [(2, 1000), (4, 1000), (3, 1500)])
def test_prioritized_entries_multi_resource(oracle_mod, sc, iv):
    """Random traces with ~20% prioritized entries over many resources, several batches."""
    import sentinel_amd as sa
    rng = np.random.default_rng(97 + sc)
    R = 200
    counts = [None if r % 13 == 0 else float(rng.integers(2, 40)) for r in range(R)]
    n = 120_000
    ridx = T.zipf_indices(R, 1.0, n, rng)
    acq = np.ones(n, np.int32)
    acq[rng.random(n) < 0.05] = 2
    prio = (rng.random(n) < 0.2).astype(np.uint8)
    ts = T.timestamps(n, 30_000.0, T.T0_ALIGNED + 61).astype(np.int64)
    svc = sa.GpuTokenService(0)
    svc.load_local_resources(counts, sample_count=sc, interval_ms=iv)
    ok_o, wait_o, nodes = _oracle_replay_prio(oracle_mod, counts, ridx, acq, ts, prio, sc, iv)
    assert wait_o.max() > 0
    sts, waits = [], []
    for a, b in [(0, 40_000), (40_000, 120_000)]:
        st, w = svc.submit_local_entry_batch_host(ridx[a:b], acq[a:b], ts[a:b], prio[a:b], with_wait=True)
        sts.append(st)
        waits.append(w)
    got, gw = np.concatenate(sts), np.concatenate(waits)
    bad = np.nonzero(((got == 0) != ok_o) | (gw != wait_o))[0]
    assert len(bad) == 0, (sc, len(bad), bad[:5])
    t = int(ts.max())
    for r in range(0, R, 17):
        if r in nodes:
            st = svc.local_node_stats(r, t)
            assert list(st[2:5]) == [nodes[r].total_pass(t), nodes[r].minute_block(t), nodes[r].minute_occupied(t)], r
