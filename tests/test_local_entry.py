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
                assert list(st) == [nodes[r].pass_sum(t), nodes[r].block_sum(t), nodes[r].total_pass(t),
                                    nodes[r].minute_block(t)], (sc, r)
    assert set(np.unique(svc.submit_local_entry_batch_host([R + 1], [1], [t]))) == {3}
