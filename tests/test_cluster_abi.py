"""Multi-device engine ABI (sentinel_cluster_*): flows partitioned shard = splitmix64(flowId) mod n,
one engine per entry of device_ids.  Two or three shards on device 0 (the ABI allows a device to
repeat) decide a config-2 trace exactly as one engine / the oracle does; the snapshot covers every
flow once; the per-call door routes to the owning shard.  SURVEY §8b/§8e."""
import threading

import numpy as np
import pytest

from sentinel_amd import trace as T


def test_shard_of_matches_python_splitmix():
    """The C router and the bench / shard.py sharding agree (CPU: the library loads, no device)."""
    from sentinel_amd import _lib
    L = _lib.load()
    ids = np.array([1, 2, 3, 10_000, 2**40 + 7, 2**62 - 1], dtype=np.int64)
    for n in (1, 2, 3, 8):
        want = T.shard_of(ids, n)
        got = [L.sentinel_shard_of(int(i), n) for i in ids]
        assert list(want) == got


pytestmark_gpu = pytest.mark.gpu


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [2, 3])
def test_cluster_matches_single_engine_and_oracle(oracle_mod, shards):
    import sentinel_amd as sa
    rules, ev = T.config2(300_000, seed=21, n_flows=2000)
    cl = sa.GpuTokenCluster([0] * shards)
    cl.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count, rules.window_interval_ms,
                        rules.namespace, rules.checker)
    assert cl.flow_count() == len(rules)
    orc = oracle_mod.TokenServiceOracle(rules.as_dicts())
    fids = rules.flow_id[np.clip(ev.flow_idx, 0, len(rules) - 1)]
    fids = np.where(ev.flow_idx < 0, 0, fids)
    for a, b in [(0, 100_000), (100_000, 300_000)]:
        st, rem, w = cl.submit_host(fids[a:b], ev.acquire[a:b], ev.ts[a:b])
        st_o, rem_o, w_o = orc.replay(ev.flow_idx[a:b], ev.acquire[a:b], ev.ts[a:b], None)
        bad = np.nonzero((st != st_o) | (rem != rem_o))[0]
        assert len(bad) == 0, (shards, len(bad), bad[:5])
    snap = cl.snapshot(int(ev.ts[-1]))
    assert sorted(snap["flow_id"].tolist()) == sorted(rules.flow_id.tolist())


@pytest.mark.gpu
def test_cluster_batchers_route_per_call(oracle_mod):
    import sentinel_amd as sa
    rng = np.random.default_rng(5)
    rules = T.make_rules(64, rng, count_lo=5, count_hi=20, sample_count=2, window_interval_ms=1000)
    cl = sa.GpuTokenCluster([0, 0])
    cl.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count, rules.window_interval_ms,
                        rules.namespace, rules.checker)
    cl.start_batchers(max_batch=256, max_wait_us=100)
    t0 = T.T0_ALIGNED + 5
    results = {}

    def worker(k):
        fid = int(rules.flow_id[k % 64])
        results[k] = cl.request_token(fid, 1, False, t0 + 10)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(64 * 30)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    # every flow got exactly floor(count) passes among its 30 requests at one instant
    for f in range(64):
        passed = sum(1 for k, r in results.items() if k % 64 == f and r.status == 0)
        assert passed == min(30, int(rules.count[f])), (f, passed, rules.count[f])
    cl.close()


@pytest.mark.gpu
def test_cluster_rejects_per_shard_namespace_limiters():
    """A namespace GlobalRequestLimiter split over flowId-hash shards would admit up to n x the cap:
    a multi-shard cluster refuses has_limiter namespaces; a single-shard cluster accepts and applies
    them exactly (GlobalRequestLimiter.java:46-55)."""
    import sentinel_amd as sa
    from sentinel_amd.token_service import ServerNamespace
    cl = sa.GpuTokenCluster([0, 0])
    with pytest.raises(sa.SentinelError):
        cl.set_namespaces([ServerNamespace(connected_count=1, has_limiter=True, max_allowed_qps=10.0)])
    cl.set_namespaces([ServerNamespace(connected_count=1, has_limiter=False)])     # no limiter: fine
    cl.close()
    one = sa.GpuTokenCluster([0])
    one.set_namespaces([ServerNamespace(connected_count=1, has_limiter=True, max_allowed_qps=10.0)])
    rng = np.random.default_rng(6)
    rules = T.make_rules(50, rng, count_lo=1000, count_hi=2000, sample_count=10, window_interval_ms=1000)
    one.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count,
                         rules.window_interval_ms, rules.namespace, rules.checker)
    fids = rules.flow_id[rng.integers(0, 50, size=200)]
    st, _, _ = one.submit_host(fids, np.ones(200, np.int32), np.full(200, T.T0_ALIGNED + 1, np.int64))
    assert int((st == 0).sum()) == 10 and int((st == -2).sum()) == 190     # the node-wide cap of 10 QPS
    one.close()
