"""The exact hot-parameter slot table stays bounded: dead slots are reclaimed and the table grows
before it could fill, so no request answers FAIL for lack of a slot, and verdicts stay bit-exact
against the oracle (ClusterParamFlowChecker.java:42-87, ClusterParamMetric.java:46-82; the reference
clears a bucket's CacheMap on reset, ClusterParameterLeapArray.java:40-49).  Plus BASELINE config 4
at its stated size (100k param resources x 1000 Long values, Zipf 1.2) and its over-cap variant.
"""
import numpy as np
import pytest

from sentinel_amd import trace as T

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["arrival", "ordered"])
def param_output(request, monkeypatch):
    """Every case with verdicts at their arrival positions and with decide-order output
    (sentinel_submit_param_batch_ordered_host, put back through its seq)."""
    if request.param == "ordered":
        from conftest import use_ordered_param_host
        use_ordered_param_host(monkeypatch)
    return request.param


def _svc(prules, capacity=None, monkeypatch=None):
    import sentinel_amd as sa
    from sentinel_amd.token_service import ServerNamespace
    if capacity is not None:
        monkeypatch.setenv("SENTINEL_PARAM_CAPACITY", str(capacity))
    svc = sa.GpuTokenService(0)
    svc.set_namespaces([ServerNamespace()])
    svc.load_param_rules([sa.ParamFlowRule(count=r["count"], cluster_config=sa.ClusterFlowConfig(
        flow_id=r["flow_id"], threshold_type=1, sample_count=r["sample_count"],
        window_interval_ms=r["window_interval_ms"]), hot_items=r.get("hot", {})) for r in prules])
    return svc


def test_slot_reclamation_and_growth(oracle_mod, monkeypatch):
    """A moving value universe over 40 simulated seconds (~400k distinct keys, ~15k live at a time)
    through a table that starts at 1024 slots: it grows, reclaims dead slots, never answers FAIL, and
    stays small; single- and multi-value batches alternate."""
    R = 50
    prules = [dict(flow_id=100 + r, count=float(5 + r % 20), sample_count=2 if r % 3 else 5, window_interval_ms=1000)
              for r in range(R)]
    svc = _svc(prules, capacity=1024, monkeypatch=monkeypatch)
    orc = oracle_mod.TokenServiceOracle([], param_rules=prules)
    rng = np.random.default_rng(17)
    t = T.T0_ALIGNED + 7
    fids = np.array([r["flow_id"] for r in prules], dtype=np.uint64)
    for sec in range(40):
        m = 20_000
        ts = np.sort(t + rng.integers(0, 1000, size=m)).astype(np.int64)
        ridx = rng.integers(0, R, size=m).astype(np.int32)
        vals = (sec * 10_000 + rng.integers(0, 300, size=m)).astype(np.uint64)   # this second's universe
        keys = (fids[ridx] << np.uint64(32)) | vals
        acq = np.where(rng.random(m) < 0.2, 2, 1).astype(np.int32)
        if sec % 4 == 3:       # multi-value requests (1..3 values) in the same table
            counts = rng.integers(1, 4, size=m).astype(np.int32)
            begin = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32)
            mv = (sec * 10_000 + rng.integers(0, 300, size=int(counts.sum()))).astype(np.uint64)
            mkeys = (np.repeat(fids[ridx], counts) << np.uint64(32)) | mv
            st_g, rem_g = svc.submit_param_multi_batch_host(ridx, acq, ts, begin, counts, mkeys)
            st_o, rem_o = orc.param_multi_replay(ridx, acq, ts, begin, counts, mkeys)
        else:
            st_g, rem_g = svc.submit_param_batch_host(ridx, acq, keys, ts)
            st_o, rem_o = orc.param_replay(ridx, acq, keys, ts)
        assert not (st_g == -1).any(), "a request answered FAIL (slot table full)"
        bad = np.nonzero((st_g != st_o) | (rem_g != rem_o))[0]
        assert len(bad) == 0, (sec, len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]])
        t += 1000
    stats = svc.param_table_stats()
    assert stats["rebuilds"] >= 3, stats
    # bounded by the live set plus a few batches of values (the headroom that keeps rebuilds rare), not
    # by history: holding all ~400k distinct keys at <= 3/4 load would take 2^20 slots
    assert stats["capacity"] <= 1 << 19, stats
    for i in range(0, 2000, 37):
        r, k = int(ridx[i]), int(keys[i])
        assert svc.param_sum(r, k, int(ts[-1])) == orc.param_sum(r, int(ts[-1]), k)


def _config4_rules(count, hot, n_rules):
    return [dict(flow_id=r + 1, count=float(count[r]), sample_count=10, window_interval_ms=1000,
                 hot={k: v for k, v in hot.get(r, {}).items()}) for r in range(n_rules)]


@pytest.mark.parametrize("universe", [1000, 100_000])
def test_config4_full_size_bitexact(oracle_mod, universe):
    """BASELINE config 4: 100k param resources, one rule each (count ~ U{5..100}, hot items), values
    Zipf(1.2) over a per-resource universe of 1000 Long keys (<= 4000 per bucket: exact parity), plus
    the over-cap universe of 100k -- identical verdicts on the exact table; where a bucket would hold
    more than 4000 values the reference's LRU would evict (parity unpinned there: reported, not
    asserted)."""
    n_rules = 100_000
    n = 2_000_000
    count, hot, rule_idx, vals, keys, ts = T.config4(2 * n, seed=4, n_rules=n_rules, universe=universe)
    prules = _config4_rules(count, hot, n_rules)
    svc = _svc(prules)
    orc = oracle_mod.TokenServiceOracle([], param_rules=prules,
                                        hot_items={r: list(hot[r].items()) for r in hot})
    acq = np.ones(2 * n, np.int32)
    for a, b in [(0, n), (n, 2 * n)]:
        st_g, rem_g = svc.submit_param_batch_host(rule_idx[a:b], acq[a:b], keys[a:b], ts[a:b])
        st_o, rem_o = orc.param_replay(rule_idx[a:b], acq[a:b], keys[a:b], ts[a:b])
        bad = np.nonzero((st_g != st_o) | (rem_g != rem_o))[0]
        assert len(bad) == 0, (universe, len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]])
    print(f"config4 universe={universe}: pass={(st_o == 0).mean():.3f} "
          f"over_capacity_bucket={orc.param_overflowed()} table={svc.param_table_stats()}")


@pytest.mark.parametrize("sample_count,interval_ms", [(4, 1000), (20, 1000), (32, 1600)])
def test_top_values_match_oracle(oracle_mod, sample_count, interval_ms):
    """ClusterParamMetric.getTopValues(5) of every rule (the snapshot's param leg) equals the oracle's,
    which is pinned by ClusterParamMetricTest (tests/golden/kat_cluster_param_metric.json).  Sample
    counts above 16 take k_ptop_sums' lanes over more than one pair of the window."""
    R = 300
    rng = np.random.default_rng(8)
    prules = [dict(flow_id=7000 + r, count=float(rng.integers(20, 200)), sample_count=sample_count,
                   window_interval_ms=interval_ms) for r in range(R)]
    svc = _svc(prules)
    orc = oracle_mod.TokenServiceOracle([], param_rules=prules)
    m = 200_000
    ts = T.timestamps(m, 150_000.0, T.T0_ALIGNED + 11)
    ridx = rng.integers(0, R, size=m).astype(np.int32)
    vals = T.zipf_indices(60, 1.3, m, rng, permute=False).astype(np.uint64)
    keys = (np.uint64(7000) + ridx.astype(np.uint64)) << np.uint64(24) | vals
    acq = rng.integers(1, 4, size=m).astype(np.int32)
    st_g, _ = svc.submit_param_batch_host(ridx, acq, keys, ts)
    st_o, _ = orc.param_replay(ridx, acq, keys, ts)
    assert np.array_equal(st_g, st_o)
    for t in (int(ts[-1]), int(ts[-1]) + 400, int(ts[-1]) + 5000):
        top = svc.param_top_values(t)
        for r in range(R):
            assert top[r] == orc.param_top_values(r, t), (t, r, top[r], orc.param_top_values(r, t))
    import torch
    from sentinel_amd import _lib
    snap = torch.zeros(R * _lib.PARAM_SNAPSHOT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    svc.param_snapshot_device(int(ts[-1]), snap)
    rec = snap.cpu().numpy().view(_lib.PARAM_SNAPSHOT_DTYPE)
    top = svc.param_top_values(int(ts[-1]))
    for r in range(R):
        assert rec["flow_id"][r] == 7000 + r and rec["n_top"][r] == len(top[r])
        assert [(int(k), float(v)) for k, v in zip(rec["key"][r][:len(top[r])], rec["avg"][r][:len(top[r])])] == top[r]


def test_top_values_expire_hints(oracle_mod):
    """The snapshot's expire hints (param_table.hpp: per slot the 1024-ms bucket from which its window
    sums to zero, kept by the key walk; k_ptop_sums then reads only slots whose window can be non-zero):
    a first snapshot computes them from the windows, later batches through the partition path keep them,
    and snapshots at times where some slots have just expired, all have, or none has, equal the oracle's
    getTopValues; a multi-value batch (the per-rule lanes, which do not keep hints) makes the next
    snapshot recompute them."""
    R = 200
    rng = np.random.default_rng(81)
    prules = [dict(flow_id=9000 + r, count=float(rng.integers(20, 300)), sample_count=10,
                   window_interval_ms=1000) for r in range(R)]
    svc = _svc(prules)
    orc = oracle_mod.TokenServiceOracle([], param_rules=prules)
    t0 = T.T0_ALIGNED + 17

    def check(ts_list):
        for t in ts_list:
            top = svc.param_top_values(t)
            for r in range(R):
                assert top[r] == orc.param_top_values(r, t), (t, r, top[r], orc.param_top_values(r, t))

    # (getTopValues rolls the reference's window to its ts -- LeapArray.currentWindow -- so every batch
    # starts after the previous snapshot time)
    for b in range(3):
        m = 60_000
        ts = np.sort(t0 + rng.integers(0, 2500, size=m)).astype(np.int64)
        t0 = int(ts[-1]) + 1101 + 50 * b
        ridx = rng.integers(0, R, size=m).astype(np.int32)
        vals = T.zipf_indices(80, 1.2, m, rng, permute=False).astype(np.uint64)
        keys = (np.uint64(9000) + ridx.astype(np.uint64)) << np.uint64(24) | vals
        acq = rng.integers(1, 3, size=m).astype(np.int32)
        st_g, _ = svc.submit_param_batch_host(ridx, acq, keys, ts)
        st_o, _ = orc.param_replay(ridx, acq, keys, ts)
        assert np.array_equal(st_g, st_o), b
        te = int(ts[-1])
        check((te, te + 600, te + 1100))
    check((te + 2100, te + 4000))
    t0 = te + 4001
    # a multi-value batch: the per-rule lanes write windows without hints
    m = 20_000
    ts = np.sort(t0 + rng.integers(0, 800, size=m)).astype(np.int64)
    ridx = rng.integers(0, R, size=m).astype(np.int32)
    b_, c_, k_ = T.param_value_lists(ridx, rng, universe=80, max_values=3)
    k_ = (np.uint64(9000) + (k_ >> np.uint64(20))) << np.uint64(24) | (k_ & np.uint64(0xFFFFF))
    acq = np.ones(m, np.int32)
    st_g, _ = svc.submit_param_multi_batch_host(ridx, acq, ts, b_, c_, k_)
    st_o, _ = orc.param_multi_replay(ridx, acq, ts, b_, c_, k_)
    assert np.array_equal(st_g, st_o)
    te = int(ts[-1])
    check((te, te + 950, te + 3000))


@pytest.mark.parametrize("path", ["part", "slot"])
def test_param_part_edges_bitexact(oracle_mod, monkeypatch, path):
    """Edge cases of the partition-local param path (param_part.hpp) against the oracle: one key hot
    enough to span many LDS chunks (and ranges far larger than a chunk), acquire counts past the packed
    field (escaped: read back from the event), a batch whose timestamps jump by 20 hours (ts - T0 past
    the packed 27-bit field), invalid requests (acquire <= 0, unknown rule, ts < 0) mixed in, hot items,
    and a second batch continuing every window.  Timestamps are non-decreasing per rule (the documented
    precondition of exact param parity)."""
    monkeypatch.setenv("SENTINEL_PARAM_PATH", path)
    R = 64
    rng = np.random.default_rng(29)
    prules = [dict(flow_id=500 + r, count=float(rng.integers(3, 400)), sample_count=(2, 4, 5, 10)[r % 4],
                   window_interval_ms=1000) for r in range(R)]
    fids = np.array([r["flow_id"] for r in prules], dtype=np.uint64)
    hot_key = int((fids[3] << np.uint64(32)) | np.uint64(7))
    prules[3]["hot"] = {hot_key: 50_000}
    svc = _svc(prules)
    orc = oracle_mod.TokenServiceOracle([], param_rules=prules,
                                        hot_items={3: [(hot_key, 50_000)]})
    t0 = T.T0_ALIGNED + 13
    for batch in range(2):
        m = 60_000
        ts = np.sort(t0 + rng.integers(0, 3000, size=m)).astype(np.int64)
        ts[m // 2:] += 20 * 3600 * 1000                  # a 20 h jump inside the batch
        ridx = rng.integers(0, R, size=m).astype(np.int32)
        vals = T.zipf_indices(400, 1.1, m, rng, permute=False).astype(np.uint64)
        keys = (fids[ridx] << np.uint64(32)) | vals
        hot = rng.random(m) < 0.5                          # half the batch on one key (~15 chunks)
        ridx[hot] = 3
        keys[hot] = hot_key
        acq = np.where(rng.random(m) < 0.1, rng.integers(400, 3000, size=m), 1).astype(np.int32)
        bad = rng.random(m)
        acq[bad < 0.002] = 0                               # BAD_REQUEST
        ridx[(bad >= 0.002) & (bad < 0.004)] = R + 5       # NO_RULE_EXISTS
        ts[(bad >= 0.004) & (bad < 0.005)] = -1            # FAIL (the reference's NPE)
        st_g, rem_g = svc.submit_param_batch_host(ridx, acq, keys, ts)
        st_o, rem_o = orc.param_replay(ridx, acq, keys, ts)
        mis = np.nonzero((st_g != st_o) | (rem_g != rem_o))[0]
        assert len(mis) == 0, (batch, len(mis), mis[:5], st_g[mis[:5]], st_o[mis[:5]], rem_g[mis[:5]], rem_o[mis[:5]])
        assert {-4, -1, 0, 1, 3} <= set(np.unique(st_o).tolist())
        t0 = int(ts.max()) + 1
    t = t0
    for i in range(0, 3000, 41):
        r, k = int(ridx[i]), int(keys[i])
        if 0 <= r < R:
            assert svc.param_sum(r, k, t) == orc.param_sum(r, t, k)
