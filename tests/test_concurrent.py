"""Cluster concurrency tokens (ConcurrentClusterFlowChecker): the oracle pinned by the reference's
ConcurrentClusterFlowCheckerTest (CPU), and the GPU engine against the oracle over batches of
interleaved acquires / releases, rule reloads and expiry sweeps (GPU)."""
import numpy as np
import pytest

from sentinel_amd import trace as T


def _rule(flow_id=111, count=10.0, threshold_type=1):
    return dict(flow_id=flow_id, count=count, threshold_type=threshold_type, sample_count=10, window_interval_ms=1000,
                namespace_idx=0, checker=0)


def _events(oracle_mod, kinds, flow_idx=0, acquire=1, tokens=None, flags=1):
    n = len(kinds)
    ev = np.zeros(n, dtype=oracle_mod.TokenServiceOracle.CONC_EVENT)
    ev["kind"] = kinds
    ev["flow_idx"] = flow_idx
    ev["acquire"] = acquire
    ev["flags"] = flags
    if tokens is not None:
        ev["token_id"] = tokens
    return ev


def test_oracle_matches_reference_concurrent_test(oracle_mod):
    """ConcurrentClusterFlowCheckerTest.java:61-84 (testEasyAcquireAndRelease) and :115-124 (expiry)."""
    o = oracle_mod.TokenServiceOracle([_rule()])
    st, tok = o.concurrent_replay(_events(oracle_mod, [0] * 20), np.arange(1, 21))
    assert list(st[:10]) == [0] * 10 and (tok[:10] != 0).all()
    assert list(st[10:]) == [1] * 10                       # BLOCKED once nowCalls == count
    st, _ = o.concurrent_replay(_events(oracle_mod, [1] * 10, tokens=tok[:10]), np.zeros(10))
    assert list(st) == [6] * 10                            # RELEASE_OK
    assert o.concurrent_now_calls(0) == 0 and o.concurrent_token_count() == 0
    st, _ = o.concurrent_replay(_events(oracle_mod, [1], tokens=tok[:1]), np.zeros(1))
    assert list(st) == [7]                                 # ALREADY_RELEASE
    o.concurrent_replay(_events(oracle_mod, [0] * 10), np.arange(100, 110))
    assert o.concurrent_expire_all() == 10
    assert o.concurrent_now_calls(0) == 0 and o.concurrent_token_count() == 0
    # validation (DefaultTokenService.java:64-75, 89-91): no address, bad id, count <= 0, unknown rule
    st, _ = o.concurrent_replay(np.concatenate([_events(oracle_mod, [0], flags=0), _events(oracle_mod, [0], flow_idx=-2),
                                                _events(oracle_mod, [0], acquire=0), _events(oracle_mod, [0], flow_idx=-1)]),
                                np.arange(4))
    assert list(st) == [-4, -4, -4, 3]


@pytest.mark.gpu
def test_gpu_reference_sequence():
    import sentinel_amd as sa
    svc = sa.GpuTokenService(0)
    svc.load_flow_rules([sa.FlowRule(count=10, cluster_config=sa.ClusterFlowConfig(flow_id=111, threshold_type=1))])
    res = [svc.request_concurrent_token("127.0.0.1", 111, 1) for _ in range(20)]
    assert all(r.status == 0 and r.token_id != 0 for r in res[:10])
    assert all(r.status == 1 for r in res[10:])
    assert len({r.token_id for r in res[:10]}) == 10
    assert all(svc.release_concurrent_token(r.token_id).status == 6 for r in res[:10])
    assert svc.concurrent_now_calls(0) == 0 and svc.concurrent_token_count() == 0
    assert svc.release_concurrent_token(res[0].token_id).status == 7
    assert svc.release_concurrent_token(None) is None
    for _ in range(10):
        svc.request_concurrent_token("127.0.0.1", 111, 1)
    assert svc.concurrent_expire(1000) == 10
    assert svc.concurrent_now_calls(0) == 0 and svc.concurrent_token_count() == 0
    assert svc.request_concurrent_token("", 111, 1).status == -4
    assert svc.request_concurrent_token("a", 999, 1).status == 3


@pytest.mark.gpu
@pytest.mark.parametrize("capacity", [None, "16384"])
def test_gpu_concurrent_batches_match_oracle(oracle_mod, monkeypatch, capacity):
    """capacity 16384: the token cache starts small, so batches keep crossing the host's bound on live +
    tombstones -- the tombstone sweep (k_tok_sweep), the compaction and the growth all run between
    batches and every later release must still find its token."""
    import sentinel_amd as sa
    from sentinel_amd.token_service import ServerNamespace
    if capacity:
        monkeypatch.setenv("SENTINEL_TOKEN_CAPACITY", capacity)
    rng = np.random.default_rng(71)
    F = 400

    def make_rules(ids):
        return [_rule(int(f), float(rng.integers(1, 12)), int(rng.integers(0, 2))) for f in ids]
    rules = make_rules(np.arange(1, F + 1))
    svc = sa.GpuTokenService(0)
    svc.set_namespaces([ServerNamespace(connected_count=3)])
    svc.load_flow_rules([sa.FlowRule(count=r["count"], cluster_config=sa.ClusterFlowConfig(
        flow_id=r["flow_id"], threshold_type=r["threshold_type"])) for r in rules])
    orc = oracle_mod.TokenServiceOracle(rules, namespaces=[dict(connected_count=3)])
    outstanding = []
    for b in range(12):
        if b == 6:   # reload: flows 1..100 removed, 401..450 added, the rest kept (nowCalls carried)
            rules = rules[100:] + make_rules(np.arange(F + 1, F + 51))
            svc.load_flow_rules([sa.FlowRule(count=r["count"], cluster_config=sa.ClusterFlowConfig(
                flow_id=r["flow_id"], threshold_type=r["threshold_type"])) for r in rules])
            orc.reload_flow_rules(rules)
        n = int(rng.integers(2000, 6000))
        kind = (rng.random(n) < 0.35).astype(np.int32)
        if not outstanding:
            kind[:] = 0
        fidx = T.zipf_indices(len(rules), 1.1, n, rng)
        acq = rng.integers(1, 4, size=n).astype(np.int32)
        flags = (rng.random(n) > 0.01).astype(np.uint32)
        tok = np.zeros(n, np.int64)
        rel = np.nonzero(kind == 1)[0]
        if len(rel):
            pick = rng.integers(0, len(outstanding), size=len(rel))
            tok[rel] = np.array(outstanding, np.int64)[pick]     # repeats -> ALREADY_RELEASE
            tok[rel[::53]] = 12345                               # never issued
        fidx[::211] = -1                                         # unknown rule
        st_g, tok_g = svc.submit_concurrent_batch_host(fidx, acq, tok, kind, flags)
        ev = np.zeros(n, dtype=orc.CONC_EVENT)
        ev["flow_idx"], ev["acquire"], ev["token_id"], ev["kind"], ev["flags"] = fidx, acq, tok, kind, flags
        st_o, tok_o = orc.concurrent_replay(ev, tok_g)
        bad = np.nonzero(st_g != st_o)[0]
        assert len(bad) == 0, (b, len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]], kind[bad[:5]])
        ok = st_g == 0
        assert (tok_g[ok] != 0).all() and len(np.unique(tok_g[ok])) == int(ok.sum())
        released = set(tok[(kind == 1) & (st_g == 6)].tolist())
        outstanding = [t for t in outstanding if t not in released] + tok_g[ok].tolist()
        for f in range(0, len(rules), 7):
            assert svc.concurrent_now_calls(f) == orc.concurrent_now_calls(f), (b, f)
        assert svc.concurrent_token_count() == orc.concurrent_token_count()
        if b in (3, 9) and svc.concurrent_token_count() <= 1000:
            assert svc.concurrent_expire(1000) == orc.concurrent_expire_all()
            outstanding = []
    assert {0, 1, 3, 6, 7, -4} <= set(np.unique(st_o).tolist()) | {6, 7}


def _device_batch(svc, fidx, acq, tok, kind, flags):
    import torch
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)   # noqa: E731
    ev = svc.concurrent_events(t(fidx.astype(np.int32)), t(acq.astype(np.int32)), t(tok.astype(np.int64)),
                               t(kind.astype(np.int32)), t(flags.astype(np.int32)))
    res = torch.full((len(kind), 2), -99, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()            # the events (and the fill) were made on torch's stream
    svc.submit_concurrent_batch(ev, results=res)
    svc.synchronize()
    r = res.cpu().numpy()
    assert (r[:, 1] != -99).all(), "an event without a result"
    return r[:, 1].astype(np.int32).astype(np.int8), r[:, 0].copy()


@pytest.mark.gpu
def test_gpu_concurrent_device_hot_flows_match_oracle(oracle_mod):
    """The device-pointer path (sentinel_submit_concurrent_batch) on hot flows: segments of thousands of
    events span many scan tiles (k_conc_scan's look-back over tile descriptors); segments with an
    acquire of 2 tokens and, after the reload that lowers every count while tokens are out, segments
    starting above their new threshold go to the one-thread walk (k_conc_serial, its start found by a
    binary search); fractional / tiny / AVG_LOCAL thresholds and duplicate releases in a batch."""
    import sentinel_amd as sa
    from sentinel_amd.token_service import ServerNamespace
    rng = np.random.default_rng(404)
    F = 64

    def make_rules(ids, scale=1.0):
        return [_rule(int(f), float(np.round(rng.uniform(0.5, 400.0) * scale, 1)), int(rng.integers(0, 2)))
                for f in ids]
    rules = make_rules(np.arange(1, F + 1))
    svc = sa.GpuTokenService(0)
    svc.set_namespaces([ServerNamespace(connected_count=2)])

    def load(rs):
        svc.load_flow_rules([sa.FlowRule(count=r["count"], cluster_config=sa.ClusterFlowConfig(
            flow_id=r["flow_id"], threshold_type=r["threshold_type"])) for r in rs])
    load(rules)
    orc = oracle_mod.TokenServiceOracle(rules, namespaces=[dict(connected_count=2)])
    outstanding = []
    for b in range(10):
        if b == 5:   # every count divided by 4: flows with tokens out start above their threshold
            rules = [dict(r, count=float(np.round(r["count"] / 4.0, 1))) for r in rules]
            load(rules)
            orc.reload_flow_rules(rules)
        n = int(rng.integers(20_000, 40_000))
        kind = (rng.random(n) < 0.45).astype(np.int32)
        if not outstanding:
            kind[:] = 0
        fidx = T.zipf_indices(len(rules), 1.3, n, rng)
        acq = np.ones(n, np.int32)
        if b % 3 == 2:
            acq[rng.random(n) < 0.02] = 2                                   # some chunks leave the scan
        flags = np.ones(n, np.int32)
        tok = np.zeros(n, np.int64)
        rel = np.nonzero(kind == 1)[0]
        if len(rel):
            pick = rng.integers(0, len(outstanding), size=len(rel))
            tok[rel] = np.array(outstanding, np.int64)[pick]                # repeats -> ALREADY_RELEASE
            tok[rel[::97]] = 777                                             # never issued
            tok[rel[1::389]] = -1                                            # the cache's empty-slot and
            tok[rel[2::389]] = -2                                            # tombstone markers as ids
        st_g, tok_g = _device_batch(svc, fidx, acq, tok, kind, flags)
        ev = np.zeros(n, dtype=orc.CONC_EVENT)
        ev["flow_idx"], ev["acquire"], ev["token_id"], ev["kind"], ev["flags"] = fidx, acq, tok, kind, flags
        st_o, tok_o = orc.concurrent_replay(ev, tok_g)
        bad = np.nonzero(st_g != st_o)[0]
        assert len(bad) == 0, (b, len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]], kind[bad[:5]], fidx[bad[:5]])
        ok = st_g == 0
        assert (tok_g[ok] != 0).all() and len(np.unique(tok_g[ok])) == int(ok.sum())
        released = set(tok[(kind == 1) & (st_g == 6)].tolist())
        outstanding = [t for t in outstanding if t not in released] + tok_g[ok].tolist()
        for f in range(len(rules)):
            assert svc.concurrent_now_calls(f) == orc.concurrent_now_calls(f), (b, f)
        assert svc.concurrent_token_count() == orc.concurrent_token_count()
    assert {0, 1, 6, 7} <= set(np.unique(st_o).tolist())


@pytest.mark.gpu
def test_gpu_qps_and_concurrent_batches_interleaved(oracle_mod):
    """QPS requestToken batches (ClusterFlowChecker) and concurrency-token batches
    (ConcurrentClusterFlowChecker) interleaved on one engine and one rule table, against the oracle
    doing the same: the two checkers keep separate state (the flow's ClusterMetric vs nowCalls / the
    token cache) and neither batch kind disturbs the other."""
    import sentinel_amd as sa
    rng = np.random.default_rng(505)
    F = 300
    rules = [_rule(int(f), float(rng.integers(2, 60)), 1) for f in range(1, F + 1)]
    svc = sa.GpuTokenService(0)
    svc.load_flow_rules([sa.FlowRule(count=r["count"], cluster_config=sa.ClusterFlowConfig(
        flow_id=r["flow_id"], threshold_type=1)) for r in rules])
    orc = oracle_mod.TokenServiceOracle(rules)
    t = T.T0_ALIGNED + 3
    outstanding = []
    for b in range(8):
        if b % 2 == 0:
            n = 30_000
            idx = T.zipf_indices(F, 1.1, n, rng)
            acq = rng.integers(1, 3, size=n).astype(np.int32)
            ts = np.sort(t + rng.integers(0, 1500, size=n)).astype(np.int64)
            t += 1500
            st_g, rem_g, _ = svc.submit_flow_batch_host(idx, acq, ts)
            st_o, rem_o = orc.replay(idx, acq, ts)[:2]
            bad = np.nonzero((st_g != st_o) | (rem_g != rem_o))[0]
            assert len(bad) == 0, (b, len(bad), bad[:5])
        else:
            n = 20_000
            kind = (rng.random(n) < 0.4).astype(np.int32)
            if not outstanding:
                kind[:] = 0
            fidx = T.zipf_indices(F, 1.1, n, rng)
            acq = np.ones(n, np.int32)
            tok = np.zeros(n, np.int64)
            rel = np.nonzero(kind == 1)[0]
            if len(rel):
                tok[rel] = np.array(outstanding, np.int64)[rng.integers(0, len(outstanding), size=len(rel))]
            st_g, tok_g = _device_batch(svc, fidx, acq, tok, kind, np.ones(n, np.int32))
            ev = np.zeros(n, dtype=orc.CONC_EVENT)
            ev["flow_idx"], ev["acquire"], ev["token_id"], ev["kind"], ev["flags"] = fidx, acq, tok, kind, 1
            st_o, _ = orc.concurrent_replay(ev, tok_g)
            bad = np.nonzero(st_g != st_o)[0]
            assert len(bad) == 0, (b, len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]])
            ok = st_g == 0
            released = set(tok[(kind == 1) & (st_g == 6)].tolist())
            outstanding = [x for x in outstanding if x not in released] + tok_g[ok].tolist()
    for f in range(0, F, 11):
        assert svc.concurrent_now_calls(f) == orc.concurrent_now_calls(f)


@pytest.mark.gpu
def test_gpu_concurrent_mixed_amounts_tombstone_reuse(oracle_mod, monkeypatch):
    """Acquires of 1..5 tokens and releases of the previous batches' tokens share every batch, on 3000
    flows, through a small token cache: inserts of a batch reuse the tombstones its own releases leave.
    A release's amount must be its own token's (read before its slot can be reused), so nowCalls of
    every flow and every status equal the oracle's."""
    import sentinel_amd as sa
    monkeypatch.setenv("SENTINEL_TOKEN_CAPACITY", "16384")
    rng = np.random.default_rng(808)
    F = 3000
    rules = [_rule(int(f), float(rng.integers(4, 40)), 1) for f in range(1, F + 1)]
    svc = sa.GpuTokenService(0)
    svc.load_flow_rules([sa.FlowRule(count=r["count"], cluster_config=sa.ClusterFlowConfig(
        flow_id=r["flow_id"], threshold_type=1)) for r in rules])
    orc = oracle_mod.TokenServiceOracle(rules)
    outstanding = []
    for b in range(10):
        n = 24_000
        kind = (rng.random(n) < 0.5).astype(np.int32)
        if not outstanding:
            kind[:] = 0
        fidx = T.zipf_indices(F, 0.9, n, rng)
        acq = rng.integers(1, 6, size=n).astype(np.int32)
        tok = np.zeros(n, np.int64)
        rel = np.nonzero(kind == 1)[0]
        if len(rel):
            pool = np.array(outstanding, np.int64)
            tok[rel] = pool[rng.permutation(len(pool))[:len(rel)]] if len(pool) >= len(rel) else pool[rng.integers(0, len(pool), size=len(rel))]
        st_g, tok_g = _device_batch(svc, fidx, acq, tok, kind, np.ones(n, np.int32))
        ev = np.zeros(n, dtype=orc.CONC_EVENT)
        ev["flow_idx"], ev["acquire"], ev["token_id"], ev["kind"], ev["flags"] = fidx, acq, tok, kind, 1
        st_o, _ = orc.concurrent_replay(ev, tok_g)
        bad = np.nonzero(st_g != st_o)[0]
        assert len(bad) == 0, (b, len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]])
        released = set(tok[(kind == 1) & (st_g == 6)].tolist())
        outstanding = [x for x in outstanding if x not in released] + tok_g[st_g == 0].tolist()
        for f in range(0, F, 13):
            assert svc.concurrent_now_calls(f) == orc.concurrent_now_calls(f), (b, f)
        assert svc.concurrent_token_count() == orc.concurrent_token_count()
    assert (st_o == 6).any() and (st_o == 1).any() and (st_o == 0).any()


@pytest.mark.gpu
def test_gpu_token_inserts_contended(oracle_mod, monkeypatch):
    """Many passing acquires inserting into a small token cache at once (12k inserts into 16384 slots,
    every acquire admitted): lost CASes on shared probe paths are the common case here.  Round 4's
    r04e / r04f hang was token_insert re-reading a slot with a plain load after
    losing its CAS: the CU's L1 kept answering the stale free key, so the lane retried the same slot
    up to capacity times.  Bit-exact statuses, unique tokens, and every token released afterwards."""
    import sentinel_amd as sa
    from sentinel_amd.token_service import ServerNamespace
    monkeypatch.setenv("SENTINEL_TOKEN_CAPACITY", "16384")
    F = 64
    rules = [_rule(int(f), 1e6, 1) for f in range(1, F + 1)]
    svc = sa.GpuTokenService(0)
    svc.set_namespaces([ServerNamespace(connected_count=1)])
    svc.load_flow_rules([sa.FlowRule(count=r["count"], cluster_config=sa.ClusterFlowConfig(
        flow_id=r["flow_id"], threshold_type=r["threshold_type"])) for r in rules])
    orc = oracle_mod.TokenServiceOracle(rules, namespaces=[dict(connected_count=1)])
    rng = np.random.default_rng(5)
    n = 12_000
    fidx = rng.integers(0, F, n).astype(np.int32)
    acq = np.ones(n, np.int32)
    kind = np.zeros(n, np.int32)
    flags = np.ones(n, np.uint32)
    st_g, tok_g = svc.submit_concurrent_batch_host(fidx, acq, np.zeros(n, np.int64), kind, flags)
    ev = np.zeros(n, dtype=orc.CONC_EVENT)
    ev["flow_idx"], ev["acquire"], ev["token_id"], ev["kind"], ev["flags"] = fidx, acq, 0, kind, flags
    st_o, _ = orc.concurrent_replay(ev, tok_g)
    assert np.array_equal(st_g, st_o) and (st_g == 0).all()
    assert len(np.unique(tok_g)) == n and svc.concurrent_token_count() == n
    rel = np.ones(n, np.int32)
    st_r, _ = svc.submit_concurrent_batch_host(fidx, acq, tok_g, rel, flags)
    assert (st_r == 6).all() and svc.concurrent_token_count() == 0


@pytest.mark.gpu
def test_conc_bench_shape_bitexact(oracle_mod):
    """The bench's own 5conc shape (bench.py ConcWorkload): 20k thread-grade rules (count~U{50..5000}),
    Zipf(1.1) flows, 4M-event batches of which half acquire one token and half release, at fixed
    positions, the tokens the previous batch handed out, first in first out (blocked acquires hold none:
    ALREADY_RELEASE);
    3 batches on the device-pointer path, every status, every flow's nowCalls and the cache size against
    the oracle's sequential replay with the engine's token ids."""
    import sentinel_amd as sa
    rng = np.random.default_rng(55)
    F = 20_000
    rules = T.make_rules(F, rng, count_lo=50, count_hi=5000, sample_count=1, window_interval_ms=1000)
    svc = sa.GpuTokenService(0)
    svc.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count,
                         rules.window_interval_ms, rules.namespace, rules.checker)
    orc = oracle_mod.TokenServiceOracle.from_arrays(rules.flow_id, rules.count, rules.threshold_type,
                                                    rules.sample_count, rules.window_interval_ms, rules.namespace,
                                                    rules.checker)
    N = 4 * 1024 * 1024
    perm = rng.permutation(N)
    acq_pos, rel_pos = np.sort(perm[: N // 2]), np.sort(perm[N // 2:])
    rel_src = acq_pos[np.sort(rng.permutation(len(acq_pos))[: len(rel_pos)])]   # (first in, first out)
    w = 1.0 / np.power(np.arange(1, F + 1, dtype=np.float64), 1.1)
    cdf = np.cumsum(w) / w.sum()
    zperm = np.random.default_rng(9).permutation(F).astype(np.int32)
    erng = np.random.default_rng(3000)
    prev_tok = np.zeros(N, np.int64)
    for b in range(3):
        fidx = zperm[np.minimum(np.searchsorted(cdf, erng.random(N), side="right"), F - 1)]
        kind = np.zeros(N, np.int32)
        kind[rel_pos] = 1
        tok = np.zeros(N, np.int64)
        tok[rel_pos] = prev_tok[rel_src]
        acq = np.ones(N, np.int32)
        flags = np.ones(N, np.int32)
        st_g, tok_g = _device_batch(svc, fidx, acq, tok, kind, flags)
        ev = np.zeros(N, dtype=orc.CONC_EVENT)
        ev["flow_idx"], ev["acquire"], ev["token_id"], ev["kind"], ev["flags"] = fidx, acq, tok, kind, flags
        st_o, _ = orc.concurrent_replay(ev, tok_g)
        bad = np.nonzero(st_g != st_o)[0]
        assert len(bad) == 0, (b, len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]], kind[bad[:5]])
        ok = st_g == 0
        assert len(np.unique(tok_g[ok])) == int(ok.sum())
        if b > 0:
            assert {0, 1, 6, 7} <= set(np.unique(st_g).tolist())
        for f in range(0, F, 37):
            assert svc.concurrent_now_calls(f) == orc.concurrent_now_calls(f), (b, f)
        assert svc.concurrent_token_count() == orc.concurrent_token_count()
        prev_tok = np.where(ok, tok_g, 0)


@pytest.mark.gpu
def test_bench_glue_forwards_release_tokens():
    """bench.py's 5conc client traffic (tools/bench_glue.hip): word 1 of event row rel_pos[i] gets word 0
    of result row rel_src[i]; every other word is untouched -- the numpy statement of the same copy, on a
    ragged count (not a multiple of the kernel's 1024 items per workgroup)."""
    import ctypes
    import os
    import torch
    so = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "libbench_glue.so")
    lib = ctypes.CDLL(so)
    lib.bench_glue_forward_tokens.restype = ctypes.c_int
    lib.bench_glue_forward_tokens.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_void_p]
    rng = np.random.default_rng(77)
    N = 300_001
    perm = rng.permutation(N)
    acq_pos, rel_pos = np.sort(perm[: N // 2]), np.sort(perm[N // 2:])
    rel_src = acq_pos[np.sort(rng.permutation(len(acq_pos))[: len(rel_pos) - 3])]
    rel_pos = rel_pos[: len(rel_src)]
    ev = rng.integers(-2**62, 2**62, size=(N, 3), dtype=np.int64)
    prev = rng.integers(-2**62, 2**62, size=(N, 2), dtype=np.int64)
    want = ev.copy()
    want[rel_pos, 1] = prev[rel_src, 0]
    dev = torch.device("cuda:0")
    ev_d, prev_d = torch.from_numpy(ev).to(dev), torch.from_numpy(prev).to(dev)
    pos_d = torch.from_numpy(rel_pos.astype(np.int32)).to(dev)
    src_d = torch.from_numpy(rel_src.astype(np.int32)).to(dev)
    torch.cuda.synchronize()
    assert lib.bench_glue_forward_tokens(ev_d.data_ptr(), prev_d.data_ptr(), pos_d.data_ptr(), src_d.data_ptr(),
                                         len(rel_pos), None) == 0
    torch.cuda.synchronize()
    assert np.array_equal(ev_d.cpu().numpy(), want)
