"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle on the same seeded traces.

Bar: bit-exact statuses, remaining counts, waitInMs and the final window counters of every touched
flow.  Full-size cases check size-independent properties instead (conservation, admission bound,
determinism).
"""
import numpy as np
import pytest

from sentinel_amd import trace as T

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["sorted", "partition", "ordered", "ordered-sorted", "small"])
def flow_path(request, monkeypatch):
    """Every flow parity case runs on every flow pipeline: the global radix sort, the
    partition-local path (prep + scan + multi-split + k_part_half), the same with decide-order output
    ("ordered": sentinel_submit_flow_batch_ordered[_host], its verdicts put back at their arrival
    positions through the returned seq -- a permutation of [0, n) -- before the comparison; "ordered-sorted":
    the same output from the radix-sort path), and the one-launch small-batch kernel over 4096-event chunks
    (the variable is read when an engine is created)."""
    path = {"ordered": "partition", "ordered-sorted": "sorted"}.get(request.param, request.param)
    monkeypatch.setenv("SENTINEL_FLOW_PATH", path)
    if request.param.startswith("ordered"):
        from sentinel_amd.token_service import GpuTokenService

        def host(self, flow_idx, acquire, ts, flags=None):
            st, rem, w, seq = self.submit_flow_batch_ordered_host(flow_idx, acquire, ts, flags)
            n = len(seq)
            assert np.array_equal(np.sort(seq), np.arange(n, dtype=np.uint32)), "seq is not a permutation"
            out = [np.empty_like(st), np.empty_like(rem), np.empty_like(w)]
            for o, x in zip(out, (st, rem, w)):
                o[seq.astype(np.int64)] = x
            return tuple(out)

        def device(self, events, flags=None, verdicts=None, stream=None):
            import torch
            v, seq = self.submit_flow_batch_ordered(events, flags=flags, stream=stream)
            self.synchronize()
            n = int(events.shape[0])
            s = seq.to(torch.int64)
            assert torch.equal(torch.sort(s).values, torch.arange(n, device=s.device)), "seq is not a permutation"
            out = verdicts if verdicts is not None else torch.empty(n, dtype=torch.int64, device=events.device)
            out[s] = v
            return out

        monkeypatch.setattr(GpuTokenService, "submit_flow_batch_host", host)
        monkeypatch.setattr(GpuTokenService, "submit_flow_batch", device)
    return request.param


def _engine(rules, namespaces=None, exceed=1.0, occ=1.0):
    import sentinel_amd as sa
    from sentinel_amd.token_service import ServerNamespace
    svc = sa.GpuTokenService(0, exceed_count=exceed, max_occupy_ratio=occ)
    if namespaces is not None:
        svc.set_namespaces([ServerNamespace(**n) for n in namespaces])
    svc.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count,
                         rules.window_interval_ms, rules.namespace, rules.checker)
    return svc


def _oracle(oracle_mod, rules, namespaces=None, exceed=1.0, occ=1.0):
    return oracle_mod.TokenServiceOracle(rules.as_dicts(), namespaces=namespaces, exceed_count=exceed,
                                         max_occupy_ratio=occ)


def _compare(svc, orc, rules, ev, check_state=True, batches=1):
    bounds = np.linspace(0, len(ev), batches + 1).astype(int)
    for b in range(batches):
        e = ev.slice(bounds[b], bounds[b + 1])
        st_g, rem_g, w_g = svc.submit_flow_batch_host(e.flow_idx, e.acquire, e.ts, e.flags)
        st_o, rem_o, w_o = orc.replay(e.flow_idx, e.acquire, e.ts, e.flags)
        bad = np.nonzero((st_g != st_o) | (rem_g != rem_o) | (w_g != w_o))[0]
        assert len(bad) == 0, (f"batch {b}: {len(bad)} mismatches, first at {bad[:5]}: "
                               f"gpu={st_g[bad[:5]]},{rem_g[bad[:5]]},{w_g[bad[:5]]} "
                               f"oracle={st_o[bad[:5]]},{rem_o[bad[:5]]},{w_o[bad[:5]]}")
    if check_state:
        touched = np.unique(ev.flow_idx[(ev.flow_idx >= 0) & (ev.flow_idx < len(rules))])
        for f in touched[:2000]:
            n = int(rules.sample_count[f])
            g = svc.dump_flow(int(f), n)
            o = orc.dump_flow(int(f))
            assert np.array_equal(g, o), (f, g, o)


def test_config2_small_bitexact(oracle_mod):
    rules, ev = T.config2(200_000, seed=2, n_flows=1000)
    _compare(_engine(rules), _oracle(oracle_mod, rules), rules, ev, batches=3)


def test_lookback_generation_and_ticket_wrap(oracle_mod, monkeypatch):
    """The radix path's look-back words carry a 30-bit launch generation and the tile tickets a host-tracked
    32-bit base (scan_sort.hpp, LBState): an engine started a few launches before both wrap
    (SENTINEL_LB_START) decides ten batches across the wraps bit-exactly.  A 20k-event batch takes ~7 tickets
    over 3 look-back launches, so the ticket count wraps around launch 17 and the generation (which re-zeroes
    the words) at launch 26 of ~30."""
    monkeypatch.setenv("SENTINEL_LB_START", f"{(1 << 30) - 26},{(1 << 32) - 40}")
    rules, ev = T.config2(200_000, seed=21, n_flows=1000)
    _compare(_engine(rules), _oracle(oracle_mod, rules), rules, ev, batches=10)


def test_config3_shape_bitexact(oracle_mod):
    rules, ev = T.config3(300_000, seed=3, n_flows=20_000, sample_count=10, window_interval_ms=1000)
    _compare(_engine(rules), _oracle(oracle_mod, rules), rules, ev, batches=2)


def test_unaligned_t0_and_odd_windows(oracle_mod):
    rng = np.random.default_rng(11)
    rules = T.make_rules(300, rng, count_lo=1, count_hi=200, sample_count=3, window_interval_ms=1500, integral=False)
    rules.sample_count[::2] = 5
    rules.window_interval_ms[::2] = 25
    rules.sample_count[1::5] = 1
    rules.window_interval_ms[1::5] = 1000
    ev = T.Events(T.zipf_indices(300, 1.05, 60_000, rng), np.ones(60_000, np.int32),
                  T.timestamps(60_000, 20_000.0, T.T0_ALIGNED + 137))
    _compare(_engine(rules, exceed=1.3), _oracle(oracle_mod, rules, exceed=1.3), rules, ev, batches=4)


def test_heterogeneous_rls_config5(oracle_mod):
    rules, ev = T.config5(100_000, seed=5, n_flows=500)
    _compare(_engine(rules), _oracle(oracle_mod, rules), rules, ev, batches=2)


def test_config5_hot_heterogeneous(oracle_mod):
    """BASELINE config 5's shape: 2000 RLS rules, Zipf(1.1) -- the hottest flow takes ~17% of a batch,
    with geometric hitsAddend.  Its heterogeneous segments (hundreds of thousands of events, both below
    and past the threshold) are decided by a whole workgroup (coop_het) on both flow paths."""
    rules, ev = T.config5(2_000_000, seed=55, n_flows=2000)
    _compare(_engine(rules), _oracle(oracle_mod, rules), rules, ev, batches=4)


def test_hot_runs_on_the_batch_stream(oracle_mod, monkeypatch):
    """The hot runs (launch_long) normally go to the engine's aux stream, concurrent with the wave runs and
    the verdict kernel (engine.hip, run_pipeline); SENTINEL_HOT_FORK=0 keeps them on the batch's stream in
    order.  Both schedules decide config 5's hot heterogeneous shape bit-exactly."""
    monkeypatch.setenv("SENTINEL_HOT_FORK", "0")
    rules, ev = T.config5(1_000_000, seed=56, n_flows=2000)
    _compare(_engine(rules), _oracle(oracle_mod, rules), rules, ev, batches=3)


def test_hot_heterogeneous_mixed(oracle_mod):
    """A hot flow whose heterogeneous segments are interleaved with prioritized requests, a clock that
    steps back and small thresholds (saturated after a few events) next to huge ones (never
    saturated): the cooperative walk hands over to the sequential path and back."""
    rng = np.random.default_rng(57)
    rules = T.make_rules(64, rng, count_lo=3, count_hi=50, sample_count=2, window_interval_ms=500)
    rules.count[5] = 1e6
    n = 400_000
    idx = rng.integers(0, 64, size=n).astype(np.int32)
    hot = rng.random(n)
    idx[hot < 0.45] = 3
    idx[(hot >= 0.45) & (hot < 0.75)] = 5
    acq = np.minimum(rng.geometric(0.4, size=n), 40).astype(np.int32)
    ts = T.timestamps(n, 200_000.0, T.T0_ALIGNED + 3)
    ts = ts + np.where(rng.random(n) < 0.0005, -rng.integers(0, 900, size=n), 0)
    flags = (rng.random(n) < 0.0003).astype(np.uint8)
    ev = T.Events(idx, acq, ts.astype(np.int64), flags)
    _compare(_engine(rules, occ=0.9), _oracle(oracle_mod, rules, occ=0.9), rules, ev, batches=2)


def test_homogeneous_acquire_gt1(oracle_mod):
    rng = np.random.default_rng(7)
    rules = T.make_rules(200, rng, count_lo=5, count_hi=300)
    ev = T.Events(T.zipf_indices(200, 1.2, 50_000, rng), np.full(50_000, 3, np.int32),
                  T.timestamps(50_000, 30_000.0, T.T0_ALIGNED))
    _compare(_engine(rules), _oracle(oracle_mod, rules), rules, ev, batches=2)


def test_large_acquire_escape(oracle_mod):
    """acquireCount >= 2047 does not fit the 11-bit field of the sorted value (escape path)."""
    rng = np.random.default_rng(37)
    rules = T.make_rules(80, rng, count_lo=20_000, count_hi=400_000)
    n = 30_000
    acq = np.where(rng.random(n) < 0.5, 3000, 2047).astype(np.int32)
    acq[::7] = 1
    ev = T.Events(rng.integers(0, 80, size=n).astype(np.int32), acq, T.timestamps(n, 30_000.0, T.T0_ALIGNED))
    _compare(_engine(rules), _oracle(oracle_mod, rules), rules, ev, batches=2)
    ev = T.Events(rng.integers(0, 80, size=n).astype(np.int32), np.full(n, 5000, np.int32),
                  T.timestamps(n, 30_000.0, T.T0_ALIGNED + 2000))
    _compare(_engine(rules), _oracle(oracle_mod, rules), rules, ev, batches=1)


def test_prioritized_occupy(oracle_mod):
    rng = np.random.default_rng(13)
    rules = T.make_rules(50, rng, count_lo=3, count_hi=40, sample_count=5, window_interval_ms=1000)
    n = 40_000
    ev = T.Events(T.zipf_indices(50, 1.0, n, rng), np.ones(n, np.int32), T.timestamps(n, 3000.0, T.T0_ALIGNED + 3),
                  flags=(rng.random(n) < 0.3).astype(np.uint8))
    _compare(_engine(rules, occ=0.8), _oracle(oracle_mod, rules, occ=0.8), rules, ev, batches=3)


def test_invalid_and_edge_events(oracle_mod):
    rng = np.random.default_rng(17)
    rules = T.make_rules(100, rng, count_lo=0, count_hi=30)
    rules.threshold_type[::3] = 0          # AVG_LOCAL
    rules.namespace[5::7] = -1             # namespace == null -> TOO_MANY_REQUEST
    rules.namespace[6::7] = 1
    n = 30_000
    idx = rng.integers(-3, 103, size=n).astype(np.int32)
    acq = rng.integers(-1, 4, size=n).astype(np.int32)
    ev = T.Events(idx, acq, T.timestamps(n, 9000.0, T.T0_ALIGNED + 999))
    ns = [dict(connected_count=0), dict(connected_count=3)]
    _compare(_engine(rules, namespaces=ns), _oracle(oracle_mod, rules, namespaces=ns), rules, ev, batches=2)


def test_namespace_limiter(oracle_mod):
    rng = np.random.default_rng(19)
    rules = T.make_rules(300, rng, count_lo=10, count_hi=500)
    rules.namespace[:] = rng.integers(0, 3, size=300)
    ns = [dict(connected_count=1, has_limiter=1, max_allowed_qps=2000.0),
          dict(connected_count=1, has_limiter=0),
          dict(connected_count=1, has_limiter=1, max_allowed_qps=777.5)]
    n = 80_000
    ev = T.Events(T.zipf_indices(300, 1.1, n, rng), np.ones(n, np.int32), T.timestamps(n, 20_000.0, T.T0_ALIGNED + 41))
    _compare(_engine(rules, namespaces=ns), _oracle(oracle_mod, rules, namespaces=ns), rules, ev, batches=3)


@pytest.mark.parametrize("lim1", ["1", "0"])
def test_single_namespace_limiter(oracle_mod, monkeypatch, lim1):
    """One namespace limiter (the reference's state after a namespace-set change with the default
    namespace): the fused prep + stable partition (k_lim1_prep) and the prep + radix pass, over
    invalid ids, non-positive acquires, flows of a namespace without limiter or of a null namespace,
    a clock that steps back now and then, and many look-back tiles.  (ts < 0 is a documented
    divergence, DESIGN.md section 1, so the trace has none.)"""
    monkeypatch.setenv("SENTINEL_LIM1", lim1)
    rng = np.random.default_rng(37)
    rules = T.make_rules(5000, rng, count_lo=5, count_hi=400)
    rules.namespace[:] = 0
    rules.namespace[3::11] = 1
    rules.namespace[5::97] = 7                  # no such namespace -> TOO_MANY_REQUEST
    ns = [dict(connected_count=1, has_limiter=1, max_allowed_qps=3100.0), dict(connected_count=2)]
    n = 150_000
    idx = T.zipf_indices(5000, 1.05, n, rng).astype(np.int32)
    idx[rng.random(n) < 0.01] = -2
    acq = np.ones(n, np.int32)
    acq[rng.random(n) < 0.01] = 0
    ts = T.timestamps(n, 20_000.0, T.T0_ALIGNED + 77)
    ts = ts + np.where(rng.random(n) < 0.02, rng.integers(-250, 1, size=n), 0)
    ev = T.Events(idx, acq, ts.astype(np.int64))
    _compare(_engine(rules, namespaces=ns), _oracle(oracle_mod, rules, namespaces=ns), rules, ev, batches=3)


def test_clock_backwards_sequential_path(oracle_mod):
    rng = np.random.default_rng(23)
    rules = T.make_rules(40, rng, count_lo=2, count_hi=50, sample_count=4, window_interval_ms=400)
    n = 20_000
    ts = T.timestamps(n, 4000.0, T.T0_ALIGNED)
    jitter = rng.integers(-450, 1, size=n)
    ts = ts + np.where(rng.random(n) < 0.05, jitter, 0)
    ev = T.Events(rng.integers(0, 40, size=n).astype(np.int32), np.ones(n, np.int32), ts.astype(np.int64))
    _compare(_engine(rules), _oracle(oracle_mod, rules), rules, ev, batches=2)


def test_wide_timestamp_span_fallback(oracle_mod):
    """A batch spanning 30 days: ts - T0 overflows the 24-bit delta of the sorted value, so those
    events are read back by position; verdicts must not change."""
    rng = np.random.default_rng(31)
    rules = T.make_rules(60, rng, count_lo=3, count_hi=40, sample_count=2, window_interval_ms=1000)
    n = 20_000
    ts = T.timestamps(n, 5000.0, T.T0_ALIGNED)
    ts[n // 2:] += 30 * 24 * 3600 * 1000        # +30 days
    ev = T.Events(rng.integers(0, 60, size=n).astype(np.int32), np.ones(n, np.int32), ts.astype(np.int64))
    _compare(_engine(rules), _oracle(oracle_mod, rules), rules, ev, batches=1)


def test_empty_single_and_all_invalid(oracle_mod):
    rng = np.random.default_rng(29)
    rules = T.make_rules(10, rng)
    svc, orc = _engine(rules), _oracle(oracle_mod, rules)
    st, rem, w = svc.submit_flow_batch_host(np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.int64))
    assert len(st) == 0
    ev = T.Events(np.array([3], np.int32), np.array([1], np.int32), np.array([T.T0_ALIGNED], np.int64))
    _compare(svc, orc, rules, ev)
    ev = T.Events(np.array([-1, -2, 50], np.int32), np.array([1, 1, 1], np.int32), np.full(3, T.T0_ALIGNED, np.int64))
    _compare(svc, orc, rules, ev)


def test_request_token_single_call(oracle_mod):
    """ClusterFlowCheckerTest sequence (disabled upstream) through the per-call TokenService API."""
    import json, os
    kat = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat_cluster_flow_checker.json")))
    import sentinel_amd as sa
    from sentinel_amd.token_service import ServerNamespace
    r = kat["rule"]
    svc = sa.GpuTokenService(0)
    svc.set_namespaces([ServerNamespace()])
    rules = sa.FlowRule(count=r["count"], cluster_config=sa.ClusterFlowConfig(
        flow_id=r["flow_id"], threshold_type=1, sample_count=r["sample_count"], window_interval_ms=r["window_interval_ms"]))
    svc.load_flow_rules([rules])
    names = {"OK": 0, "BLOCKED": 1, "SHOULD_WAIT": 2}
    t = kat["t0"][0]
    for step in kat["steps"]:
        t += step[0]
        res = svc.request_token(r["flow_id"], 1, step[1], ts=t)
        assert res.status == names[step[2]]
        if len(step) > 3:
            assert res.wait_in_ms == step[3]
    assert svc.request_token(None, 1, False, ts=t).status == sa.TokenResultStatus.BAD_REQUEST
    assert svc.request_token(12345, 1, False, ts=t).status == sa.TokenResultStatus.NO_RULE_EXISTS
    assert svc.request_token(r["flow_id"], 0, False, ts=t).status == sa.TokenResultStatus.BAD_REQUEST


def test_snapshot_matches_oracle_avgs(oracle_mod):
    rules, ev = T.config2(50_000, seed=31, n_flows=300)
    svc, orc = _engine(rules), _oracle(oracle_mod, rules)
    _compare(svc, orc, rules, ev, check_state=False)
    t = int(ev.ts[-1]) + 250
    snap = svc.snapshot(t)
    for f in range(0, 300, 7):
        cm = orc.dump_flow(f)     # just ensure the flow exists
        assert snap["flow_id"][f] == rules.flow_id[f]
    # recompute with the oracle's avg functions on its own metric objects via request-free reads
    # (ClusterMetricNodeGenerator reads getAvg(BLOCK), getAvg(PASS) at t)
    for f in range(0, 300, 7):
        n = int(rules.sample_count[f])
        d = svc.dump_flow(f, n).reshape(-1)[: n * 8].reshape(n, 8)
        w = int(rules.window_interval_ms[f]) // n
        E = t // w
        valid = (d[:, 0] >= 0) & (d[:, 0] // w > E - n)
        I_s = int(rules.window_interval_ms[f]) / 1000.0
        assert snap["pass_qps"][f] == float(d[valid, 1].sum()) / I_s
        assert snap["block_qps"][f] == float(d[valid, 2].sum()) / I_s


@pytest.mark.parametrize("path", ["part", "slot", "rule"])
def test_param_single_value_bitexact(oracle_mod, monkeypatch, path):
    """Exact single-value requests through the partition-local path (default), the per-slot segment
    pipeline and the per-rule walk."""
    monkeypatch.setenv("SENTINEL_PARAM_PATH", path)
    count, hot, rule_idx, vals, keys, ts = T.config4(120_000, seed=4, n_rules=200, universe=300)
    import sentinel_amd as sa
    from sentinel_amd.token_service import ServerNamespace
    prules = [sa.ParamFlowRule(count=float(count[r]), cluster_config=sa.ClusterFlowConfig(
        flow_id=r + 1, threshold_type=1, sample_count=2 if r % 2 else 5, window_interval_ms=1000),
        hot_items=hot.get(r, {})) for r in range(len(count))]
    svc = sa.GpuTokenService(0)
    svc.set_namespaces([ServerNamespace()])
    svc.load_param_rules(prules)
    orc = oracle_mod.TokenServiceOracle([], param_rules=[dict(flow_id=r + 1, count=float(count[r]), threshold_type=1,
                                                              sample_count=2 if r % 2 else 5, window_interval_ms=1000)
                                                         for r in range(len(count))],
                                        hot_items={r: list(hot[r].items()) for r in hot})
    acq = np.where(np.arange(len(ts)) % 3 == 0, 2, 1).astype(np.int32)
    for a, b in [(0, 50_000), (50_000, 120_000)]:
        st_g, rem_g = svc.submit_param_batch_host(rule_idx[a:b], acq[a:b], keys[a:b], ts[a:b])
        st_o, rem_o = orc.param_replay(rule_idx[a:b], acq[a:b], keys[a:b], ts[a:b])
        bad = np.nonzero((st_g != st_o) | (rem_g != rem_o))[0]
        assert len(bad) == 0, (len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]], rem_g[bad[:5]], rem_o[bad[:5]])
    assert not orc.param_overflowed()
    t = int(ts[-1])
    for i in range(0, 5000, 97):
        r, k = int(rule_idx[i]), int(keys[i])
        assert svc.param_sum(r, k, t) == orc.param_sum(r, t, k)


def test_full_size_properties_config3():
    """BASELINE config 3 shape at full per-GPU batch size (8M events, 1M flows): properties only."""
    import torch
    import sentinel_amd as sa
    rules, _ = T.config3(1, seed=3)
    svc = _engine(rules)
    n = 8 * 1024 * 1024
    g = torch.Generator(device="cuda").manual_seed(3)
    idx = torch.randint(0, len(rules), (n,), dtype=torch.int32, device="cuda", generator=g)
    acq = torch.ones(n, dtype=torch.int32, device="cuda")
    rate = 2.0 * float(rules.count.sum())
    ts = (T.T0_ALIGNED + torch.floor(torch.arange(n, device="cuda", dtype=torch.float64) * (1000.0 / rate))).to(torch.int64)
    from sentinel_amd.token_service import decode_verdicts, device_events
    ev = device_events(idx, acq, ts)
    v = svc.submit_flow_batch(ev)
    svc.synchronize()
    st_c, rem_c, _ = decode_verdicts(v)
    assert set(np.unique(st_c)).issubset({0, 1})
    # conservation: passes per flow == PASS counter growth; admission bound: passes <= threshold
    passes = np.bincount(idx.cpu().numpy()[st_c == 0], minlength=len(rules))
    sample = np.random.default_rng(0).choice(len(rules), 200, replace=False)
    for f in sample:
        d = svc.dump_flow(int(f), 10)[:80].reshape(10, 8)
        assert d[:, 1].sum() == passes[f]
        assert passes[f] <= rules.count[f] * 1.0 + 1e-9
    # determinism: a fresh engine on the same input gives identical verdicts
    svc2 = _engine(rules)
    v2 = svc2.submit_flow_batch(ev)
    svc2.synchronize()
    assert torch.equal(v, v2)


@pytest.mark.parametrize("world", [1, 2, 8])
def test_bench_rank_shapes_bitexact(oracle_mod, world):
    """Bit-exact at the exact per-rank shapes of the bench (`bench.py --gpus N`): rank 0's shard
    (splitmix64(flowId) mod N) of the 1M-flowId config-3 universe, 8M-event batches, two batches
    so the second rolls windows written by the first; oracle = the flow-sharded replay."""
    import torch
    from sentinel_amd.token_service import decode_verdicts, device_events
    rng = np.random.default_rng(3)
    rules = T.make_rules(1_000_000, rng, sample_count=10, window_interval_ms=1000)
    if world > 1:
        rules = rules.subset(np.nonzero(T.shard_of(rules.flow_id, world) == 0)[0])
    F = len(rules)
    svc = _engine(rules)
    orc = oracle_mod.TokenServiceOracle.from_arrays(rules.flow_id, rules.count, rules.threshold_type,
                                                    rules.sample_count, rules.window_interval_ms,
                                                    rules.namespace, rules.checker)
    n = 8 * 1024 * 1024
    ms_per_event = 1000.0 / (2.0 * float(rules.count.sum()))
    erng = np.random.default_rng(100 + world)
    for b in range(2):
        idx = erng.integers(0, F, n, dtype=np.int32)
        ts = (T.T0_ALIGNED + np.floor(np.arange(b * n, (b + 1) * n, dtype=np.float64) * ms_per_event)).astype(np.int64)
        acq = np.ones(n, np.int32)
        v = svc.submit_flow_batch(device_events(torch.from_numpy(idx).cuda(), torch.from_numpy(acq).cuda(),
                                                torch.from_numpy(ts).cuda()))
        svc.synchronize()
        st_g, rem_g, _ = decode_verdicts(v)
        st_o, rem_o, _, _ = orc.replay_mt(idx, acq, ts, 16)
        bad = np.nonzero((st_g != st_o) | (rem_g != rem_o))[0]
        assert len(bad) == 0, (world, b, len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]])
    for f in np.random.default_rng(1).choice(F, 300, replace=False):
        assert np.array_equal(svc.dump_flow(int(f), 10), orc.dump_flow(int(f))), f


@pytest.mark.parametrize("F", [1_000_000, 400_000])
def test_window_boundary_inside_batch(oracle_mod, F):
    """Batches whose time span holds a window boundary (T0 + 1 s: a boundary of every rule's window): a flow's
    run is two homogeneous segments, epoch E then E2 (partition.hpp, part_run_single's two-segment closed
    form -- 1M flows: one thread per flow; 400k: the cooperative verdict sweep).  Windows n = 10 / 2 / 1 over
    1 s (with n = 1 both segments share one slot), acquire counts that change at the boundary, small
    thresholds (blocked events in both segments), batches before / across / after the boundary so the
    rolled slots carry state, and one batch whose halves lie 2 s apart (the second segment's window holds
    nothing of the first); bit-exact statuses, remaining and window counters."""
    import torch
    from sentinel_amd.token_service import decode_verdicts, device_events
    rng = np.random.default_rng(29)
    rules = T.make_rules(F, rng, count_lo=1, count_hi=30, sample_count=10, window_interval_ms=1000)
    rules.sample_count[1::3] = 2
    rules.sample_count[2::3] = 1
    svc = _engine(rules)
    orc = oracle_mod.TokenServiceOracle.from_arrays(rules.flow_id, rules.count, rules.threshold_type,
                                                    rules.sample_count, rules.window_interval_ms,
                                                    rules.namespace, rules.checker)
    n = 4 * 1024 * 1024
    erng = np.random.default_rng(30)
    # the last batch jumps 2 s between its halves: its second segments start past every slot of the first
    # (E2 - E >= n for every window)
    for b, (t_lo, t_hi) in enumerate([(985, 993), (996, 1004), (1004, 1012), (1990, 3998)]):
        idx = erng.integers(0, F, n, dtype=np.int32)
        ts = (T.T0_ALIGNED + t_lo + np.floor(np.arange(n, dtype=np.float64) * ((t_hi - t_lo) / n))).astype(np.int64)
        if b == 3:
            ts = np.where(np.arange(n) < n // 2, T.T0_ALIGNED + 1990 + np.arange(n) * 4 // n,
                          T.T0_ALIGNED + 3994 + np.arange(n) * 4 // n).astype(np.int64)
        acq = (1 + (idx.astype(np.int64) + (ts >= T.T0_ALIGNED + 1000) + (ts >= T.T0_ALIGNED + 3000)) % 3).astype(np.int32)
        v = svc.submit_flow_batch(device_events(torch.from_numpy(idx).cuda(), torch.from_numpy(acq).cuda(),
                                                torch.from_numpy(ts).cuda()))
        svc.synchronize()
        st_g, rem_g, _ = decode_verdicts(v)
        st_o, rem_o, _, _ = orc.replay_mt(idx, acq, ts, 16)
        bad = np.nonzero((st_g != st_o) | (rem_g != rem_o))[0]
        assert len(bad) == 0, (F, b, len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]])
        if b == 1:
            assert 0.05 < float((st_o == 1).mean()) < 0.95, float((st_o == 1).mean())   # both outcomes
    for f in np.random.default_rng(2).choice(F, 300, replace=False):
        assert np.array_equal(svc.dump_flow(int(f), int(rules.sample_count[f])), orc.dump_flow(int(f))), f


def test_batcher_concurrent_threads():
    """Many threads calling the per-call API concurrently: batched on the GPU, and the result set
    equals a sequential replay in some arrival order (homogeneous acquire => order-free counts)."""
    import threading
    import sentinel_amd as sa
    from sentinel_amd.token_service import TokenBatcher
    svc = sa.GpuTokenService(0)
    svc.load_flow_rules([sa.FlowRule(count=50, cluster_config=sa.ClusterFlowConfig(
        flow_id=777, threshold_type=1, sample_count=2, window_interval_ms=1000))])
    b = TokenBatcher(svc, max_batch=256, max_wait_us=200)
    results = []
    lock = threading.Lock()
    t = T.T0_ALIGNED + 10

    def worker():
        for _ in range(25):
            r = b.request_token(777, 1, False, ts=t)
            with lock:
                results.append(r)

    th = [threading.Thread(target=worker) for _ in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    ok = sorted(r.remaining for r in results if r.status == 0)
    assert len(results) == 400
    assert ok == list(range(50))[::-1][::-1] and len(ok) == 50
    assert sum(1 for r in results if r.status == 1) == 350
    nb, nr = b.stats()
    assert nr == 400 and 1 <= nb <= 400
    assert b.request_token(None, 1, False, ts=t).status == sa.TokenResultStatus.BAD_REQUEST
    b.close()


def test_hot_flow_long_runs(oracle_mod):
    """One flow takes most of the batch (runs far longer than one lane should walk): the partition
    path hands it to a whole workgroup; heterogeneous acquires, prioritized events and a clock
    that steps back put sequential segments inside the long run."""
    rng = np.random.default_rng(41)
    rules = T.make_rules(100, rng, count_lo=50, count_hi=4000, sample_count=4, window_interval_ms=400)
    n = 90_000
    idx = rng.integers(0, 100, size=n).astype(np.int32)
    idx[rng.random(n) < 0.6] = 7
    acq = np.ones(n, np.int32)
    acq[rng.random(n) < 0.03] = 2
    ts = T.timestamps(n, 30_000.0, T.T0_ALIGNED + 11)
    ts = ts + np.where(rng.random(n) < 0.002, -rng.integers(0, 300, size=n), 0)
    flags = (rng.random(n) < 0.01).astype(np.uint8)
    ev = T.Events(idx, acq, ts.astype(np.int64), flags)
    _compare(_engine(rules, occ=0.9), _oracle(oracle_mod, rules, occ=0.9), rules, ev, batches=3)


def test_partition_ballot_ranking_split_halves(oracle_mod):
    """4096 flows (4 per range, 2 per half) with ~50 events per flow per batch: every half of the
    partition path takes the stable ballot ranking (runs longer than the per-run insertion sort)."""
    rng = np.random.default_rng(43)
    rules = T.make_rules(4096, rng, count_lo=5, count_hi=200, sample_count=2, window_interval_ms=1000)
    n = 400_000
    idx = rng.integers(0, 4096, size=n).astype(np.int32)
    acq = np.ones(n, np.int32)
    acq[rng.random(n) < 0.02] = 3
    ts = T.timestamps(n, 150_000.0, T.T0_ALIGNED + 5)
    ev = T.Events(idx, acq, ts.astype(np.int64), None)
    _compare(_engine(rules), _oracle(oracle_mod, rules), rules, ev, batches=2)


@pytest.mark.parametrize("hot_frac", [0.024, 0.045])
def test_partition_oversized_half(oracle_mod, hot_frac):
    """65536 flows (64 per range): one half of one range gets ~7000 events (0.024: more than fit in
    LDS while its range stays under the key capacity, so that half is sorted through HBM and the other
    half stays in LDS, both writing the same range) or ~13500 (0.045: the range exceeds the key
    capacity, both halves through HBM).  Oversized halves are listed by k_part_half and decided by
    k_part_big."""
    rng = np.random.default_rng(47)
    F = 65536
    rules = T.make_rules(F, rng, count_lo=5, count_hi=500, sample_count=10, window_interval_ms=1000)
    n = 300_000
    idx = rng.integers(0, F, size=n).astype(np.int32)
    hot = rng.random(n) < hot_frac                 # into flows 352..383 (range 5, half 1)
    idx[hot] = 352 + rng.integers(0, 32, size=int(hot.sum()))
    ts = T.timestamps(n, 400_000.0, T.T0_ALIGNED + 3)
    ev = T.Events(idx, np.ones(n, np.int32), ts.astype(np.int64), None)
    _compare(_engine(rules), _oracle(oracle_mod, rules), rules, ev, batches=1)


def test_stream_host_pipelined_bitexact(oracle_mod):
    """sentinel_submit_flow_stream_host: the trace in uneven consecutive batches pipelined over the
    copy streams (odd tail batch, both staging slots reused several times, prioritized flags) equals
    the oracle's sequential replay of the whole trace, and every batch reports a latency."""
    rules, ev = T.config2(250_000, seed=21, n_flows=3000)
    flags = (np.random.default_rng(5).random(len(ev.ts)) < 0.01).astype(np.uint8)
    svc = _engine(rules)
    st_g, rem_g, w_g, ms = svc.submit_flow_stream_host(ev.flow_idx, ev.acquire, ev.ts, flags, batch=37_000)
    st_o, rem_o, w_o = _oracle(oracle_mod, rules).replay(ev.flow_idx, ev.acquire, ev.ts, flags)
    assert np.array_equal(st_g, st_o) and np.array_equal(rem_g, rem_o) and np.array_equal(w_g, w_o)
    assert len(ms) == 7 and (ms > 0).all()


def _norm_dump(d, n):
    """Window dump with absent slots and present all-zero slots made equal (a snapshot's roll of a
    stale slot leaves it present and empty; the next event's own roll would produce the same)."""
    d = np.array(d, dtype=np.int64).reshape(-1)
    w = d[: n * 8].reshape(n, 8).copy()
    w[(w[:, 1:] == 0).all(axis=1), 0] = -1
    return w, d[n * 8:]


def test_path_switches_snapshots_and_epoch_gaps(oracle_mod):
    """One engine, one flow table written by all three pipelines in turn (sentinel_set_flow_path) and by
    snapshots (which roll windows) between batches; batches advance by 0, 1, 2..n-1 and >= n epochs,
    some with heterogeneous acquire counts (the general walk).  Every verdict must equal the
    oracle's, and the final windows too (absent == present-and-empty)."""
    rng = np.random.default_rng(41)
    F = 3000
    rules = T.make_rules(F, rng, count_lo=5, count_hi=60)
    ns = np.array([2, 4, 10])[np.arange(F) % 3].astype(np.int32)
    rules.sample_count[:] = ns
    rules.window_interval_ms[:] = ns * 100                   # w = 100 ms for every flow
    svc, orc = _engine(rules), _oracle(oracle_mod, rules)
    t = T.T0_ALIGNED + 37
    # (epochs advanced before the batch, pipeline, snapshot before the batch)
    plan = [(0, "partition", False), (0, "partition", False), (1, "small", False), (1, "sorted", False),
            (0, "partition", False), (1, "partition", True), (0, "partition", False), (2, "small", False),
            (3, "partition", False), (12, "partition", False), (1, "partition", False), (0, "sorted", False),
            (1, "small", False), (1, "partition", True), (0, "partition", False), (25, "small", False)]
    for b, (adv, path, snap) in enumerate(plan):
        t += adv * 100
        if snap:
            svc.snapshot(t)
        svc.set_flow_path(path)
        m = 20_000
        idx = rng.integers(0, F, size=m).astype(np.int32)
        ts = np.sort(t + rng.integers(0, 40, size=m)).astype(np.int64)   # mostly one epoch per flow
        acq = np.ones(m, np.int32)
        if b in (4, 12):
            acq = rng.integers(1, 3, size=m).astype(np.int32)   # heterogeneous runs: the general walk
        st_g, rem_g, w_g = svc.submit_flow_batch_host(idx, acq, ts)
        st_o, rem_o, w_o = orc.replay(idx, acq, ts)
        bad = np.nonzero((st_g != st_o) | (rem_g != rem_o) | (w_g != w_o))[0]
        assert len(bad) == 0, (b, path, len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]], rem_g[bad[:5]], rem_o[bad[:5]])
        t = int(ts[-1])
    for f in range(0, F, 11):
        n = int(ns[f])
        g, go = _norm_dump(svc.dump_flow(f, n), n)
        o, oo = _norm_dump(orc.dump_flow(f), n)
        assert np.array_equal(g, o) and np.array_equal(go, oo), (f, g, o)


@pytest.mark.parametrize("batch", [1 << 20, 1 << 22])
def test_config2_full_size_bitexact(oracle_mod, batch):
    """BASELINE config 2 at its stated size: 10k flowIds, QPS grade, 1 s / 2-bucket windows, Zipf(1.1)
    requests at 2x the summed thresholds, acquire 1, batches of 1M and 4M events (two batches, so the
    second rolls windows the first wrote); bit-exact verdicts and windows on both flow pipelines."""
    rules, ev = T.config2(2 * batch, seed=2, n_flows=10_000)
    _compare(_engine(rules), _oracle(oracle_mod, rules), rules, ev, batches=2)
