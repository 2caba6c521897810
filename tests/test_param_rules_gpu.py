"""GPU parity of the per-rule hot-parameter paths (param_rules.hpp) against the CPU oracle:
multi-value cluster requests (bit-exact), count-min mode (one-sided: audited on exact counters),
and the local ParamFlowChecker token bucket (bit-exact, including the reference's KAT sequences)."""
import json
import os

import numpy as np
import pytest

from sentinel_amd import trace as T

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _cluster_pair(oracle_mod, count, hot, sample_count=lambda r: 2 if r % 2 else 5, namespaces=None,
                  threshold_type=lambda r: 1):
    import sentinel_amd as sa
    from sentinel_amd.token_service import ServerNamespace
    R = len(count)
    prules = [sa.ParamFlowRule(count=float(count[r]), cluster_config=sa.ClusterFlowConfig(
        flow_id=r + 1, threshold_type=threshold_type(r), sample_count=sample_count(r), window_interval_ms=1000),
        hot_items=hot.get(r, {}), namespace=(r % len(namespaces)) if namespaces else 0) for r in range(R)]
    svc = sa.GpuTokenService(0)
    ns = namespaces or [dict()]
    svc.set_namespaces([ServerNamespace(**n) for n in ns])
    svc.load_param_rules(prules)
    orc = oracle_mod.TokenServiceOracle(
        [], namespaces=[dict(connected_count=n.get("connected_count", 0), has_limiter=n.get("has_limiter", 0),
                             max_allowed_qps=n.get("max_allowed_qps", 30000.0)) for n in ns],
        param_rules=[dict(flow_id=r + 1, count=float(count[r]), threshold_type=threshold_type(r), sample_count=sample_count(r),
                          window_interval_ms=1000, namespace_idx=(r % len(namespaces)) if namespaces else 0)
                     for r in range(R)],
        hot_items={r: list(hot[r].items()) for r in hot})
    return svc, orc


def _slice_lists(b, c, k, lo, hi):
    bb = b[lo:hi]
    start = int(bb[0]) if len(bb) else 0
    end = int(bb[-1] + c[hi - 1]) if len(bb) else 0
    return (bb - start).astype(np.int32), c[lo:hi], k[start:end]


def test_multi_value_exact_bitexact(oracle_mod):
    count, hot, rule_idx, vals, keys, ts = T.config4(80_000, seed=44, n_rules=150, universe=250)
    rng = np.random.default_rng(44)
    b, c, k = T.param_value_lists(rule_idx, rng, universe=250)
    acq = np.where(np.arange(len(ts)) % 5 == 0, 2, 1).astype(np.int32)
    svc, orc = _cluster_pair(oracle_mod, count, hot)
    for lo, hi in [(0, 30_000), (30_000, 80_000)]:
        bb, cc, kk = _slice_lists(b, c, k, lo, hi)
        sg, rg = svc.submit_param_multi_batch_host(rule_idx[lo:hi], acq[lo:hi], ts[lo:hi], bb, cc, kk)
        so, ro = orc.param_multi_replay(rule_idx[lo:hi], acq[lo:hi], ts[lo:hi], bb, cc, kk)
        bad = np.nonzero((sg != so) | (rg != ro))[0]
        assert len(bad) == 0, (len(bad), bad[:5], sg[bad[:5]], so[bad[:5]], rg[bad[:5]], ro[bad[:5]])
    assert set(np.unique(so)) <= {0, 1} and (so == 1).any() and (so == 0).any()
    t = int(ts[-1])
    for j in range(0, len(k), 331):
        r = int(k[j] >> np.uint64(20))
        assert svc.param_sum(r, int(k[j]), t) == orc.param_sum(r, t, int(k[j]))


def test_single_and_multi_batches_share_exact_counters(oracle_mod):
    """Single-value fast path (per key) and the per-rule path interleave on one set of counters."""
    count, hot, rule_idx, vals, keys, ts = T.config4(60_000, seed=45, n_rules=80, universe=120)
    rng = np.random.default_rng(45)
    b, c, k = T.param_value_lists(rule_idx, rng, universe=120, max_values=3)
    acq = np.ones(len(ts), np.int32)
    svc, orc = _cluster_pair(oracle_mod, count, hot)
    cuts = [0, 15_000, 30_000, 45_000, 60_000]
    for i in range(4):
        lo, hi = cuts[i], cuts[i + 1]
        if i % 2 == 0:
            sg, rg = svc.submit_param_batch_host(rule_idx[lo:hi], acq[lo:hi], keys[lo:hi], ts[lo:hi])
            so, ro = orc.param_replay(rule_idx[lo:hi], acq[lo:hi], keys[lo:hi], ts[lo:hi])
        else:
            bb, cc, kk = _slice_lists(b, c, k, lo, hi)
            sg, rg = svc.submit_param_multi_batch_host(rule_idx[lo:hi], acq[lo:hi], ts[lo:hi], bb, cc, kk)
            so, ro = orc.param_multi_replay(rule_idx[lo:hi], acq[lo:hi], ts[lo:hi], bb, cc, kk)
        assert np.array_equal(sg, so) and np.array_equal(rg, ro), i


def test_multi_value_edge_cases_and_limiter(oracle_mod):
    rng = np.random.default_rng(46)
    count = rng.integers(3, 30, size=60).astype(np.float64)
    ns = [dict(connected_count=1, has_limiter=1, max_allowed_qps=900.0), dict(connected_count=2)]
    svc, orc = _cluster_pair(oracle_mod, count, {}, namespaces=ns)
    n = 20_000
    ridx = rng.integers(-3, 63, size=n).astype(np.int32)
    ridx[ridx == -3] = -2                                  # BAD id
    acq = rng.integers(-1, 3, size=n).astype(np.int32)
    b, c, k = T.param_value_lists(np.clip(ridx, 0, 59), rng, universe=40, max_values=4)
    c = c.copy()
    c[::97] = 0                                            # empty params -> BAD_REQUEST
    ts = T.timestamps(n, 4000.0, T.T0_ALIGNED + 77)
    sg, rg = svc.submit_param_multi_batch_host(ridx, acq, ts, b, c, k)
    so, ro = orc.param_multi_replay(ridx, acq, ts, b, c, k)
    bad = np.nonzero((sg != so) | (rg != ro))[0]
    assert len(bad) == 0, (len(bad), bad[:5], sg[bad[:5]], so[bad[:5]])
    assert {-4, -2, 0, 1, 3} <= set(np.unique(so).tolist())


def test_count_min_is_one_sided(oracle_mod):
    """Narrow sketch (width 64): collisions happen; every pass must still be admissible on exact
    counters replaying the sketch's own decisions.  Wide sketch: false blocks vanish."""
    import sentinel_amd as sa
    count, hot, rule_idx, vals, keys, ts = T.config4(60_000, seed=47, n_rules=60, universe=400, offered_ratio=40.0)
    rng = np.random.default_rng(47)
    b, c, k = T.param_value_lists(rule_idx, rng, universe=400, max_values=3)
    acq = np.ones(len(ts), np.int32)
    rates = {}
    for width in (64, 8192):
        svc, orc = _cluster_pair(oracle_mod, count, hot)
        svc.set_param_mode(sa._lib.PARAM_COUNT_MIN, depth=4, width=width)
        sg, _ = svc.submit_param_multi_batch_host(rule_idx, acq, ts, b, c, k)
        viol, fb, dec = orc.param_cm_audit(rule_idx, acq, ts, b, c, k, sg)
        assert viol == 0, (width, viol)
        assert dec == len(ts)
        rates[width] = fb / dec
        # estimates never undercount the value's own (sketch-admitted) window count
        t = int(ts[-1])
        for j in range(0, len(k), 997):
            r = int(k[j] >> np.uint64(20))
            assert svc.param_sum(r, int(k[j]), t) >= orc.param_sum(r, t, int(k[j]))
    assert rates[64] > rates[8192]
    assert rates[8192] < 1e-3, rates
    # single-value batches go through the sketch too in count-min mode
    svc, orc = _cluster_pair(oracle_mod, count, hot)
    svc.set_param_mode(sa._lib.PARAM_COUNT_MIN, depth=2, width=32)
    sg, _ = svc.submit_param_batch_host(rule_idx[:20_000], acq[:20_000], keys[:20_000], ts[:20_000])
    n1 = np.ones(20_000, np.int32)
    viol, fb, dec = orc.param_cm_audit(rule_idx[:20_000], acq[:20_000], ts[:20_000], np.arange(20_000), n1,
                                       keys[:20_000], sg)
    assert viol == 0 and dec == 20_000


@pytest.mark.gpu
@pytest.mark.parametrize("levels", ["keys", "keys-c64", "keys-global", "launch", "coop"])
def test_shared_count_min_is_one_sided(oracle_mod, monkeypatch, levels):
    """One sketch for every rule (BASELINE config 4's layout), narrow enough that rules collide, on
    batches spanning ~75 epochs.  "keys" / "keys-global": the key walk, one lane per (rule, value) key,
    every read of the batch before any add -- in one workgroup per sketch block staged in LDS
    (k_pp_cm_block, the default; 32-bit LDS cells, or 64-bit with "keys-c64"), or with "keys-global" in two
    launches on HBM cells (k_pp_cm_read, then k_pp_cm_walk: decisions and memory-side atomic adds); "launch" / "coop": one lane per rule moving through the
    epochs band by band (k_prule_cm_level / k_prule_cm_sync).  Either way no reset of a shared cell slot
    drops a count a check still needs -- zero violations of one-sidedness, and the false-block rate
    shrinks with the width."""
    import sentinel_amd as sa
    # the key walk (the default), one launch per band of rule lanes, or the grid barrier
    monkeypatch.setenv("SENTINEL_CM_LEVELS", "keys" if levels.startswith("keys") else levels)
    monkeypatch.setenv("SENTINEL_CM_BLOCK", "0" if levels == "keys-global" else "1")
    # the block walk's LDS cells: 32-bit (tags mod 256 around the batch's newest epoch) or 64-bit
    monkeypatch.setenv("SENTINEL_CM_C32", "0" if levels == "keys-c64" else "1")
    count, hot, rule_idx, vals, keys, ts = T.config4(200_000, seed=53, n_rules=5000, universe=200)
    acq = np.ones(len(ts), np.int32)
    rates = {}
    for width in (1 << 10, 1 << 16):
        svc, orc = _cluster_pair(oracle_mod, count, hot, sample_count=lambda r: 10)   # one window for all
        svc.set_param_mode(sa._lib.PARAM_COUNT_MIN_SHARED, depth=4, width=width)
        st = np.concatenate([svc.submit_param_batch_host(rule_idx[i:i + 50_000], acq[i:i + 50_000], keys[i:i + 50_000],
                                                         ts[i:i + 50_000])[0] for i in range(0, len(ts), 50_000)])
        n1 = np.ones(len(ts), np.int32)
        viol, fb, dec = orc.param_cm_audit(rule_idx, acq, ts, np.arange(len(ts)), n1, keys, st)
        assert viol == 0 and dec == len(ts), (width, viol)
        rates[width] = fb / dec
        cs = svc.param_cm_stats()
        if levels.startswith("keys"):
            assert cs["key_walk"] >= 1 and cs["block"] == (0 if levels == "keys-global" else cs["key_walk"]), cs
    assert rates[1 << 10] > rates[1 << 16]


@pytest.mark.gpu
@pytest.mark.parametrize("block", ["0", "1", "1-c64", "1-ordered"])
def test_shared_count_min_full_size_audit(oracle_mod, monkeypatch, block):
    """BASELINE config 4's count-min mode at its own size: 100k hot-parameter rules, Zipf values over
    1000 per rule, 2M requests in 4 batches, the shared sketch at d = 4, w = 2^20 (bench config 4cm):
    every sketch verdict replayed on exact counters with the same admitted history -- zero
    one-sidedness violations -- and a false-block rate far below the e/w bound.  Every key walk: the
    block-owned walk (the default) with 32-bit or 64-bit LDS cells, and the two-phase HBM walk."""
    import sentinel_amd as sa
    monkeypatch.setenv("SENTINEL_CM_BLOCK", block[0])
    monkeypatch.setenv("SENTINEL_CM_C32", "0" if block.endswith("c64") else "1")
    if block.endswith("ordered"):                       # decide-order output, put back through its seq
        from conftest import use_ordered_param_host
        use_ordered_param_host(monkeypatch)
    count, hot, rule_idx, vals, keys, ts = T.config4(2_000_000, seed=61, n_rules=100_000, universe=1000)
    acq = np.ones(len(ts), np.int32)
    svc, orc = _cluster_pair(oracle_mod, count, hot, sample_count=lambda r: 10)
    svc.set_param_mode(sa._lib.PARAM_COUNT_MIN_SHARED, depth=4, width=1 << 20)
    st = np.concatenate([svc.submit_param_batch_host(rule_idx[i:i + 500_000], acq[i:i + 500_000], keys[i:i + 500_000],
                                                     ts[i:i + 500_000])[0] for i in range(0, len(ts), 500_000)])
    n1 = np.ones(len(ts), np.int32)
    viol, fb, dec = orc.param_cm_audit(rule_idx, acq, ts, np.arange(len(ts)), n1, keys, st)
    assert viol == 0 and dec == len(ts), viol
    assert fb / dec < 1e-4, fb / dec
    assert svc.param_cm_stats()["block"] == (4 if block[0] == "1" else 0), svc.param_cm_stats()


@pytest.mark.gpu
def test_shared_count_min_block_epoch_edges(oracle_mod, monkeypatch):
    """The block walk's 32-bit LDS cells hold epochs mod 256 around the batch's newest one, and are used
    only for batches spanning < 200 epochs.  Batches that stress that: one over ~80 epochs (32-bit cells),
    one 400 epochs after it (every slot older than 255 epochs loads empty), one spanning ~300 epochs (the
    64-bit cells take it), one right after it (32-bit again, reading what the 64-bit batch wrote), and one
    whose first requests sit exactly n epochs after the previous batch's end -- every verdict audited on
    exact counters replaying the sketch's own decisions: zero one-sidedness violations."""
    import sentinel_amd as sa
    monkeypatch.setenv("SENTINEL_CM_BLOCK", "1")
    monkeypatch.setenv("SENTINEL_CM_C32", "1")
    count, hot, rule_idx, vals, keys, ts0 = T.config4(250_000, seed=71, n_rules=3000, universe=300)
    acq = np.ones(len(ts0), np.int32)
    svc, orc = _cluster_pair(oracle_mod, count, hot, sample_count=lambda r: 10)   # w = 100 ms
    svc.set_param_mode(sa._lib.PARAM_COUNT_MIN_SHARED, depth=4, width=1 << 14)
    t = T.T0_ALIGNED + 7
    spans = [8_000, 3_000, 30_000, 5_000, 6_000]          # ms: 80, 30, 300, 50, 60 epochs
    gaps = [0, 40_000, 0, 0, 1_000]                       # ms before each batch
    ts = np.empty(len(ts0), np.int64)
    st = []
    per = len(ts0) // len(spans)
    for b, (span, gap) in enumerate(zip(spans, gaps)):
        s = slice(b * per, (b + 1) * per)
        t += gap
        ts[s] = t + np.floor(np.arange(per, dtype=np.float64) * (span / per)).astype(np.int64)
        t = int(ts[s][-1]) + 1
        st.append(svc.submit_param_batch_host(rule_idx[s], acq[s], keys[s], ts[s])[0])
    m = per * len(spans)
    st = np.concatenate(st)
    viol, fb, dec = orc.param_cm_audit(rule_idx[:m], acq[:m], ts[:m], np.arange(m), np.ones(m, np.int32), keys[:m], st)
    assert viol == 0 and dec == m, (viol, dec)
    assert (st == 1).any() and (st == 0).any()
    assert svc.param_cm_stats()["block"] == len(spans), svc.param_cm_stats()


# idle gaps (epochs) between a key's admission and its re-admission, all multiples of the ring (2n = 20):
# 140 / 160 / 240 lie in (128, 256) -- the 32-bit LDS cells' tag mod 256 of the old epoch reads as
# "newer" under a half-range test -- and 2^23 + 12 in (2^23, 2^24) does the same to the 24-bit HBM tags;
# 100 and 300 are controls
RETOUCH_GAPS = (100, 140, 160, 240, 300, (1 << 23) + 12)


@pytest.mark.gpu
@pytest.mark.parametrize("walk", ["block32", "block64", "global", "launch", "coop"])
def test_shared_count_min_retouch_after_idle(oracle_mod, monkeypatch, walk):
    """a key K admitted up to its threshold at epoch E0, idle for g epochs (g a
    multiple of the 2n-slot ring, so its ring slot still holds E0), re-admitted at E0 + g at the end of a
    batch, then probed one epoch later.  The re-admission's add must restart the slot at E0 + g; if it
    kept E0's tag (a lost add), the probe's window misses the re-admitted count and passes what the exact
    checker blocks.  A sketch wide for its ~1200 keys (w = 2^16: 1024 blocks of 64 columns, one key per
    block on average -- narrow enough that small batches still take the block walk), so no collision can
    hide a lost add;
    filler batches of other keys (each < 100 epochs) carry the clock across the short gaps.  Every walk
    of the shared sketch: the block walk with 32-bit or 64-bit LDS cells, the two-phase HBM walk and both
    per-rule lane schedules.  Every verdict audited on exact counters: zero violations, and the probe
    blocks all of K's requests."""
    import sentinel_amd as sa
    monkeypatch.setenv("SENTINEL_CM_LEVELS", walk if walk in ("launch", "coop") else "keys")
    monkeypatch.setenv("SENTINEL_CM_BLOCK", "0" if walk == "global" else "1")
    monkeypatch.setenv("SENTINEL_CM_C32", "0" if walk == "block64" else "1")
    R, w = 40, 100                                         # rule 0 = K's rule (count 5); 1 s / 10 buckets
    count = np.full(R, 1e6)
    count[0] = 5.0
    kkey = np.uint64(7)                                    # rule 0, value 7
    rng = np.random.default_rng(91)
    failures = []
    for g in RETOUCH_GAPS:
        svc, orc = _cluster_pair(oracle_mod, count, {}, sample_count=lambda r: 10)
        svc.set_param_mode(sa._lib.PARAM_COUNT_MIN_SHARED, depth=4, width=1 << 16)
        t0 = T.T0_ALIGNED + 7
        E0 = t0 // w
        batches = []

        def batch(ep_lo, ep_hi, k_epoch=None, n_fill=120):
            fr = rng.integers(1, R, size=n_fill).astype(np.int32)
            fk = (fr.astype(np.uint64) << np.uint64(20)) | rng.integers(0, 30, size=n_fill).astype(np.uint64)
            ft = np.sort(rng.integers(ep_lo * w, ep_hi * w + w, size=n_fill)).astype(np.int64)
            r, k, t = [fr], [fk], [ft]
            if k_epoch is not None:                        # K's 10 requests after the filler, in epoch k_epoch
                t[0] = np.minimum(ft, k_epoch * w)
                r.append(np.zeros(10, np.int32))
                k.append(np.full(10, kkey, np.uint64))
                t.append(k_epoch * w + 3 + np.arange(10, dtype=np.int64))
            batches.append((np.concatenate(r), np.concatenate(k), np.concatenate(t)))

        batch(E0, E0, k_epoch=E0)                          # K admitted up to its threshold at E0
        if g < 1000:                                       # filler batches up to E0 + g - 1
            e = E0 + 1
            while e < E0 + g - 1:
                hi = min(e + 90, E0 + g - 1)
                batch(e, hi)
                e = hi + 1
        batch(E0 + g, E0 + g, k_epoch=E0 + g)              # re-admission at the batch's newest epoch
        batch(E0 + g + 1, E0 + g + 1, k_epoch=E0 + g + 1)  # probe: the window (E0+g-9, E0+g+1] holds 5
        st = []
        for r, k, t in batches:
            st.append(svc.submit_param_batch_host(r, np.ones(len(r), np.int32), k, t)[0])
        ridx = np.concatenate([b[0] for b in batches])
        keys = np.concatenate([b[1] for b in batches])
        ts = np.concatenate([b[2] for b in batches])
        st = np.concatenate(st)
        m = len(ts)
        viol, fb, dec = orc.param_cm_audit(ridx, np.ones(m, np.int32), ts, np.arange(m), np.ones(m, np.int32), keys, st)
        isk = keys == kkey
        kst = st[isk].reshape(-1, 10)                      # K's verdicts: admission, re-admission, probe
        passes = (kst == 0).sum(axis=1).tolist()
        if viol or dec != m or passes != [5, 5, 0]:
            failures.append(dict(gap=g, violations=viol, k_passes=passes))
        if walk in ("block32", "block64"):
            assert svc.param_cm_stats()["block"] == len(batches), svc.param_cm_stats()
    assert not failures, failures


@pytest.mark.gpu
def test_avg_local_params_follow_connected_count(oracle_mod):
    """ClusterParamFlowChecker.calcGlobalThreshold reads ConnectionManager.getConnectedCount on every
    request (CPFC:101-111): AVG_LOCAL param rules (hot items included) must see a connected count that
    changes between batches, as clients PING in and leave."""
    import sentinel_amd as sa
    count, hot, rule_idx, vals, keys, ts = T.config4(40_000, seed=59, n_rules=40, universe=60)
    # rules of namespace 0 and 1 alternate; every third rule is GLOBAL, the others AVG_LOCAL
    svc, orc = _cluster_pair(oracle_mod, count, hot, namespaces=[dict(connected_count=1), dict(connected_count=3)],
                             threshold_type=lambda r: 1 if r % 3 == 0 else 0)
    acq = np.ones(len(ts), np.int32)
    for step, (c0, c1) in enumerate([(1, 3), (4, 0), (2, 5), (0, 1)]):
        svc.set_connected_count(0, c0)
        svc.set_connected_count(1, c1)
        orc.set_connected_count(0, c0)
        orc.set_connected_count(1, c1)
        a, b = step * 10_000, (step + 1) * 10_000
        st_g, rem_g = svc.submit_param_batch_host(rule_idx[a:b], acq[a:b], keys[a:b], ts[a:b])
        st_o, rem_o = orc.param_replay(rule_idx[a:b], acq[a:b], keys[a:b], ts[a:b])
        bad = np.nonzero((st_g != st_o) | (rem_g != rem_o))[0]
        assert len(bad) == 0, (step, len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]])
        assert (st_o == 1).any() and (st_o == 0).any(), step


def _local_pair(oracle_mod, rules):
    import sentinel_amd as sa
    svc = sa.GpuTokenService(0)
    svc.load_local_param_rules([sa.LocalParamRule(count=r[0], burst_count=r[1], duration_in_sec=r[2],
                                                  hot_items=r[3]) for r in rules])
    return svc, oracle_mod.LocalParamOracle(rules)


def test_local_param_kat_sequences(oracle_mod):
    kat = json.load(open(os.path.join(GOLDEN, "kat_param_default_checker.json")))
    for case in kat["cases"]:
        for t0 in kat["t0"]:
            svc, _ = _local_pair(oracle_mod, [(case["token_count"], case["burst"], case["duration"], {})])
            t, ts = t0, []
            for dt, _x in case["steps"]:
                t += dt
                ts.append(t)
            n = len(ts)
            # one batch per step: the sequence crosses batches like the reference's calls cross time
            got = [int(svc.submit_local_param_batch_host([0], [1], [ts[i]], [0], [1], [7])[0]) for i in range(n)]
            assert got == [0 if x else 1 for _, x in case["steps"]], case["name"]
            # and the whole sequence as ONE batch gives the same answers (sequential per key)
            svc2, _ = _local_pair(oracle_mod, [(case["token_count"], case["burst"], case["duration"], {})])
            st = svc2.submit_local_param_batch_host(np.zeros(n), np.ones(n), ts, np.arange(n), np.ones(n), np.full(n, 7))
            assert list(st) == got, case["name"]


def test_local_param_bitexact(oracle_mod):
    rng = np.random.default_rng(48)
    R = 300
    rules = []
    for r in range(R):
        hot = {}
        if r % 7 == 0:
            for v in range(3):
                hot[int((r << 20) | v)] = int(rng.integers(0, 6))
        rules.append((float(rng.integers(0, 40)) + (0.5 if r % 5 == 0 else 0.0), int(rng.integers(0, 4)),
                      int(rng.choice([1, 1, 2, 5])), hot))
    rules[3] = (-1.0, 0, 1, {})                 # invalid rule -> NO_RULE_EXISTS
    svc, orc = _local_pair(oracle_mod, rules)
    n = 120_000
    ridx = T.zipf_indices(R, 1.05, n, rng)
    ridx[::501] = R + 3                         # unknown rule
    acq = rng.integers(1, 4, size=n).astype(np.int32)
    b, c, k = T.param_value_lists(np.minimum(ridx, R - 1), rng, universe=60, max_values=3)
    c = c.copy()
    c[::613] = 0                                # empty collection passes
    ts = T.timestamps(n, 20_000.0, T.T0_ALIGNED + 13)
    for lo, hi in [(0, 40_000), (40_000, 120_000)]:
        bb, cc, kk = _slice_lists(b, c, k, lo, hi)
        sg = svc.submit_local_param_batch_host(ridx[lo:hi], acq[lo:hi], ts[lo:hi], bb, cc, kk)
        so = orc.replay(ridx[lo:hi], acq[lo:hi], ts[lo:hi], bb, cc, kk)
        bad = np.nonzero(sg != so)[0]
        assert len(bad) == 0, (len(bad), bad[:5], sg[bad[:5]], so[bad[:5]])
    assert {0, 1, 3} <= set(np.unique(so).tolist())
    for j in range(0, len(k), 401):
        r = int(k[j] >> np.uint64(20))
        lo_, to_ = orc.state(r, int(k[j]))
        lg, tg = svc.local_param_state(int(k[j]))
        assert (lg, tg) == (lo_, to_), (j, lg, tg, lo_, to_)


def _hot_key_batches(n_batches=3, n=30_000, hot_reqs=3000, seed=58):
    """Config-4-shaped batches where, in the first two, one (rule, value) key takes `hot_reqs` requests
    (> PG_CAP = 1280, one LDS chunk of k_pp_group) spread over the batch; the last batch has no such key."""
    count, hot, rule_idx, vals, keys, ts = T.config4(n * n_batches, seed=seed, n_rules=500, universe=100)
    rng = np.random.default_rng(seed)
    rule_idx, keys = rule_idx.copy(), keys.copy()
    for b in range(n_batches - 1):
        pos = b * n + rng.choice(n, size=hot_reqs, replace=False)
        rule_idx[pos] = 7
        keys[pos] = (np.uint64(7) << np.uint64(20)) | np.uint64(3)
    return count, hot, rule_idx, keys, ts


@pytest.mark.parametrize("output", ["arrival", "ordered"])
def test_shared_count_min_subrange_over_chunk_falls_back(oracle_mod, monkeypatch, output):
    """A shared count-min batch with one key over PG_CAP requests: its key-hash sub-range cannot be grouped
    in one LDS chunk, so k_pp_group raises the overflow flag (no workgroup decides or emits anything for
    it) and the whole batch goes to the per-rule lanes -- the path that faulted while the key walk was
    being built.  The fallback batches and the key-walk batch after them are audited
    on exact counters replaying the sketch's own decisions: zero one-sidedness violations."""
    import sentinel_amd as sa
    monkeypatch.setenv("SENTINEL_CM_BLOCK", "1")
    if output == "ordered":
        from conftest import use_ordered_param_host
        use_ordered_param_host(monkeypatch)
    count, hot, rule_idx, keys, ts = _hot_key_batches()
    svc, orc = _cluster_pair(oracle_mod, count, hot, sample_count=lambda r: 10)
    svc.set_param_mode(sa._lib.PARAM_COUNT_MIN_SHARED, depth=4, width=1 << 12)
    acq = np.ones(len(ts), np.int32)
    n = 30_000
    st = []
    for b in range(3):
        s = slice(b * n, (b + 1) * n)
        st.append(svc.submit_param_batch_host(rule_idx[s], acq[s], keys[s], ts[s])[0])
        assert svc.param_cm_stats() == dict(key_walk=max(0, b - 1), overflow=min(b + 1, 2), block=max(0, b - 1)), \
            (b, svc.param_cm_stats())
    st = np.concatenate(st)
    viol, fb, dec = orc.param_cm_audit(rule_idx, acq, ts, np.arange(len(ts)), np.ones(len(ts), np.int32), keys, st)
    assert viol == 0 and dec == len(ts), (viol, dec)
    hk = keys == ((np.uint64(7) << np.uint64(20)) | np.uint64(3))
    assert (st[hk] == 0).any() and (st[hk] == 1).any()


@pytest.mark.parametrize("output", ["arrival", "ordered"])
def test_exact_subrange_over_chunk_bitexact(oracle_mod, monkeypatch, output):
    """The exact twin of the batches above: the hot key's sub-range is decided inside k_pp_group, chunk
    after chunk in arrival order (the key walked once per chunk), bit for bit against the oracle -- also
    with decide-order output, where that sub-range's positions come from a second count of its range."""
    if output == "ordered":
        from conftest import use_ordered_param_host
        use_ordered_param_host(monkeypatch)
    count, hot, rule_idx, keys, ts = _hot_key_batches()
    svc, orc = _cluster_pair(oracle_mod, count, hot, sample_count=lambda r: 10)
    acq = np.where(np.arange(len(ts)) % 7 == 0, 2, 1).astype(np.int32)
    n = 30_000
    for b in range(3):
        s = slice(b * n, (b + 1) * n)
        sg, rg = svc.submit_param_batch_host(rule_idx[s], acq[s], keys[s], ts[s])
        so, ro = orc.param_replay(rule_idx[s], acq[s], keys[s], ts[s])
        bad = np.nonzero((sg != so) | (rg != ro))[0]
        assert len(bad) == 0, (b, len(bad), bad[:5], sg[bad[:5]], so[bad[:5]], rg[bad[:5]], ro[bad[:5]])
    t = int(ts[-1])
    hk = int((np.uint64(7) << np.uint64(20)) | np.uint64(3))
    assert svc.param_sum(7, hk, t) == orc.param_sum(7, t, hk)
