"""The one-sweep partition front (k_part_split, partition.hpp) against the oracle.

k_part_split replaces k_part_prep + the three scan launches + k_part_scatter for batches of >= 64K
events on an engine that is alone on its device.  These cases pin what is specific to it: every
events-per-thread instantiation (8 / 16 / 32: batches of 64K .. 8M events over 8 .. 256
workgroups), ragged batch ends (a last workgroup with a partial chunk and waves with no events),
range digits of 0 .. 10 bits (flow tables from 1000 to 1M flows), rejected events of every kind
mixed in (their verdicts come from the split kernel; ts < 0 is a documented divergence and left
out), prioritized flags carried into the sorted values, and consecutive batches (the monotonic
barrier counter across launches).  Bar: bit-exact
statuses, remaining counts and waits, and window dumps.
"""
import gc

import numpy as np
import pytest

from sentinel_amd import trace as T

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _partition(monkeypatch):
    monkeypatch.setenv("SENTINEL_FLOW_PATH", "partition")
    monkeypatch.setenv("SENTINEL_PART_SPLIT", "1")
    gc.collect()                    # engines of earlier tests: the split path needs its engine alone on the device


def _engine(rules):
    import sentinel_amd as sa
    svc = sa.GpuTokenService(0)
    svc.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count,
                         rules.window_interval_ms, rules.namespace, rules.checker)
    return svc


def _oracle(oracle_mod, rules):
    return oracle_mod.TokenServiceOracle.from_arrays(rules.flow_id, rules.count, rules.threshold_type,
                                                     rules.sample_count, rules.window_interval_ms,
                                                     rules.namespace, rules.checker)


def _trace(rng, F, n, t0, ms_per_event, bad=True, prio=True):
    idx = rng.integers(0, F, n, dtype=np.int64).astype(np.int32)
    acq = np.ones(n, np.int32)
    ts = (t0 + np.floor(np.arange(n, dtype=np.float64) * ms_per_event)).astype(np.int64)
    flags = None
    if bad:
        k = rng.choice(n, size=max(4, n // 500), replace=False)
        kind = np.arange(len(k)) % 5
        idx[k[kind == 0]] = -1                       # NO_RULE (unknown flowId)
        idx[k[kind == 1]] = F + 7                    # NO_RULE (past the table)
        acq[k[kind == 2]] = 0                        # BAD_REQUEST
        acq[k[kind == 3]] = -3                       # BAD_REQUEST
        idx[k[kind == 4]] = -2                       # BAD_REQUEST (null flowId)
        # (ts < 0 is a documented divergence -- FAIL here, an NPE in the reference -- so the trace has none)
    if prio:
        flags = (rng.random(n) < 0.002).astype(np.uint8)
    return idx, acq, ts, flags


def _run(oracle_mod, F, n, batches, seed, sample_count=10, expect_split=True):
    rng = np.random.default_rng(seed)
    rules = T.make_rules(F, rng, sample_count=sample_count, window_interval_ms=1000)
    svc = _engine(rules)
    orc = _oracle(oracle_mod, rules)
    ms = 1000.0 / (2.0 * float(rules.count.sum()))
    t0 = T.T0_ALIGNED + 3
    for b in range(batches):
        idx, acq, ts, fl = _trace(rng, F, n, t0, ms)
        t0 = int(ts.max()) + 1
        st_g, rem_g, w_g = svc.submit_flow_batch_host(idx, acq, ts, fl)
        if n <= 1_000_000:
            st_o, rem_o, w_o = orc.replay(idx, acq, ts, fl)
        else:
            st_o, rem_o, w_o, _ = orc.replay_mt(idx, acq, ts, 16, fl)
        bad = np.nonzero((st_g != st_o) | (rem_g != rem_o) | (w_g != w_o))[0]
        assert len(bad) == 0, (F, n, b, len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]], rem_g[bad[:5]], rem_o[bad[:5]])
    for f in np.random.default_rng(1).choice(F, min(F, 300), replace=False):
        assert np.array_equal(svc.dump_flow(int(f), sample_count), orc.dump_flow(int(f))), f
    stats = svc.flow_path_stats()
    if expect_split:
        assert stats["split"] == batches and stats["partition"] == 0, stats
    return svc, stats


@pytest.mark.parametrize("F,n", [
    (1000, 65_536),          # 8 events per thread, 8 workgroups, lb = 0 (one flow per range)
    (50_000, 300_001),       # ragged: a partial last chunk, waves with no events; 6-bit local keys
    (1_000_000, 2_100_000),  # 16 events per thread (2.1M > 256 x 8K), 10-bit local keys
])
def test_split_bitexact(oracle_mod, F, n):
    _run(oracle_mod, F, n, batches=3, seed=F + n)


def test_split_full_size_32_items(oracle_mod):
    """The bench's own shape: 8M events over 256 workgroups of 32 events per thread, 1M flows."""
    _run(oracle_mod, 1_000_000, 8 * 1024 * 1024, batches=2, seed=77)


def test_split_needs_engine_alone_on_device(oracle_mod):
    """With a second engine on the device the batch takes prep + scan + scatter (no grid barrier
    between two persistent launches), and is still bit-exact."""
    import sentinel_amd as sa
    other = sa.GpuTokenService(0)
    try:
        _, stats = _run(oracle_mod, 20_000, 200_000, batches=1, seed=5, expect_split=False)
        assert stats["split"] == 0 and stats["partition"] == 1, stats
    finally:
        other.close()
