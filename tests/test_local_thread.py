"""THREAD grade and exits on the local path:
DefaultController over curThreadNum, StatisticSlot.exit booking (SUCCESS / RT / minRt / EXCEPTION,
thread count), and ParamFlowChecker's THREAD grade with ParameterMetric's thread counts.

The oracle is pinned by the reference's own tests (DefaultControllerTest.testCanPassForThreadCount,
ParamFlowCheckerTest.testSingleValueCheckThreadCountWithExceptionItems,
ParameterMetricTest.testAddAndDecreaseThreadCount, StatisticNodeTest's minRt / totals); the GPU
path is checked against the oracle on seeded entry / exit traces."""
import numpy as np
import pytest

from sentinel_amd import trace as T

QPS, THREAD, FIRST = 1, 2, 4
PRIO, EXIT, ERROR = 1, 2, 4


# ---------------------------------------------------------------- oracle KATs (CPU)

def test_default_controller_thread_kat(oracle_mod):
    """DefaultControllerTest.testCanPassForThreadCount (DefaultControllerTest.java:29-39): threshold 8,
    curThreadNum 7 -> pass, 8 -> block; here the thread count comes from passing entries."""
    n = oracle_mod.StatisticNode(2, 1000)
    t = T.T0_ALIGNED
    for i in range(7):
        assert n.entry_ex(0, 8, THREAD, 1, t + i) == (True, 0)
    assert n.metrics(t + 7)[13] == 7
    assert n.entry_ex(0, 8, THREAD, 1, t + 8) == (True, 0)      # cur 7: 7 + 1 <= 8
    assert n.entry_ex(0, 8, THREAD, 1, t + 9) == (False, 0)     # cur 8: 8 + 1 > 8
    n.exit(1, 5, t + 10)
    assert n.metrics(t + 10)[13] == 7
    assert n.entry_ex(0, 8, THREAD, 1, t + 11) == (True, 0)


def test_param_thread_kat(oracle_mod):
    """ParamFlowCheckerTest.testSingleValueCheckThreadCountWithExceptionItems
    (ParamFlowCheckerTest.java:99-145): global threshold 5, hot items B = 3, D = 7; a value passes iff
    its thread count + 1 <= threshold.  Counts are built by passing checks (the entry callback)."""
    A, B, C_, D = 11, 12, 13, 14
    L = oracle_mod.LocalParamOracle([(5, 0, 1, {B: 3, D: 7})], grades=[0])

    def check(v):
        return int(L.replay([0], [1], [T.T0_ALIGNED], [0], [1], [v])[0]) == 0

    # counts 4 (A, C), 2 -> 3 for B? build to the KAT's first block: A=4, B=4 (over), C=4, D=6
    for v, k in ((A, 4), (C_, 4), (D, 6)):
        for _ in range(k):
            assert check(v)
    for _ in range(3):
        assert check(B)
    assert L.thread_count(0, A) == 4 and L.thread_count(0, B) == 3 and L.thread_count(0, D) == 6
    assert check(A)              # 4 + 1 <= 5
    assert not check(B)          # 3 + 1 > 3
    assert check(C_)             # 4 + 1 <= 5
    assert check(D)              # 6 + 1 <= 7
    assert not check(A)          # 5 + 1 > 5
    assert not check(D)          # 7 + 1 > 7


def test_param_thread_count_add_decrease(oracle_mod):
    """ParameterMetricTest.testAddAndDecreaseThreadCount (ParameterMetricTest.java:80-160): n adds ->
    n, n - 1 decreases -> 1, one more -> removed; a decrease of an absent value leaves a 0 entry."""
    vals = [19, 3, 8]
    L = oracle_mod.LocalParamOracle([(100, 0, 1, {})], grades=[0])
    n = 3
    for _ in range(n):
        st = L.replay([0], [1], [T.T0_ALIGNED], [0], [3], vals)
        assert st[0] == 0
    assert [L.thread_count(0, v) for v in vals] == [n] * 3
    for _ in range(n - 1):
        L.replay([0], [1], [T.T0_ALIGNED], [0], [3], vals, kinds=[1])
    assert [L.thread_count(0, v) for v in vals] == [1] * 3
    L.replay([0], [1], [T.T0_ALIGNED], [0], [3], vals, kinds=[1])
    assert [L.thread_count(0, v) for v in vals] == [-1] * 3
    L.replay([0], [1], [T.T0_ALIGNED], [0], [1], [vals[0]], kinds=[1])
    assert L.thread_count(0, vals[0]) == 0


def test_exit_booking_and_min_rt(oracle_mod):
    """StatisticNodeTest (StatisticNodeTest.java:100-114): no traffic -> minRt = statisticMaxRt (5000);
    addRtAndSuccess books SUCCESS / RT into both windows, minRt = the smallest rt of the valid buckets
    (ArrayMetric.minRt: max(1, ...)), exceptions only for traced errors."""
    n = oracle_mod.StatisticNode(2, 1000)
    t = T.T0_ALIGNED
    m = n.metrics(t)
    assert m[5] == 5000 and m[12] == 5000 and m[13] == 0
    for i in range(4):
        assert n.entry_ex(10, 0, QPS, 2, t + i)[0]
    n.exit(2, 30, t + 100)
    n.exit(2, 7, t + 200, error=True)
    n.exit(2, 0, t + 300)
    m = n.metrics(t + 300)
    assert list(m[:6]) == [8, 0, 2, 6, 37, 1]             # minRt 0 -> max(1, 0)
    assert list(m[6:]) == [8, 0, 0, 2, 6, 37, 1, 1]
    m = n.metrics(t + 2500)                               # the second window has moved on
    assert list(m[:6]) == [0, 0, 0, 0, 0, 5000]
    assert m[13] == 1


# ---------------------------------------------------------------- GPU vs oracle

def _local_trace(rng, n_res, batches, per_batch, t0, thread_pool_max=4000):
    """Batches of entries (some prioritized) plus exits of entries that passed in earlier batches."""
    out = []
    t = t0
    for _ in range(batches):
        ts = np.sort(t + rng.integers(0, 400, size=per_batch)).astype(np.int64)
        res = rng.integers(0, n_res, size=per_batch).astype(np.int32)
        acq = np.where(rng.random(per_batch) < 0.2, 2, 1).astype(np.int32)
        prio = (rng.random(per_batch) < 0.05).astype(np.uint8)
        out.append((res, acq, ts, prio))
        t += 400
    return out


@pytest.mark.gpu
def test_local_thread_grade_and_exits_vs_oracle(oracle_mod):
    import sentinel_amd as sa
    rng = np.random.default_rng(61)
    R = 24
    qps = [None if r % 6 == 5 else float(rng.integers(5, 60)) for r in range(R)]
    thr = [None if r % 3 == 0 else float(rng.integers(2, 30)) for r in range(R)]
    first = [r % 4 == 1 for r in range(R)]
    svc = sa.GpuTokenService(0)
    svc.load_local_resources_ex(qps, thr, first, sample_count=2, interval_ms=1000)
    nodes = [oracle_mod.StatisticNode(2, 1000) for _ in range(R)]
    flags_of = [(0 if qps[r] is None else QPS) | (0 if thr[r] is None else THREAD) | (FIRST if first[r] else 0)
                for r in range(R)]
    live = []            # (resource, acquire, entry ts) of passed entries not exited yet
    t = T.T0_ALIGNED + 17
    for b in range(30):
        m = 3000
        ts = np.sort(t + rng.integers(0, 300, size=m)).astype(np.int64)
        res = rng.integers(0, R, size=m).astype(np.int32)
        acq = np.where(rng.random(m) < 0.2, 2, 1).astype(np.int32)
        fl = (rng.random(m) < 0.05).astype(np.uint8) * PRIO
        rt = np.zeros(m, np.int64)
        # exits of earlier passed entries replace some events of this batch
        n_exit = min(len(live), m // 3)
        if n_exit:
            pick = rng.choice(len(live), size=n_exit, replace=False)
            slots = rng.choice(m, size=n_exit, replace=False)
            for p, sl in zip(pick, slots):
                r, a, te = live[p]
                res[sl], acq[sl] = r, a
                fl[sl] = EXIT | (ERROR if rng.random() < 0.1 else 0)
                rt[sl] = ts[sl] - te
            live = [x for i, x in enumerate(live) if i not in set(pick.tolist())]
        st_g, w_g = svc.submit_local_batch_host(res, acq, ts, fl, rt)
        st_o = np.zeros(m, np.int8)
        w_o = np.zeros(m, np.int64)
        for i in range(m):
            r = int(res[i])
            nd = nodes[r]
            if fl[i] & EXIT:
                nd.exit(int(acq[i]), int(rt[i]), int(ts[i]), error=bool(fl[i] & ERROR))
                continue
            ok, w = nd.entry_ex(qps[r] or 0.0, thr[r] or 0.0, flags_of[r], int(acq[i]), int(ts[i]), bool(fl[i] & PRIO))
            st_o[i] = 0 if ok else 1
            w_o[i] = w
            if ok:
                live.append((r, int(acq[i]), int(ts[i])))
        bad = np.nonzero((st_g != st_o) | (w_g != w_o))[0]
        assert len(bad) == 0, (b, len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]], w_g[bad[:5]], w_o[bad[:5]])
        t += 300
        if b % 5 == 4:
            for r in range(R):
                g, o = svc.local_node_metrics(r, int(ts[-1])), nodes[r].metrics(int(ts[-1]))
                assert np.array_equal(g, o), (b, r, g, o)


@pytest.mark.gpu
def test_local_param_thread_grade_vs_oracle(oracle_mod):
    import sentinel_amd as sa
    rng = np.random.default_rng(62)
    R = 12
    rules = []
    for r in range(R):
        hot = {((r << 20) | v): int(rng.integers(1, 6)) for v in range(2)} if r % 4 == 0 else {}
        rules.append(sa.LocalParamRule(count=float(rng.integers(2, 10)), burst_count=0, duration_in_sec=1,
                                       hot_items=hot))
    grades = [0 if r % 2 == 0 else 1 for r in range(R)]
    svc = sa.GpuTokenService(0)
    svc.load_local_param_rules(rules)
    svc.set_local_param_grades(grades)
    orc = oracle_mod.LocalParamOracle([(x.count, x.burst_count, x.duration_in_sec, x.hot_items) for x in rules],
                                      grades=grades)
    live = []
    t = T.T0_ALIGNED + 3
    for b in range(20):
        m = 2000
        ridx = rng.integers(0, R, size=m).astype(np.int32)
        counts = rng.integers(1, 3, size=m).astype(np.int32)
        begin = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32)
        vals = ((np.repeat(ridx, counts).astype(np.uint64) << np.uint64(20)) |
                rng.integers(0, 6, size=int(counts.sum())).astype(np.uint64))
        kinds = np.zeros(m, np.uint8)
        # exits of earlier passed THREAD checks: reuse their values
        vlist = [vals[begin[i]:begin[i] + counts[i]] for i in range(m)]
        n_exit = min(len(live), m // 3)
        if n_exit:
            pick = rng.choice(len(live), size=n_exit, replace=False)
            slots = rng.choice(m, size=n_exit, replace=False)
            for p, sl in zip(pick, slots):
                r, vv = live[p]
                ridx[sl] = r
                vlist[sl] = vv
                kinds[sl] = 1
            live = [x for i, x in enumerate(live) if i not in set(pick.tolist())]
        counts = np.array([len(v) for v in vlist], np.int32)
        begin = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32)
        vals = np.concatenate(vlist).astype(np.uint64)
        ts = np.sort(t + rng.integers(0, 500, size=m)).astype(np.int64)
        acq = np.ones(m, np.int32)
        st_g = svc.submit_local_param_batch_ex_host(ridx, acq, ts, begin, counts, vals, kinds)
        st_o = orc.replay(ridx, acq, ts, begin, counts, vals, kinds=kinds)
        bad = np.nonzero(st_g != st_o)[0]
        assert len(bad) == 0, (b, len(bad), bad[:5], st_g[bad[:5]], st_o[bad[:5]])
        for i in range(m):
            if kinds[i] == 0 and st_o[i] == 0 and grades[ridx[i]] == 0:
                live.append((int(ridx[i]), vlist[i]))
        t += 500
    for r in range(0, R, 2):
        for v in range(6):
            key = (r << 20) | v
            assert svc.local_param_state(key)[1] == orc.thread_count(r, key), (r, v)
