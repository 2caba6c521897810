"""The concurrent front doors of the TokenService contract (TokenService.java:36 under Netty worker
threads, NettyTransportServer.java:53-54): the blocking batcher and its asynchronous variant."""
import ctypes as C
import threading

import numpy as np
import pytest

from sentinel_amd import trace as T

pytestmark = pytest.mark.gpu

CB = C.CFUNCTYPE(None, C.c_void_p, C.c_uint64, C.c_void_p)


def test_async_batcher_callbacks():
    """1000 asynchronous requests for one flow (count 100) from 4 threads: exactly 100 pass with the
    remaining counts 99..0 (homogeneous acquire: the set of verdicts does not depend on the order the
    batcher interleaves the threads), every callback fires once, unknown flowIds answer NO_RULE_EXISTS."""
    import sentinel_amd as sa
    from sentinel_amd import _lib
    svc = sa.GpuTokenService(0)
    svc.load_flow_rules([sa.FlowRule(count=100, cluster_config=sa.ClusterFlowConfig(
        flow_id=4242, threshold_type=1, sample_count=2, window_interval_ms=1000))])
    L = svc._L
    L.sentinel_batcher_request_token_async.restype = C.c_int
    L.sentinel_batcher_request_token_async.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_int64, CB,
                                                      C.c_void_p, C.c_uint64]
    b = C.c_void_p()
    assert L.sentinel_batcher_create(svc.handle, 256, 100, C.byref(b)) == 0
    got = {}
    lock = threading.Lock()
    done = threading.Event()

    def on_done(ctx, tag, res):
        r = C.cast(res, C.POINTER(_lib.TokenResultC)).contents
        with lock:
            assert tag not in got
            got[tag] = (r.status, r.remaining)
            if len(got) == 1001:
                done.set()

    cb = CB(on_done)
    t = T.T0_ALIGNED + 50

    def worker(k):
        for i in range(250):
            assert L.sentinel_batcher_request_token_async(b, 4242, 1, 0, t, cb, None, k * 1000 + i) == 0

    th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert L.sentinel_batcher_request_token_async(b, 999, 1, 0, t, cb, None, 99999) == 0
    assert done.wait(30)
    ok = sorted(r for s, r in got.values() if s == 0)
    assert ok == list(range(100))
    assert sum(1 for s, _ in got.values() if s == 1) == 900
    assert got[99999][0] == sa.TokenResultStatus.NO_RULE_EXISTS
    L.sentinel_batcher_destroy(b)


def test_sync_batcher_survives_reload_and_destroy():
    """Blocking callers across a rule reload (the lookup happens with the decision, under the engine
    lock) and a destroy while callers are still being woken."""
    import sentinel_amd as sa
    from sentinel_amd.token_service import TokenBatcher
    svc = sa.GpuTokenService(0)
    rule = lambda fid, c: sa.FlowRule(count=c, cluster_config=sa.ClusterFlowConfig(
        flow_id=fid, threshold_type=1, sample_count=2, window_interval_ms=1000))
    svc.load_flow_rules([rule(1, 1e9), rule(2, 1e9)])
    b = TokenBatcher(svc, max_batch=64, max_wait_us=50)
    stop = threading.Event()
    seen = []

    def worker():
        t = T.T0_ALIGNED
        while not stop.is_set():
            t += 1
            r = b.request_token(2, 1, False, ts=t)
            seen.append(r.status)

    th = [threading.Thread(target=worker) for _ in range(8)]
    for x in th:
        x.start()
    for k in range(10):
        svc.load_flow_rules([rule(2, 1e9)] if k % 2 else [rule(1, 1e9), rule(2, 1e9)])
    stop.set()
    for x in th:
        x.join()
    b.close()
    assert seen and set(seen) == {0}


def test_async_batcher_large_batches_decide_order(oracle_mod, monkeypatch):
    """Batches larger than the one-launch kernel's 4096 events are decided by the partition path with
    decide-order output (sentinel_submit_flow_batch_ordered): the batcher answers each request from
    (seq[j], verdict[j]) -- the wire server's path -- with no arrival-order permutation anywhere.
    60k asynchronous requests in one call (Zipf flows, acquire 1..3, prioritized requests, unknown and
    invalid flowIds), decided as batches of up to 32768 in arrival order: every callback fires once,
    with the oracle's verdict for its own request."""
    import sentinel_amd as sa
    from sentinel_amd import _lib
    monkeypatch.setenv("SENTINEL_FLOW_PATH", "partition")
    n = 60_000
    rules, ev = T.config2(n, seed=21, n_flows=5000)
    svc = sa.GpuTokenService(0)
    svc.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count,
                         rules.window_interval_ms, rules.namespace, rules.checker)
    rng = np.random.default_rng(21)
    idx = ev.flow_idx.astype(np.int32).copy()
    acq = rng.integers(1, 4, size=n).astype(np.int32)
    flags = (rng.random(n) < 0.02).astype(np.uint8)
    ids = np.asarray(rules.flow_id, dtype=np.int64)[idx]
    ids[::997] = 10 ** 12 + 5                               # no rule -> NO_RULE_EXISTS
    idx[::997] = _lib.IDX_NO_RULE
    ids[::1499] = 0                                         # flowId <= 0 -> BAD_REQUEST
    idx[::1499] = _lib.IDX_BAD_ID
    ts = np.ascontiguousarray(ev.ts, dtype=np.int64)
    L = svc._L
    L.sentinel_batcher_request_tokens_async.restype = C.c_int
    L.sentinel_batcher_request_tokens_async.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                                       C.c_void_p, CB, C.c_void_p, C.c_void_p]
    b = C.c_void_p()
    assert L.sentinel_batcher_create(svc.handle, 32768, 200_000, C.byref(b)) == 0
    st = np.full(n, -100, np.int32)
    rem = np.zeros(n, np.int32)
    wt = np.zeros(n, np.int32)
    fired = np.zeros(n, np.int32)
    done = threading.Event()
    cnt = [0]

    def on_done(ctx, tag, res):
        r = C.cast(res, C.POINTER(_lib.TokenResultC)).contents
        st[tag], rem[tag], wt[tag] = r.status, r.remaining, r.wait_in_ms
        fired[tag] += 1
        cnt[0] += 1
        if cnt[0] == n:
            done.set()

    cb = CB(on_done)
    tags = np.arange(n, dtype=np.uint64)
    assert L.sentinel_batcher_request_tokens_async(b, n, ids.ctypes.data, acq.ctypes.data, flags.ctypes.data,
                                                   ts.ctypes.data, cb, None, tags.ctypes.data) == 0
    assert done.wait(120)
    nb, nr = C.c_int64(), C.c_int64()
    assert L.sentinel_batcher_stats(b, C.byref(nb), C.byref(nr)) == 0
    L.sentinel_batcher_destroy(b)
    assert (fired == 1).all()
    assert nr.value == n and nb.value >= 2
    assert svc.flow_path_stats()["ordered"] >= 2, svc.flow_path_stats()    # decide-order partition batches
    orc = oracle_mod.TokenServiceOracle(rules.as_dicts())
    st_o, rem_o, w_o = orc.replay(idx, acq, ts, flags)
    bad = np.nonzero((st != st_o) | (rem != rem_o) | (wt != w_o))[0]
    assert len(bad) == 0, (len(bad), bad[:5], st[bad[:5]], st_o[bad[:5]], rem[bad[:5]], rem_o[bad[:5]])
    assert {0, 1, sa.TokenResultStatus.NO_RULE_EXISTS, sa.TokenResultStatus.BAD_REQUEST} <= set(np.unique(st_o).tolist())
