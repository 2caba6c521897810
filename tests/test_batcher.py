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
