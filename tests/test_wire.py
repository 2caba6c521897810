"""Token-server wire front end (sentinel_amd/wire.py): the reference's frame layouts and codec
behaviour on CPU, and an end-to-end TCP run on the GPU checked against the oracle replaying the
server's decision log."""
import struct
import threading

import numpy as np
import pytest

from sentinel_amd import wire as W
from sentinel_amd import trace as T


def test_flow_request_layout_and_framing():
    f = W.encode_flow_request(7, 111, 3, True)
    # [u16 len=18][i32 xid][i8 type=1][i64 flowId][i32 count][i8 prio]  (FlowRequestDataDecoder.java:28)
    assert f == bytes.fromhex("0012" "00000007" "01" "000000000000006f" "00000003" "01")
    d = W.FrameDecoder()
    bodies = []
    for i in range(len(f) * 2):                     # byte-at-a-time delivery of two frames
        bodies += d.feed((f + f)[i:i + 1])
    assert bodies == [f[2:], f[2:]]
    req = W.decode_request(bodies[0])
    assert (req.xid, req.type, req.data) == (7, 1, (111, 3, True))
    # the priority byte is optional (FlowRequestDataDecoder.java:42-44)
    assert W.decode_request(f[2:-1]).data == (111, 3, False)
    assert W.decode_request(f[2:8]).data is None    # < 12 data bytes -> null data
    assert W.decode_request(f[2:7]).data is None    # no data at all -> null data
    assert W.decode_request(f[2:6]) is None         # < 5 bytes: nothing decoded
    assert W.decode_request(struct.pack(">ib", 1, 9) + b"\0" * 13) is None   # no decoder for type 9


def test_too_long_frames_are_discarded():
    d = W.FrameDecoder()
    big = struct.pack(">H", 1023) + b"\x01" * 1023  # 1023 + 2 > 1024: TooLongFrameException, skipped
    ok = W.encode_flow_request(1, 5, 1)
    out = d.feed(big[:300]) + d.feed(big[300:] + ok)
    assert out == [ok[2:]]
    assert d.feed(struct.pack(">H", 1022) + b"\0" * 1022) == [b"\0" * 1022]   # 1022 + 2 fits


def test_param_request_codec():
    params = [W.jint(1), W.jlong(1), W.jstr("abc"), W.jdouble(2.5), W.jfloat(-0.0), W.jbool(True),
              W.jbyte(-3), W.jshort(300), W.jdouble(float("nan"))]
    f = W.encode_param_request(9, 42, 2, params)
    req = W.decode_request(W.FrameDecoder().feed(f)[0])
    assert req.type == W.MSG_TYPE_PARAM_FLOW and req.data[0] == 42 and req.data[1] == 2
    assert req.data[2] == params
    assert W.jint(1) != W.jlong(1) and W.jfloat(0.0) != W.jfloat(-0.0)       # Java equals()
    assert W.jdouble(float("nan")) == W.jdouble(-float("nan"))              # doubleToLongBits canonical NaN
    # amount <= 0 -> null data; an unknown type byte is skipped on its own (decoder java:86-88)
    assert W.decode_request(struct.pack(">ibqii", 1, 2, 42, 1, 0)).data is None
    body = struct.pack(">ibqii", 1, 2, 42, 1, 2) + b"\x09" + struct.pack(">bi", 0, 5)
    assert W.decode_request(body).data == (42, 1, [W.jint(5)])
    # truncated value: Netty raises, nothing reaches the handler
    assert W.decode_request(struct.pack(">ibqii", 1, 2, 42, 1, 1) + b"\x01\x00") is None


def test_client_param_size_cap_matches_reference_test():
    """ParamFlowRequestDataWriterTest.java:31-55: cap 15 bytes keeps 1, 64, 3 (5 B each) and drops 5."""
    ps = [W.jint(1), W.jint(64), W.jint(3)]
    assert W.resolve_valid_params(ps, 15) == ps
    assert W.jint(5) not in W.resolve_valid_params(ps + [W.jint(5)], 15)
    assert W.resolve_valid_params([W.TypedValue(99, object())], 15) == []


def test_response_codec():
    r = W.encode_response(5, W.MSG_TYPE_FLOW, 1, (12, 13))     # FlowResponseDataDecoderTest: 12, 13
    assert r == bytes.fromhex("000e" "00000005" "01" "01" "0000000c" "0000000d")
    assert W.decode_response(r[2:]) == (5, 1, 1, (12, 13))
    assert W.decode_response(W.encode_response(6, W.MSG_TYPE_FLOW, -4, (0, 0))[2:])[2] == -4
    assert W.decode_response(W.encode_response(7, W.MSG_TYPE_PING, 0, 2147483647)[2:]) == (7, 0, 0, 2147483647)
    assert W.encode_response(8, W.MSG_TYPE_PING, -1) == bytes.fromhex("0006" "00000008" "00" "ff")
    ping = W.encode_ping(3, "ns-a")
    req = W.decode_request(ping[2:])
    assert (req.type, req.data) == (0, "ns-a")


def test_interner_is_injective_per_rule():
    it = W.ParamKeyInterner()
    a = it.key(1, W.jint(7))
    assert it.key(1, W.jint(7)) == a
    assert len({a, it.key(1, W.jlong(7)), it.key(2, W.jint(7)), it.key(1, W.jstr("7"))}) == 4


@pytest.mark.gpu
def test_server_end_to_end_against_oracle(oracle_mod):
    import sentinel_amd as sa
    from sentinel_amd.token_service import ServerNamespace
    rng = np.random.default_rng(61)
    F = 200
    rules, _ = T.config2(1, seed=61, n_flows=F)
    rules.count[:] = rng.integers(5, 60, size=F)
    rules.threshold_type[::4] = 0                   # AVG_LOCAL: threshold x connectedCount of "default"
    svc = sa.GpuTokenService(0)
    svc.set_namespaces([ServerNamespace(connected_count=0)])
    svc.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count,
                         rules.window_interval_ms, rules.namespace, rules.checker)
    interner = W.ParamKeyInterner()
    svc.load_param_rules([sa.ParamFlowRule(count=4.0, cluster_config=sa.ClusterFlowConfig(
        flow_id=900 + r, threshold_type=1, sample_count=2, window_interval_ms=1000),
        hot_items={interner.key(900 + r, W.jstr("vip")): 1}) for r in range(10)])
    tick = [T.T0_ALIGNED]
    lock = threading.Lock()

    def clock():
        with lock:
            tick[0] += 1
            return tick[0] // 3
    server = W.ClusterTokenServer(svc, ["default"], clock=clock, interner=interner, record=True, max_wait_ms=0.3)
    port = server.start()
    n_clients, per_client = 6, 300
    answers = [dict() for _ in range(n_clients)]
    pinged = threading.Barrier(n_clients)

    def client(c):
        cl = W.TokenClient("127.0.0.1", port)
        r = np.random.default_rng(100 + c)
        cl.send(W.encode_ping(1, "default"))
        answers[c][1] = cl.recv()
        pinged.wait(60)                              # every client is connected before any request
        for k in range(per_client):
            xid = 2 + k
            if k % 5 == 4:
                vals = [W.jstr("vip") if r.random() < 0.3 else W.jint(int(r.integers(0, 5)))
                        for _ in range(int(r.integers(1, 3)))]
                cl.send(W.encode_param_request(xid, 900 + int(r.integers(0, 11)), 1, vals))
            else:
                cl.send(W.encode_flow_request(xid, int(rules.flow_id[int(r.integers(0, F))]) if k % 37 else -5,
                                              int(r.integers(0, 3)), bool(r.random() < 0.1)))
            if k % 50 == 49:                         # pipelined: collect replies in bursts
                while len(answers[c]) < xid:
                    x = cl.recv()
                    answers[c][x[0]] = x
        while len(answers[c]) < per_client + 1:
            x = cl.recv()
            answers[c][x[0]] = x
        pinged.wait(60)                              # nobody disconnects (connectedCount--) before all are done
        cl.close()

    th = [threading.Thread(target=client, args=(c,)) for c in range(n_clients)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    server.stop()
    assert all(len(a) == per_client + 1 for a in answers)
    # replay the server's decision log through the oracle (connectedCount = every client)
    kinds = [k for k, _, _ in server.log]
    assert kinds[:n_clients] == ["ping"] * n_clients and "ping" not in kinds[n_clients:]
    last = max(i for i, k in enumerate(kinds) if k in ("flow", "param"))
    assert "disconnect" not in kinds[:last]
    orc = oracle_mod.TokenServiceOracle(rules.as_dicts(), namespaces=[dict(connected_count=n_clients)],
                                        param_rules=[dict(flow_id=900 + r, count=4.0, threshold_type=1, sample_count=2,
                                                          window_interval_ms=1000) for r in range(10)],
                                        hot_items={r: [(interner.key(900 + r, W.jstr("vip")), 1)] for r in range(10)})
    expect = []
    for kind, payload, ts in server.log[n_clients:]:
        if kind == "flow":
            idx, acq, prio = payload
            s, rem, wt = orc.replay(idx, acq, ts, prio)
            expect.extend(zip(s.tolist(), rem.tolist(), wt.tolist()))
        elif kind == "param":
            idx, acq, begin, cnt, keys = payload
            s, rem = orc.param_multi_replay(idx, acq, ts, begin, cnt, keys)
            expect.extend(zip(s.tolist(), rem.tolist(), [0] * len(s)))
    got = sorted((x[2], x[3][0], x[3][1]) for a in answers for xid, x in a.items() if xid > 1)
    assert got == sorted(expect)
    assert {a[1][3] for a in answers} <= set(range(1, n_clients + 1))   # connectedCount replies
    assert server.batches >= 1



def test_native_interner_equality_classes_match_python():
    """sentinel_param_interner (C++) partitions (flowId, typed value) pairs exactly as the Python
    ParamKeyInterner does: Java equals() -- the tag separates Integer(1) / Long(1), NaNs collapse,
    -0.0 != 0.0, strings compare by their decoded text."""
    nat = W.NativeParamInterner()
    py = W.ParamKeyInterner()
    vals = [W.jint(1), W.jlong(1), W.jint(-1), W.jbyte(1), W.jshort(1), W.jbool(True), W.jbool(False),
            W.jdouble(0.0), W.jdouble(-0.0), W.jdouble(float("nan")), W.TypedValue(W.PARAM_TYPE_DOUBLE, 0x7FF0000000000001),
            W.jfloat(float("nan")), W.TypedValue(W.PARAM_TYPE_FLOAT, 0x7F800001), W.jfloat(1.5), W.jdouble(1.5),
            W.jstr("vip"), W.jstr("VIP"), W.jstr(""), W.jstr("été"), W.jint(1)]
    # Python keys the values its decoder produces (NaN payloads canonical after the float round trip);
    # the native interner gets the raw wire bits
    decoded = W.decode_request(W.encode_param_request(1, 7, 1, vals)[2:]).data[2]
    assert len(decoded) == len(vals)
    for fid in (7, 8):
        n = [nat.key(fid, v) for v in vals]
        p = [py.key(fid, v) for v in decoded]
        for i in range(len(vals)):
            for j in range(len(vals)):
                assert (n[i] == n[j]) == (p[i] == p[j]), (vals[i], vals[j])
    assert nat.key(7, W.jint(1)) != nat.key(8, W.jint(1))
    assert min(nat.key(7, v) for v in vals) >= 1
    nat.close()


def test_native_interner_is_bounded():
    """A flood of distinct values cannot grow the native interner without limit: past max_entries,
    values idle for longer than idle_ms go first (exact: their windows are empty), then the least
    recently used; a value in use keeps its key; keys are never reused."""
    nat = W.NativeParamInterner()
    nat.set_limits(1000, 5000)
    hot = nat.key(7, W.jlong(-1), ts=0)
    seen = set()
    for i in range(20_000):
        t = i                                       # 1 ms apart: the last 5000 are inside the horizon
        seen.add(nat.key(7, W.jlong(i), ts=t))
        if i % 100 == 0:
            assert nat.key(7, W.jlong(-1), ts=t) == hot      # recently used: same key
        assert nat.stats()["entries"] <= 1000
    st = nat.stats()
    assert st["evicted"] >= 19_000 and len(seen) == 20_000  # keys are unique, never recycled
    # an idle value comes back with a fresh key (its window expired; the reference's CacheMaps are empty too)
    assert nat.key(7, W.jlong(0), ts=20_000) not in seen
    nat.close()


def test_native_interner_steady_churn_scans_rarely():
    """Distinct values arriving 1 ms apart with idle_ms just under the cap's span: every insert past the
    cap finds exactly one idle entry.  Each full pass must end at the 3/4 low-water mark, so passes run
    at most once per cap / 4 inserts (one pass per insert before the hysteresis)."""
    nat = W.NativeParamInterner()
    nat.set_limits(1000, 999)
    n = 20_000
    for i in range(n):
        nat.key(7, W.jlong(i), ts=i)
        assert nat.stats()["entries"] <= 1000
    st = nat.stats()
    assert st["scans"] <= n // 250 + 2, st
    assert nat.key(7, W.jlong(n - 1), ts=n) is not None
    nat.close()


def _ask(cl, frame):
    cl.send(frame)
    return cl.recv()


@pytest.mark.gpu
def test_native_server_sequential_matches_oracle(oracle_mod):
    """sentinel_wire_server over TCP, one request at a time with a controlled clock: every FLOW and
    PARAM response equals the oracle replaying the same requests in the same order (connectedCount
    from the PINGs: AVG_LOCAL thresholds), and the protocol edge cases behave as wire.py's."""
    import sentinel_amd as sa
    from sentinel_amd.token_service import ServerNamespace
    rng = np.random.default_rng(62)
    F = 120
    rules, _ = T.config2(1, seed=62, n_flows=F)
    rules.count[:] = rng.integers(3, 30, size=F)
    rules.threshold_type[::4] = 0
    svc = sa.GpuTokenService(0)
    svc.set_namespaces([ServerNamespace(connected_count=0)])
    svc.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count,
                         rules.window_interval_ms, rules.namespace, rules.checker)
    interner = W.NativeParamInterner()
    svc.load_param_rules([sa.ParamFlowRule(count=3.0, cluster_config=sa.ClusterFlowConfig(
        flow_id=900 + r, threshold_type=1, sample_count=2, window_interval_ms=1000),
        hot_items={interner.key(900 + r, W.jstr("vip")): 1}) for r in range(6)])
    now = [T.T0_ALIGNED + 5]
    server = W.NativeTokenServer(svc, ["default"], clock=lambda: now[0], interner=interner, io_threads=2)
    try:
        a, b = W.TokenClient("127.0.0.1", server.port), W.TokenClient("127.0.0.1", server.port)
        assert _ask(a, W.encode_ping(1, "default")) == (1, 0, 0, 1)
        assert _ask(b, W.encode_ping(2, "default")) == (2, 0, 0, 2)
        assert _ask(a, W.encode_ping(3, " \t")) == (3, 0, -1, None)          # blank namespace: BAD
        assert _ask(a, W._frame(struct.pack(">ib", 4, 0))) == (4, 0, -1, None)   # no data: BAD
        # frames that produce nothing: too long (skipped), unknown type, flow with null data
        a.send(struct.pack(">H", 1023) + b"\x01" * 1023)
        a.send(W._frame(struct.pack(">ib", 5, 9) + b"\0" * 13))
        a.send(W._frame(struct.pack(">ibq", 6, 1, 5)))
        orc = oracle_mod.TokenServiceOracle(rules.as_dicts(), namespaces=[dict(connected_count=2)],
                                            param_rules=[dict(flow_id=900 + r, count=3.0, threshold_type=1,
                                                              sample_count=2, window_interval_ms=1000) for r in range(6)],
                                            hot_items={r: [(interner.key(900 + r, W.jstr("vip")), 1)] for r in range(6)})
        fid_to_idx = {int(f): i for i, f in enumerate(rules.flow_id)}
        for k in range(500):
            now[0] += int(rng.integers(0, 40))
            xid = 100 + k
            cl = a if k % 3 else b
            if k % 5 == 4:
                r = int(rng.integers(0, 8))          # 6: no rule; 7: flowId 0 or < 0 (BAD_REQUEST)
                fid = 900 + r if r < 7 else int(rng.integers(-3, 1))
                vals = [W.jstr("vip") if rng.random() < 0.3 else W.jint(int(rng.integers(0, 4)))
                        for _ in range(int(rng.integers(1, 3)))]
                got = _ask(cl, W.encode_param_request(xid, fid, 1, vals))
                keys = np.array([interner.key(fid, v) for v in vals], dtype=np.uint64)
                s, rem = orc.param_multi_replay(np.array([r if r < 6 else (-1 if r == 6 else -2)], np.int32), np.ones(1, np.int32),
                                                np.array([now[0]], np.int64), np.zeros(1, np.int32),
                                                np.array([len(vals)], np.int32), keys)
                assert got == (xid, 2, int(s[0]), (int(rem[0]), 0)), (k, got, s, rem)
            else:
                fid = int(rules.flow_id[int(rng.integers(0, F))]) if k % 37 else -5
                acq = int(rng.integers(0, 3))
                prio = bool(rng.random() < 0.1)
                got = _ask(cl, W.encode_flow_request(xid, fid, acq, prio))
                idx = np.array([fid_to_idx.get(fid, -2 if fid <= 0 else -1)], np.int32)
                s, rem, wt = orc.replay(idx, np.array([acq], np.int32), np.array([now[0]], np.int64),
                                        np.array([1 if prio else 0], np.uint8))
                assert got == (xid, 1, int(s[0]), (int(rem[0]), int(wt[0]))), (k, got, s, rem, wt)
        st = server.stats()
        assert st["connections"] == 2 and st["flow_requests"] == 400 and st["param_requests"] == 100
        a.close()
        b.close()
    finally:
        server.stop()
        interner.close()


@pytest.mark.gpu
def test_native_server_pipelined_clients():
    """Many connections with deep pipelines: every request answered exactly once with its own xid,
    statuses OK / BLOCKED / SHOULD_WAIT only, and a flow's passes within one second never exceed its
    count (the server clock is frozen, so every request lands in one window)."""
    import sentinel_amd as sa
    from sentinel_amd.token_service import ServerNamespace
    F = 50
    rules, _ = T.config2(1, seed=63, n_flows=F)
    rules.count[:] = 40
    svc = sa.GpuTokenService(0)
    svc.set_namespaces([ServerNamespace(connected_count=1)])
    svc.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count,
                         rules.window_interval_ms, rules.namespace, rules.checker)
    server = W.NativeTokenServer(svc, ["default"], clock=lambda: T.T0_ALIGNED + 500, io_threads=3)
    n_clients, per_client = 8, 2000
    passes = np.zeros(F, np.int64)
    lock = threading.Lock()
    errors = []

    def client(c):
        try:
            cl = W.TokenClient("127.0.0.1", server.port)
            r = np.random.default_rng(200 + c)
            fids = r.integers(0, F, size=per_client)
            buf = b"".join(W.encode_flow_request(1 + k, int(rules.flow_id[fids[k]]), 1) for k in range(per_client))
            cl.send(buf)
            seen = {}
            while len(seen) < per_client:
                xid, typ, status, data = cl.recv()
                assert typ == 1 and xid not in seen and 1 <= xid <= per_client
                seen[xid] = status
            local = np.zeros(F, np.int64)
            for xid, status in seen.items():
                assert status in (0, 1)
                if status == 0:
                    local[fids[xid - 1]] += 1
            with lock:
                passes[:] += local
            cl.close()
        except Exception as ex:        # surfaced below
            errors.append(ex)

    th = [threading.Thread(target=client, args=(c,)) for c in range(n_clients)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    st = server.stats()
    server.stop()
    assert not errors, errors
    assert st["flow_requests"] == n_clients * per_client
    assert (passes <= 40).all() and passes.sum() == 40 * F        # every flow saturates exactly
