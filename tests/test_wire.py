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

