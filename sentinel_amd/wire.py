"""Cluster token-server wire front end over the MI355X engine.

The reference's token server is Netty (paths relative to
sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/alibaba/csp/sentinel/cluster/server/):

  framing   NettyTransportServer.java:89-92   LengthFieldBasedFrameDecoder(1024, 0, 2, 0, 2) in,
                                               LengthFieldPrepender(2) out: a big-endian u16 length
  request   codec/DefaultRequestEntityDecoder.java:42-63   [i32 xid][i8 type][data]
            codec/data/PingRequestDataDecoder.java:29-39    type 0: [i32 len][bytes namespace]
            codec/data/FlowRequestDataDecoder.java:37-48    type 1: [i64 flowId][i32 count][bool prio]?
            codec/data/ParamFlowRequestDataDecoder.java:35-90  type 2: [i64 flowId][i32 count][i32 n]{[i8 type][value]}
  response  codec/DefaultResponseEntityWriter.java:35-52  [i32 xid][i8 type][i8 status] + data
            codec/data/FlowResponseDataWriter.java:30-33   [i32 remaining][i32 waitInMs] (types 1, 2)
            codec/data/PingResponseDataWriter.java:30-35   [i32 connectedCount] (type 0)
  handling  handler/TokenServerHandler.java:61-106, processor/FlowRequestProcessor.java:36-53,
            processor/ParamFlowRequestProcessor.java:38-55, connection/ConnectionManager.java

Instead of one synchronous TokenService call per frame, the server decodes frames from every
connection on one event loop and a dispatcher decides them in GPU batches, in arrival order:
maximal runs of FLOW or PARAM requests become one batch each, PINGs update the namespace's
connectedCount between runs (AVG_LOCAL thresholds depend on it).  Responses go back on each
connection in its own request order, as Netty writes them.
"""
from __future__ import annotations

import asyncio
import math
import socket
import struct
import threading
import time
from dataclasses import dataclass
from typing import Callable, Dict, List, NamedTuple, Optional, Sequence, Tuple

import numpy as np

from .token_service import GpuTokenService, TokenResultStatus

MSG_TYPE_PING, MSG_TYPE_FLOW, MSG_TYPE_PARAM_FLOW = 0, 1, 2            # ClusterConstants.java:24-26
RESPONSE_STATUS_BAD, RESPONSE_STATUS_OK = -1, 0                         # ClusterConstants.java:31-32
(PARAM_TYPE_INTEGER, PARAM_TYPE_LONG, PARAM_TYPE_BYTE, PARAM_TYPE_DOUBLE, PARAM_TYPE_FLOAT, PARAM_TYPE_SHORT,
 PARAM_TYPE_BOOLEAN, PARAM_TYPE_STRING) = range(8)                      # ClusterConstants.java:34-41
MAX_FRAME_LENGTH = 1024
DEFAULT_PARAM_MAX_SIZE = 1024                                           # ParamFlowRequestDataWriter


class TypedValue(NamedTuple):
    """A Java-typed parameter value with Java equals() semantics: the tag keeps Integer(1) != Long(1);
    Double / Float compare by doubleToLongBits / floatToIntBits (NaNs canonical, -0.0 != 0.0)."""
    tag: int
    value: object


def jint(v: int) -> TypedValue: return TypedValue(PARAM_TYPE_INTEGER, int(np.int32(v)))
def jlong(v: int) -> TypedValue: return TypedValue(PARAM_TYPE_LONG, int(np.int64(v)))
def jbyte(v: int) -> TypedValue: return TypedValue(PARAM_TYPE_BYTE, int(np.int8(v)))
def jshort(v: int) -> TypedValue: return TypedValue(PARAM_TYPE_SHORT, int(np.int16(v)))
def jbool(v: bool) -> TypedValue: return TypedValue(PARAM_TYPE_BOOLEAN, bool(v))
def jstr(v: str) -> TypedValue: return TypedValue(PARAM_TYPE_STRING, str(v))


def jdouble(v: float) -> TypedValue:
    if math.isnan(v):
        return TypedValue(PARAM_TYPE_DOUBLE, 0x7FF8000000000000)
    return TypedValue(PARAM_TYPE_DOUBLE, struct.unpack(">Q", struct.pack(">d", v))[0])


def jfloat(v: float) -> TypedValue:
    if math.isnan(v):
        return TypedValue(PARAM_TYPE_FLOAT, 0x7FC00000)
    return TypedValue(PARAM_TYPE_FLOAT, struct.unpack(">I", struct.pack(">f", v))[0])


# ------------------------------------------------------------------ framing + codecs

class FrameDecoder:
    """LengthFieldBasedFrameDecoder(maxFrameLength 1024, offset 0, length 2, adjustment 0, strip 2):
    frames whose length + 2 exceed 1024 are discarded (failFast TooLongFrameException)."""

    def __init__(self):
        self.buf = bytearray()
        self.discard = 0

    def feed(self, data: bytes) -> List[bytes]:
        self.buf += data
        out = []
        while True:
            if self.discard:
                d = min(self.discard, len(self.buf))
                del self.buf[:d]
                self.discard -= d
                if self.discard:
                    break
            if len(self.buf) < 2:
                break
            length = (self.buf[0] << 8) | self.buf[1]
            if length + 2 > MAX_FRAME_LENGTH:
                del self.buf[:2]
                self.discard = length
                continue
            if len(self.buf) < 2 + length:
                break
            out.append(bytes(self.buf[2:2 + length]))
            del self.buf[:2 + length]
        return out


@dataclass
class Request:
    xid: int
    type: int
    data: object      # PING: str | None; FLOW: (flowId, count, prio) | None; PARAM: (flowId, count, [TypedValue]) | None


class _Reader:
    def __init__(self, b: bytes):
        self.b, self.i = b, 0

    def readable(self) -> int:
        return len(self.b) - self.i

    def take(self, fmt: str):
        n = struct.calcsize(fmt)
        if self.readable() < n:
            raise IndexError("readerIndex out of bounds")
        v = struct.unpack_from(fmt, self.b, self.i)
        self.i += n
        return v[0] if len(v) == 1 else v

    def bytes(self, n: int) -> bytes:
        if n < 0 or self.readable() < n:
            raise IndexError("readerIndex out of bounds")
        v = self.b[self.i:self.i + n]
        self.i += n
        return v


def _decode_ping(r: _Reader):
    if r.readable() >= 4:
        length = r.take(">i")
        if length > 0 and r.readable() > 0:
            return r.bytes(length).decode("utf-8", errors="replace")     # new String(bytes)
    return None


def _decode_flow(r: _Reader):
    if r.readable() >= 12:
        flow_id, count = r.take(">qi")
        prio = r.take(">b") != 0 if r.readable() >= 1 else False
        return flow_id, count, prio
    return None


def _decode_param_value(r: _Reader, params: List[TypedValue]) -> None:
    t = r.take(">b")
    if t == PARAM_TYPE_INTEGER:
        params.append(jint(r.take(">i")))
    elif t == PARAM_TYPE_STRING:
        params.append(jstr(r.bytes(r.take(">i")).decode("utf-8", errors="replace")))
    elif t == PARAM_TYPE_BOOLEAN:
        params.append(jbool(r.take(">b") != 0))
    elif t == PARAM_TYPE_DOUBLE:
        params.append(jdouble(r.take(">d")))
    elif t == PARAM_TYPE_LONG:
        params.append(jlong(r.take(">q")))
    elif t == PARAM_TYPE_FLOAT:
        params.append(jfloat(r.take(">f")))
    elif t == PARAM_TYPE_BYTE:
        params.append(jbyte(r.take(">b")))
    elif t == PARAM_TYPE_SHORT:
        params.append(jshort(r.take(">h")))
    # unknown type: only its type byte was consumed (ParamFlowRequestDataDecoder.java:86-88)


def _decode_param(r: _Reader):
    if r.readable() >= 16:
        flow_id, count, amount = r.take(">qii")
        if amount > 0:
            params: List[TypedValue] = []
            for _ in range(amount):
                _decode_param_value(r, params)
            return flow_id, count, params
    return None


_DECODERS = {MSG_TYPE_PING: _decode_ping, MSG_TYPE_FLOW: _decode_flow, MSG_TYPE_PARAM_FLOW: _decode_param}


def decode_request(body: bytes) -> Optional[Request]:
    """DefaultRequestEntityDecoder.decode: None when nothing is emitted (short header, unknown type,
    or a decoder running out of bytes -- Netty raises, the handler never sees a request)."""
    if len(body) < 5:
        return None
    xid, typ = struct.unpack_from(">ib", body, 0)
    dec = _DECODERS.get(typ)
    if dec is None:
        return None
    r = _Reader(body[5:])
    if r.readable() == 0:
        return Request(xid, typ, None)
    try:
        return Request(xid, typ, dec(r))
    except IndexError:
        return None


def encode_response(xid: int, typ: int, status: int, data=None) -> bytes:
    """DefaultResponseEntityWriter + LengthFieldPrepender(2)."""
    if typ in (MSG_TYPE_FLOW, MSG_TYPE_PARAM_FLOW):
        body = struct.pack(">ibb", xid, typ, status) + (struct.pack(">ii", *data) if data is not None else b"")
    elif typ == MSG_TYPE_PING:
        body = struct.pack(">ibb", xid, typ, status) + (struct.pack(">i", data) if data is not None else b"")
    else:
        body = struct.pack(">ibb", xid, typ, RESPONSE_STATUS_BAD)
    return struct.pack(">H", len(body)) + body


def _frame(body: bytes) -> bytes:
    return struct.pack(">H", len(body)) + body


def encode_flow_request(xid: int, flow_id: int, count: int, prio: bool = False) -> bytes:
    """Client FlowRequestDataWriter layout: [i64 flowId][i32 count][bool prio]."""
    return _frame(struct.pack(">ibqib", xid, MSG_TYPE_FLOW, flow_id, count, 1 if prio else 0))


def _param_transport_size(v: TypedValue) -> int:
    """ParamFlowRequestDataWriter.calculateParamTransportSize."""
    return {PARAM_TYPE_INTEGER: 5, PARAM_TYPE_BOOLEAN: 2, PARAM_TYPE_LONG: 9, PARAM_TYPE_DOUBLE: 9,
            PARAM_TYPE_FLOAT: 5, PARAM_TYPE_BYTE: 2, PARAM_TYPE_SHORT: 3}.get(
        v.tag, 5 + len(str(v.value).encode("utf-8")) if v.tag == PARAM_TYPE_STRING else 0)


def resolve_valid_params(params: Sequence[TypedValue], max_size: int = DEFAULT_PARAM_MAX_SIZE) -> List[TypedValue]:
    """ParamFlowRequestDataWriter.resolveValidParams: drop unsupported values, stop at the byte cap."""
    out, size = [], 0
    for p in params:
        s = _param_transport_size(p) if isinstance(p, TypedValue) else 0
        if s <= 0:
            continue
        if size + s > max_size:
            break
        size += s
        out.append(p)
    return out


def _encode_value(v: TypedValue) -> bytes:
    t = v.tag
    if t == PARAM_TYPE_INTEGER:
        return struct.pack(">bi", t, v.value)
    if t == PARAM_TYPE_STRING:
        b = str(v.value).encode("utf-8")
        return struct.pack(">bi", t, len(b)) + b
    if t == PARAM_TYPE_BOOLEAN:
        return struct.pack(">bb", t, 1 if v.value else 0)
    if t == PARAM_TYPE_LONG:
        return struct.pack(">bq", t, v.value)
    if t == PARAM_TYPE_DOUBLE:
        return struct.pack(">bQ", t, v.value)
    if t == PARAM_TYPE_FLOAT:
        return struct.pack(">bI", t, v.value)
    if t == PARAM_TYPE_BYTE:
        return struct.pack(">bb", t, v.value)
    if t == PARAM_TYPE_SHORT:
        return struct.pack(">bh", t, v.value)
    return b""


def encode_param_request(xid: int, flow_id: int, count: int, params: Sequence[TypedValue],
                         max_size: int = DEFAULT_PARAM_MAX_SIZE) -> bytes:
    """Client ParamFlowRequestDataWriter layout."""
    ps = resolve_valid_params(params, max_size)
    body = struct.pack(">ibqii", xid, MSG_TYPE_PARAM_FLOW, flow_id, count, len(ps)) + b"".join(_encode_value(p) for p in ps)
    return _frame(body)


def encode_ping(xid: int, namespace: str) -> bytes:
    b = namespace.encode("utf-8")
    return _frame(struct.pack(">ibi", xid, MSG_TYPE_PING, len(b)) + b)


def decode_response(body: bytes):
    """(xid, type, status, data): data (remaining, wait) for flow/param, connectedCount for ping."""
    xid, typ, status = struct.unpack_from(">ibb", body, 0)
    rest = body[6:]
    data = None
    if typ in (MSG_TYPE_FLOW, MSG_TYPE_PARAM_FLOW) and len(rest) >= 8:
        data = struct.unpack_from(">ii", rest, 0)
    elif typ == MSG_TYPE_PING and len(rest) >= 4:
        data = struct.unpack_from(">i", rest, 0)[0]
    return xid, typ, status, data


class ParamKeyInterner:
    """Injective (flowId, Java-typed value) -> 64-bit engine param key: dense ids from 1, so the
    reserved all-ones key never appears.  Host rules (hot items) and requests share one interner."""

    def __init__(self):
        self._ids: Dict[Tuple[int, TypedValue], int] = {}
        self._lock = threading.Lock()

    def key(self, flow_id: int, value: TypedValue) -> int:
        k = (int(flow_id), value)
        with self._lock:
            v = self._ids.get(k)
            if v is None:
                v = len(self._ids) + 1
                self._ids[k] = v
        return v


# ------------------------------------------------------------------ server

@dataclass
class _Pending:
    conn: "_Conn"
    req: Request
    ts: int


class _Conn(asyncio.Protocol):
    def __init__(self, server: "ClusterTokenServer"):
        self.server = server
        self.frames = FrameDecoder()
        self.transport = None
        self.address = None

    def connection_made(self, transport):
        self.transport = transport
        peer = transport.get_extra_info("peername")
        self.address = f"{peer[0]}:{peer[1]}" if peer else None

    def data_received(self, data: bytes):
        for body in self.frames.feed(data):
            req = decode_request(body)
            if req is not None:
                self.server._enqueue(self, req)

    def connection_lost(self, exc):
        self.server._connection_lost(self)


class ClusterTokenServer:
    """NettyTransportServer + TokenServerHandler over one GpuTokenService (one GPU shard).

    `namespaces` names the engine's namespace table (the order given to svc.set_namespaces);
    PINGs of those namespaces update connectedCount in the engine.  `clock()` returns the
    TimeUtil.currentTimeMillis() stamped on each request when it is decoded."""

    def __init__(self, svc: GpuTokenService, namespaces: Sequence[str] = ("default",), host: str = "127.0.0.1",
                 port: int = 0, max_batch: int = 65536, max_wait_ms: float = 0.2,
                 clock: Optional[Callable[[], int]] = None, interner: Optional[ParamKeyInterner] = None,
                 record: bool = False):
        self.svc = svc
        self.ns_index = {n: i for i, n in enumerate(namespaces)}
        self.host, self.port = host, port
        self.max_batch, self.max_wait = max_batch, max_wait_ms / 1000.0
        self.clock = clock or (lambda: int(time.time() * 1000))
        self.interner = interner or ParamKeyInterner()
        self.record = record
        self.log: List[tuple] = []          # (kind, payload, ts) in decision order when record=True
        self.connections: Dict[str, set] = {}
        self._conn_lock = threading.Lock()
        self._pending: List[_Pending] = []
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._thread: Optional[threading.Thread] = None
        self._ready = threading.Event()
        self._wake: Optional[asyncio.Event] = None
        self._stopping = False
        self.batches = 0

    # -- lifecycle
    def start(self) -> int:
        self._thread = threading.Thread(target=self._run, name="sentinel-token-server", daemon=True)
        self._thread.start()
        if not self._ready.wait(30):
            raise RuntimeError("token server did not start")
        return self.port

    def stop(self):
        if self._loop is None:
            return
        self._stopping = True
        self._loop.call_soon_threadsafe(self._shutdown)
        self._thread.join(30)

    def _run(self):
        self._loop = asyncio.new_event_loop()
        asyncio.set_event_loop(self._loop)
        self._wake = asyncio.Event()
        srv = self._loop.run_until_complete(self._loop.create_server(lambda: _Conn(self), self.host, self.port))
        self.port = srv.sockets[0].getsockname()[1]
        self._server = srv
        self._dispatcher = self._loop.create_task(self._dispatch())
        self._ready.set()
        self._loop.run_forever()
        self._loop.run_until_complete(asyncio.gather(self._dispatcher, return_exceptions=True))
        self._loop.close()

    def _shutdown(self):
        self._server.close()
        self._dispatcher.cancel()
        self._loop.stop()

    # -- event loop side
    def _enqueue(self, conn: _Conn, req: Request):
        self._pending.append(_Pending(conn, req, int(self.clock())))
        if len(self._pending) == 1 or len(self._pending) >= self.max_batch:
            self._wake.set()

    def _connection_lost(self, conn: _Conn):
        with self._conn_lock:
            for ns, addrs in self.connections.items():    # ConnectionManager.removeConnection
                if conn.address in addrs:
                    addrs.discard(conn.address)
                    self._set_connected(ns)
                    if self.record:
                        self.log.append(("disconnect", ns, int(self.clock())))

    def _set_connected(self, ns: str):
        i = self.ns_index.get(ns)
        if i is not None:
            self.svc.set_connected_count(i, len(self.connections.get(ns, ())))

    async def _dispatch(self):
        while True:
            await self._wake.wait()
            self._wake.clear()
            if len(self._pending) < self.max_batch and self.max_wait > 0:
                await asyncio.sleep(self.max_wait)
            while self._pending:
                take, self._pending = self._pending[:self.max_batch], self._pending[self.max_batch:]
                replies = await self._loop.run_in_executor(None, self._decide, take)
                for conn, frame in replies:
                    if conn.transport is not None and not conn.transport.is_closing():
                        conn.transport.write(frame)

    # -- dispatcher side (worker thread): runs of one kind -> one GPU batch each
    def _decide(self, items: List[_Pending]):
        out = []
        i = 0
        while i < len(items):
            typ = items[i].req.type
            j = i
            while j < len(items) and items[j].req.type == typ:
                j += 1
            run = items[i:j]
            if typ == MSG_TYPE_PING:
                out.extend(self._ping(p) for p in run)
            else:
                ok = [p for p in run if p.req.data is not None]      # null data: processor NPE, no reply
                if ok:
                    out.extend(self._flow(ok) if typ == MSG_TYPE_FLOW else self._param(ok))
            i = j
        self.batches += 1
        return out

    def _ping(self, p: _Pending):
        ns = p.req.data
        if ns is None or ns.strip() == "":
            return p.conn, encode_response(p.req.xid, MSG_TYPE_PING, RESPONSE_STATUS_BAD)
        with self._conn_lock:
            self.connections.setdefault(ns, set()).add(p.conn.address)   # ConnectionManager.addConnection
            self._set_connected(ns)
            count = len(self.connections[ns])
        if self.record:
            self.log.append(("ping", ns, p.ts))
        return p.conn, encode_response(p.req.xid, MSG_TYPE_PING, RESPONSE_STATUS_OK, count)

    def _flow(self, run: List[_Pending]):
        ids = np.array([p.req.data[0] for p in run], dtype=np.int64)
        idx = self.svc.lookup_flow_idx(ids)
        acq = np.array([p.req.data[1] for p in run], dtype=np.int32)
        prio = np.array([1 if p.req.data[2] else 0 for p in run], dtype=np.uint8)
        ts = np.array([p.ts for p in run], dtype=np.int64)
        st, rem, wait = self.svc.submit_flow_batch_host(idx, acq, ts, prio)
        if self.record:
            self.log.append(("flow", (idx, acq, prio), ts))
        return [(p.conn, encode_response(p.req.xid, MSG_TYPE_FLOW, int(st[k]), (int(rem[k]), int(wait[k]))))
                for k, p in enumerate(run)]

    def _param(self, run: List[_Pending]):
        ids = np.array([p.req.data[0] for p in run], dtype=np.int64)
        idx = self.svc.lookup_param_idx(ids)
        acq = np.array([p.req.data[1] for p in run], dtype=np.int32)
        ts = np.array([p.ts for p in run], dtype=np.int64)
        cnt = np.array([len(p.req.data[2]) for p in run], dtype=np.int32)
        begin = np.zeros(len(run), dtype=np.int32)
        begin[1:] = np.cumsum(cnt)[:-1]
        keys = np.array([self.interner.key(p.req.data[0], v) for p in run for v in p.req.data[2]], dtype=np.uint64)
        st, rem = self.svc.submit_param_multi_batch_host(idx, acq, ts, begin, cnt, keys)
        if self.record:
            self.log.append(("param", (idx, acq, begin, cnt, keys), ts))
        return [(p.conn, encode_response(p.req.xid, MSG_TYPE_PARAM_FLOW, int(st[k]), (int(rem[k]), 0)))
                for k, p in enumerate(run)]


class TokenClient:
    """Blocking client speaking the reference's client wire format (NettyTransportClient codecs)."""

    def __init__(self, host: str, port: int, timeout: float = 10.0):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.frames = FrameDecoder()
        self.ready: List[bytes] = []

    def send(self, frame: bytes):
        self.sock.sendall(frame)

    def recv(self):
        while not self.ready:
            data = self.sock.recv(65536)
            if not data:
                raise ConnectionError("server closed the connection")
            self.ready.extend(self.frames.feed(data))
        return decode_response(self.ready.pop(0))

    def close(self):
        self.sock.close()


# ------------------------------------------------------------------ native server (C++ behind the ABI)

def _value_bytes(v: TypedValue) -> bytes:
    """A value's wire bytes after its type byte (string: the UTF-8 bytes, no length)."""
    if v.tag == PARAM_TYPE_STRING:
        return str(v.value).encode("utf-8")
    return _encode_value(v)[1:]


class NativeParamInterner:
    """sentinel_param_interner_*: the native server's (flowId, Java-typed value) -> key table."""

    def __init__(self):
        from . import _lib
        import ctypes as C
        self._L = _lib.load()
        h = C.c_void_p()
        _lib.check(self._L.sentinel_param_interner_create(C.byref(h)), "param_interner_create")
        self.handle = h

    def key(self, flow_id: int, value: TypedValue, ts: Optional[int] = None) -> int:
        """The value's key; `ts` (ms) is the request time that last used it (None: no aging)."""
        from . import _lib
        import ctypes as C
        b = _value_bytes(value)
        k = C.c_uint64()
        buf = C.create_string_buffer(b, len(b)) if b else None
        t = -(1 << 63) if ts is None else int(ts)
        _lib.check(self._L.sentinel_param_interner_key_at(self.handle, int(flow_id), int(value.tag), buf, len(b), t,
                                                          C.byref(k)), "param_interner_key")
        return int(k.value)

    def set_limits(self, max_entries: int, idle_ms: int):
        from . import _lib
        _lib.check(self._L.sentinel_param_interner_set_limits(self.handle, int(max_entries), int(idle_ms)),
                   "param_interner_set_limits")

    def stats(self):
        import ctypes as C
        n, ev = C.c_int64(), C.c_int64()
        sc = C.c_int64()
        self._L.sentinel_param_interner_stats(self.handle, C.byref(n), C.byref(ev))
        self._L.sentinel_param_interner_scans(self.handle, C.byref(sc))
        return {"entries": n.value, "evicted": ev.value, "scans": sc.value}

    def close(self):
        if self.handle:
            self._L.sentinel_param_interner_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class NativeTokenServer:
    """sentinel_wire_server_*: the same protocol and handling as ClusterTokenServer, in C++ (epoll
    I/O threads, one batcher call per socket read, one flush per decided batch).  `clock()`, when
    given, replaces the wall clock (it is called from the I/O threads)."""

    def __init__(self, svc: GpuTokenService, namespaces: Sequence[str] = ("default",), host: str = "127.0.0.1",
                 port: int = 0, io_threads: int = 2, max_batch: int = 4096, max_wait_us: int = 20,
                 clock: Optional[Callable[[], int]] = None, interner: Optional[NativeParamInterner] = None):
        from . import _lib
        import ctypes as C
        self._L = _lib.load()
        self.svc = svc
        self._names = (C.c_char_p * max(len(namespaces), 1))(*[n.encode() for n in namespaces])
        self._clock = _lib.CLOCK_FN(lambda _ctx: int(clock())) if clock else _lib.CLOCK_FN()
        cfg = _lib.WireConfig(host.encode(), int(port), int(io_threads), int(max_batch), int(max_wait_us),
                              self._names, len(namespaces), interner.handle if interner else None, self._clock, None)
        h = C.c_void_p()
        self.handle = None
        self.interner = interner         # kept alive as long as the server may use it
        _lib.check(self._L.sentinel_wire_server_create(svc.handle, C.byref(cfg), C.byref(h)), "wire_server_create")
        self.handle = h
        self.port = int(self._L.sentinel_wire_server_port(h))
        svc._attach_server(self)         # the service keeps the server and stops it before it closes

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()

    def __del__(self):
        try:
            self.stop()
        except Exception:
            pass

    def stats(self):
        import ctypes as C
        f, p, b, c = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int32()
        self._L.sentinel_wire_server_stats(self.handle, C.byref(f), C.byref(p), C.byref(b), C.byref(c))
        return {"flow_requests": f.value, "param_requests": p.value, "batches": b.value, "connections": c.value}

    def stop(self):
        if self.handle:
            self._L.sentinel_wire_server_destroy(self.handle)
            self.handle = None
