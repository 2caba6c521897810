"""Host-side mirror of Sentinel's cluster TokenService SPI over the MI355X engine.

Mirrors (paths relative to the reference repo):
  TokenService        sentinel-core/src/main/java/com/alibaba/csp/sentinel/cluster/TokenService.java:26-63
  TokenResult         sentinel-core/src/main/java/com/alibaba/csp/sentinel/cluster/TokenResult.java:26-98
  TokenResultStatus   sentinel-core/src/main/java/com/alibaba/csp/sentinel/cluster/TokenResultStatus.java:22-73
  ClusterFlowConfig   sentinel-core/src/main/java/com/alibaba/csp/sentinel/slots/block/flow/ClusterFlowConfig.java:39-51
  DefaultTokenService sentinel-cluster/sentinel-cluster-server-default/.../cluster/flow/DefaultTokenService.java:37-62

The per-call methods (request_token / request_param_token) keep the reference's names, argument
meaning and error convention (status codes, never exceptions for bad input).  The batched methods
(submit_*) are the hot path: one call decides a whole batch of events on the GPU.
"""
from __future__ import annotations

import atexit
import ctypes as C
import time
import weakref
from dataclasses import dataclass, field
from typing import Iterable, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import SentinelError, check


class TokenResultStatus:
    BAD_REQUEST = -4
    TOO_MANY_REQUEST = -2
    FAIL = -1
    OK = 0
    BLOCKED = 1
    SHOULD_WAIT = 2
    NO_RULE_EXISTS = 3
    NO_REF_RULE_EXISTS = 4
    NOT_AVAILABLE = 5
    RELEASE_OK = 6
    ALREADY_RELEASE = 7


class ClusterRuleConstant:
    FLOW_THRESHOLD_AVG_LOCAL = 0
    FLOW_THRESHOLD_GLOBAL = 1
    DEFAULT_CLUSTER_SAMPLE_COUNT = 10


@dataclass
class TokenResult:
    status: int
    remaining: int = 0
    wait_in_ms: int = 0
    token_id: int = 0


@dataclass
class ClusterFlowConfig:
    flow_id: Optional[int] = None
    threshold_type: int = ClusterRuleConstant.FLOW_THRESHOLD_AVG_LOCAL
    sample_count: int = ClusterRuleConstant.DEFAULT_CLUSTER_SAMPLE_COUNT
    window_interval_ms: int = 1000
    fallback_to_local_when_fail: bool = True


@dataclass
class FlowRule:
    """Cluster-mode FlowRule (only the fields the cluster checkers read)."""
    resource: str = ""
    count: float = 0.0
    cluster_mode: bool = True
    cluster_config: ClusterFlowConfig = field(default_factory=ClusterFlowConfig)
    namespace: int = 0                 # index into the server namespace set
    checker: int = _lib.CHECKER_CLUSTER


@dataclass
class ParamFlowRule:
    resource: str = ""
    count: float = 0.0
    cluster_config: ClusterFlowConfig = field(default_factory=ClusterFlowConfig)
    namespace: int = 0
    hot_items: dict = field(default_factory=dict)   # param key -> int count


@dataclass
class LocalParamRule:
    """Local ParamFlowRule as passDefaultLocalCheck reads it (QPS grade, default behaviour)."""
    count: float = 0.0
    burst_count: int = 0
    duration_in_sec: int = 1
    hot_items: dict = field(default_factory=dict)   # param key -> int count


@dataclass
class ServerNamespace:
    connected_count: int = 0
    has_limiter: bool = False
    max_allowed_qps: float = 30000.0   # ServerFlowConfig.DEFAULT_MAX_ALLOWED_QPS


# Engines and batchers still alive at interpreter exit are closed by an atexit hook (batchers
# first), while the HIP runtime is still up; finalizers of module globals would run too late.
_LIVE_BATCHERS: "weakref.WeakSet" = weakref.WeakSet()
_LIVE_ENGINES: "weakref.WeakSet" = weakref.WeakSet()


@atexit.register
def _close_all():
    for group in (_LIVE_BATCHERS, _LIVE_ENGINES):
        for obj in list(group):
            try:
                obj.close()
            except Exception:
                pass


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def _now_ms() -> int:
    return int(time.time() * 1000)


class GpuTokenService:
    """TokenService implemented on one MI355X (one shard of the flowId space)."""

    def __init__(self, device: int = 0, exceed_count: float = 1.0, max_occupy_ratio: float = 1.0,
                 namespaces: Optional[Sequence[ServerNamespace]] = None):
        self._L = _lib.load()
        self._h = C.c_void_p()
        cfg = _lib.ServerConfig(exceed_count, max_occupy_ratio)
        check(self._L.sentinel_engine_create(device, C.byref(cfg), C.byref(self._h)), "sentinel_engine_create")
        _LIVE_ENGINES.add(self)
        self.device = device
        self.sample_counts = {}
        self._flow_rules = []
        self._servers = weakref.WeakSet()    # native wire servers running on this engine
        if namespaces is not None:
            self.set_namespaces(namespaces)

    def _attach_server(self, srv):
        self._servers.add(srv)

    def close(self):
        """Destroys the engine; native wire servers still running on it are stopped first (their I/O
        and dispatcher threads hold the engine pointer)."""
        for srv in list(getattr(self, "_servers", ())):
            srv.stop()
        if getattr(self, "_h", None) and self._h.value:
            self._L.sentinel_engine_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    @property
    def stream(self) -> int:
        return int(self._L.sentinel_engine_stream(self._h) or 0)

    # ---------------------------------------------------------------- config
    def set_server_config(self, exceed_count=1.0, max_occupy_ratio=1.0):
        cfg = _lib.ServerConfig(exceed_count, max_occupy_ratio)
        check(self._L.sentinel_set_server_config(self._h, C.byref(cfg)), "set_server_config")

    def set_namespaces(self, namespaces: Sequence[ServerNamespace]):
        arr = (_lib.Namespace * max(len(namespaces), 1))()
        for i, ns in enumerate(namespaces):
            arr[i] = _lib.Namespace(int(ns.connected_count), int(bool(ns.has_limiter)), float(ns.max_allowed_qps))
        check(self._L.sentinel_set_namespaces(self._h, arr, len(namespaces)), "set_namespaces")

    def set_connected_count(self, namespace: int, connected: int):
        check(self._L.sentinel_set_connected_count(self._h, namespace, connected), "set_connected_count")

    def load_flow_rules(self, rules: Sequence[FlowRule]):
        """ClusterFlowRuleManager.loadRules for the server (ClusterFlowRuleManager.java:325-372)."""
        arr = (_lib.FlowRuleC * max(len(rules), 1))()
        for i, r in enumerate(rules):
            cc = r.cluster_config
            fid = cc.flow_id if cc.flow_id is not None else 0
            arr[i] = _lib.FlowRuleC(int(fid), float(r.count), int(cc.threshold_type), int(cc.sample_count),
                                    int(cc.window_interval_ms), int(r.namespace), int(r.checker), 0)
        check(self._L.sentinel_load_flow_rules(self._h, arr, len(rules)), "load_flow_rules")
        self._flow_rules = list(rules)

    def load_rules_array(self, flow_ids, counts, threshold_type=1, sample_count=10, window_interval_ms=1000,
                         namespace=0, checker=0):
        """Vectorised rule load for large synthetic tables (1M flows)."""
        n = len(flow_ids)
        rec = np.zeros(n, dtype=[("flow_id", "<i8"), ("count", "<f8"), ("threshold_type", "<i4"),
                                 ("sample_count", "<i4"), ("window_interval_ms", "<i4"),
                                 ("namespace_idx", "<i4"), ("checker", "<i4"), ("reserved", "<i4")])
        rec["flow_id"] = flow_ids
        rec["count"] = counts
        rec["threshold_type"] = threshold_type
        rec["sample_count"] = sample_count
        rec["window_interval_ms"] = window_interval_ms
        rec["namespace_idx"] = namespace
        rec["checker"] = checker
        check(self._L.sentinel_load_flow_rules(self._h, C.c_void_p(rec.ctypes.data), n), "load_flow_rules")

    def load_param_rules(self, rules: Sequence[ParamFlowRule]):
        arr = (_lib.ParamRuleC * max(len(rules), 1))()
        keys, counts = [], []
        for i, r in enumerate(rules):
            cc = r.cluster_config
            fid = cc.flow_id if cc.flow_id is not None else 0
            arr[i] = _lib.ParamRuleC(int(fid), float(r.count), int(cc.threshold_type), int(cc.sample_count),
                                     int(cc.window_interval_ms), int(r.namespace), len(keys), len(r.hot_items))
            for k, c in r.hot_items.items():
                keys.append(k)
                counts.append(c)
        hk = np.array(keys or [0], dtype=np.uint64)
        hc = np.array(counts or [0], dtype=np.int32)
        check(self._L.sentinel_load_param_rules(self._h, arr, len(rules), _p(hk), _p(hc), len(keys)),
              "load_param_rules")


    def flow_count(self) -> int:
        return int(self._L.sentinel_flow_count(self._h))

    def param_count(self) -> int:
        """Dense param rules loaded (valid, one per flowId)."""
        return int(self._L.sentinel_param_count(self._h))

    def lookup_flow_idx(self, flow_ids) -> np.ndarray:
        ids = np.ascontiguousarray(flow_ids, dtype=np.int64)
        out = np.empty(len(ids), dtype=np.int32)
        check(self._L.sentinel_lookup_flow_idx(self._h, len(ids), _p(ids), _p(out)), "lookup_flow_idx")
        return out

    def lookup_param_idx(self, flow_ids) -> np.ndarray:
        ids = np.ascontiguousarray(flow_ids, dtype=np.int64)
        out = np.empty(len(ids), dtype=np.int32)
        check(self._L.sentinel_lookup_param_idx(self._h, len(ids), _p(ids), _p(out)), "lookup_param_idx")
        return out

    # ---------------------------------------------------------------- TokenService (per call)
    def request_token(self, rule_id: Optional[int], acquire_count: int, prioritized: bool,
                      ts: Optional[int] = None) -> TokenResult:
        """TokenService.requestToken (TokenService.java:36)."""
        out = _lib.TokenResultC()
        fid = 0 if rule_id is None else int(rule_id)
        rc = self._L.sentinel_request_token(self._h, fid, int(acquire_count), int(bool(prioritized)),
                                            _now_ms() if ts is None else int(ts), C.byref(out))
        check(rc, "request_token")
        return TokenResult(out.status, out.remaining, out.wait_in_ms)

    def request_param_token(self, rule_id: Optional[int], acquire_count: int, params: Iterable[int],
                            ts: Optional[int] = None) -> TokenResult:
        """TokenService.requestParamToken (TokenService.java:46) for one parameter value.  Values are
        64-bit param keys (the host's injective encoding of the Java typed value)."""
        params = list(params) if params is not None else []
        if rule_id is None or int(rule_id) <= 0 or acquire_count <= 0 or not params:
            return TokenResult(TokenResultStatus.BAD_REQUEST)       # DefaultTokenService.java:53-55
        if len(params) != 1:   # ClusterParamFlowChecker over the whole value list (CPFC:58-86)
            idx = int(self.lookup_param_idx([int(rule_id)])[0])
            st, rem = self.submit_param_multi_batch_host(
                np.array([idx], np.int32), np.array([acquire_count], np.int32),
                np.array([_now_ms() if ts is None else int(ts)], np.int64), np.array([0], np.int32),
                np.array([len(params)], np.int32), np.array(params, dtype=np.uint64))
            return TokenResult(int(st[0]), int(rem[0]), 0)
        out = _lib.TokenResultC()
        check(self._L.sentinel_request_param_token(self._h, int(rule_id), int(acquire_count), int(params[0]),
                                                   _now_ms() if ts is None else int(ts), C.byref(out)),
              "request_param_token")
        return TokenResult(out.status, out.remaining, out.wait_in_ms)

    def request_concurrent_token(self, client_address: Optional[str], rule_id: Optional[int],
                                 acquire_count: int) -> TokenResult:
        """TokenService.requestConcurrentToken (TokenService.java:56): OK carries the token id."""
        fid = 0 if rule_id is None else int(rule_id)
        idx = int(self.lookup_flow_idx([fid])[0])
        st, tok = self.submit_concurrent_batch_host([idx], [acquire_count], [0], [_lib.CONCURRENT_ACQUIRE],
                                                    [1 if client_address else 0])
        return TokenResult(int(st[0]), token_id=int(tok[0]))

    def release_concurrent_token(self, token_id: Optional[int]) -> Optional[TokenResult]:
        """TokenService.releaseConcurrentToken (TokenService.java:62); returns the checker's status
        (RELEASE_OK / ALREADY_RELEASE / NO_RULE_EXISTS), None for a null token like the reference."""
        if token_id is None:
            return None
        st, _ = self.submit_concurrent_batch_host([0], [0], [int(token_id)], [_lib.CONCURRENT_RELEASE], [0])
        return TokenResult(int(st[0]))

    def submit_concurrent_batch_host(self, flow_idx, acquire, token_id, kind, flags):
        """A batch of concurrent acquires / releases in arrival order -> (status, token_id) arrays."""
        ev = np.empty(len(kind), dtype=_lib.CONC_EVENT_DTYPE)
        ev["flow_idx"], ev["acquire"], ev["token_id"], ev["kind"], ev["flags"] = flow_idx, acquire, token_id, kind, flags
        out = np.empty(len(ev), dtype=_lib.CONC_RESULT_DTYPE)
        check(self._L.sentinel_submit_concurrent_batch_host(self._h, len(ev), _p(ev), _p(out)),
              "submit_concurrent_batch_host")
        return out["status"].astype(np.int8), out["token_id"].copy()

    def submit_concurrent_batch(self, events, results=None, stream=None):
        """Concurrency-token acquires / releases on device tensors (sentinel_submit_concurrent_batch):
        `events` int64 (n, 3) of sentinel_concurrent_event_t records (word0 = acquire << 32 | flow_idx,
        word1 = token_id, word2 = flags << 32 | kind); `results` int64 (n, 2) of
        sentinel_concurrent_result_t ({token_id, status}).  Asynchronous on `stream`."""
        import torch
        n = int(events.shape[0])
        if results is None:
            results = torch.empty((n, 2), dtype=torch.int64, device=events.device)
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        check(self._L.sentinel_submit_concurrent_batch(self._h, n, C.c_void_p(events.data_ptr()),
                                                       C.c_void_p(results.data_ptr()),
                                                       None if s is None else C.c_void_p(s)),
              "submit_concurrent_batch")
        return results

    @staticmethod
    def concurrent_events(flow_idx, acquire, token_id, kind, flags):
        """(n, 3) int64 device tensor of sentinel_concurrent_event_t from torch tensors."""
        import torch
        w0 = (acquire.to(torch.int64) << 32) | (flow_idx.to(torch.int64) & 0xFFFFFFFF)
        w2 = (flags.to(torch.int64) << 32) | (kind.to(torch.int64) & 0xFFFFFFFF)
        return torch.stack([w0, token_id.to(torch.int64), w2], dim=1).contiguous()

    def concurrent_now_calls(self, flow_idx: int) -> int:
        v = C.c_int32()
        check(self._L.sentinel_concurrent_now_calls(self._h, int(flow_idx), C.byref(v)), "concurrent_now_calls")
        return v.value

    def concurrent_token_count(self) -> int:
        v = C.c_int64()
        check(self._L.sentinel_concurrent_token_count(self._h, C.byref(v)), "concurrent_token_count")
        return v.value

    def concurrent_expire(self, max_tokens: int = 1000) -> int:
        """One RegularExpireStrategy sweep (executeCount 1000 by default)."""
        v = C.c_int64()
        check(self._L.sentinel_concurrent_expire(self._h, int(max_tokens), C.byref(v)), "concurrent_expire")
        return v.value

    # ---------------------------------------------------------------- batched hot path
    @staticmethod
    def pack_events(flow_idx, acquire, ts) -> np.ndarray:
        ev = np.empty(len(ts), dtype=_lib.EVENT_DTYPE)
        ev["flow_idx"] = flow_idx
        ev["acquire"] = acquire
        ev["ts"] = ts
        return ev

    @staticmethod
    def pack_param_events(rule_idx, acquire, param_key, ts) -> np.ndarray:
        ev = np.empty(len(ts), dtype=_lib.PARAM_EVENT_DTYPE)
        ev["rule_idx"] = rule_idx
        ev["acquire"] = acquire
        ev["ts"] = ts
        ev["param_key"] = param_key
        return ev

    def submit_flow_batch(self, events, flags=None, verdicts=None, stream=None):
        """Decide a batch of device-resident events.  `events` is a torch int64 tensor of shape
        (n, 2) holding sentinel_event_t records (word0 = acquire << 32 | flow_idx, word1 = ts);
        verdicts is an int64 tensor (n,) of packed sentinel_verdict_t.  Asynchronous on `stream`
        (torch stream or raw hipStream_t; default the engine stream)."""
        import torch
        n = int(events.shape[0])
        if verdicts is None:
            verdicts = torch.empty(n, dtype=torch.int64, device=events.device)
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        rc = self._L.sentinel_submit_flow_batch(
            self._h, n, C.c_void_p(events.data_ptr()), None if flags is None else C.c_void_p(flags.data_ptr()),
            C.c_void_p(verdicts.data_ptr()), None if s is None else C.c_void_p(s))
        check(rc, "submit_flow_batch")
        return verdicts

    def submit_flow_batch_ordered(self, events, flags=None, verdicts=None, seq=None, stream=None):
        """submit_flow_batch with decide-order output (sentinel_submit_flow_batch_ordered): returns
        (verdicts, seq), int64 (n,) and int32 (n,) device tensors; verdicts[j] answers the event at arrival
        position seq[j].  Asynchronous on `stream`."""
        import torch
        n = int(events.shape[0])
        if verdicts is None:
            verdicts = torch.empty(n, dtype=torch.int64, device=events.device)
        if seq is None:
            seq = torch.empty(n, dtype=torch.int32, device=events.device)
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        rc = self._L.sentinel_submit_flow_batch_ordered(
            self._h, n, C.c_void_p(events.data_ptr()), None if flags is None else C.c_void_p(flags.data_ptr()),
            C.c_void_p(verdicts.data_ptr()), C.c_void_p(seq.data_ptr()), None if s is None else C.c_void_p(s))
        check(rc, "submit_flow_batch_ordered")
        return verdicts, seq

    def submit_flow_batch_ordered_host(self, flow_idx, acquire, ts, flags=None):
        """Host arrays in; (status, remaining, wait_in_ms, seq) numpy arrays out in decide order: entry j
        answers the event at arrival position seq[j] (synchronous)."""
        ev = self.pack_events(flow_idx, acquire, ts)
        flags = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint8)
        out = np.empty(len(ev), dtype=_lib.VERDICT_DTYPE)
        seq = np.empty(len(ev), dtype=np.uint32)
        check(self._L.sentinel_submit_flow_batch_ordered_host(self._h, len(ev), _p(ev), _p(flags), _p(out), _p(seq)),
              "submit_flow_batch_ordered_host")
        return out["status"].astype(np.int8), out["remaining"].copy(), out["wait_in_ms"].astype(np.int32), seq

    def submit_flow_batches(self, events_list, verdicts_list, flags_list=None, stream=None):
        """Device batches in order under one engine lock (sentinel_submit_flow_batches): each events tensor int64
        (n, 2) of sentinel_event_t, each verdict tensor int64 (n,)."""
        k = len(events_list)
        ns = (C.c_int64 * max(k, 1))(*[int(e.shape[0]) for e in events_list])
        evp = (C.c_void_p * max(k, 1))(*[e.data_ptr() for e in events_list])
        outp = (C.c_void_p * max(k, 1))(*[v.data_ptr() for v in verdicts_list])
        flp = None if flags_list is None else (C.c_void_p * max(k, 1))(*[f.data_ptr() for f in flags_list])
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        check(self._L.sentinel_submit_flow_batches(self._h, k, ns, evp, flp, outp, None if s is None else C.c_void_p(s)),
              "submit_flow_batches")
        return verdicts_list

    def set_flow_path(self, path: str):
        """Flow pipeline of the following batches: "auto", "sorted" (global radix sort),
        "partition" (partition-local) or "small" (one-launch chunks of 4096 events); verdicts are
        identical on every path."""
        check(self._L.sentinel_set_flow_path(self._h, {"auto": 0, "sorted": 1, "partition": 2, "small": 3}[path]),
              "sentinel_set_flow_path")

    def submit_flow_batch_host(self, flow_idx, acquire, ts, flags=None):
        """Host arrays in, (status, remaining, wait_in_ms) numpy arrays out (synchronous)."""
        ev = self.pack_events(flow_idx, acquire, ts)
        flags = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint8)
        out = np.empty(len(ev), dtype=_lib.VERDICT_DTYPE)
        check(self._L.sentinel_submit_flow_batch_host(self._h, len(ev), _p(ev), _p(flags), _p(out)),
              "submit_flow_batch_host")
        return out["status"].astype(np.int8), out["remaining"].copy(), out["wait_in_ms"].astype(np.int32)

    def submit_flow_stream_host(self, flow_idx, acquire, ts, flags=None, batch=1 << 20):
        """Like submit_flow_batch_host, pipelined in batches of `batch` events over side streams
        (H2D / decide / D2H overlap).  Returns (status, remaining, wait_in_ms, batch_ms)."""
        ev = self.pack_events(flow_idx, acquire, ts)
        flags = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint8)
        out = np.empty(len(ev), dtype=_lib.VERDICT_DTYPE)
        ms = np.zeros(max(1, -(-len(ev) // batch)), dtype=np.float32)
        check(self._L.sentinel_submit_flow_stream_host(self._h, len(ev), _p(ev), _p(flags), _p(out), batch, _p(ms)),
              "submit_flow_stream_host")
        return out["status"].astype(np.int8), out["remaining"].copy(), out["wait_in_ms"].astype(np.int32), ms

    def submit_param_batch(self, events, verdicts=None, stream=None):
        """events: torch int64 tensor (n, 3) of sentinel_param_event_t records."""
        import torch
        n = int(events.shape[0])
        if verdicts is None:
            verdicts = torch.empty(n, dtype=torch.int64, device=events.device)
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        check(self._L.sentinel_submit_param_batch(self._h, n, C.c_void_p(events.data_ptr()),
                                                  C.c_void_p(verdicts.data_ptr()), None if s is None else C.c_void_p(s)),
              "submit_param_batch")
        return verdicts

    def submit_param_batch_host(self, rule_idx, acquire, param_key, ts):
        ev = self.pack_param_events(rule_idx, acquire, param_key, ts)
        out = np.empty(len(ev), dtype=_lib.VERDICT_DTYPE)
        check(self._L.sentinel_submit_param_batch_host(self._h, len(ev), _p(ev), _p(out)), "submit_param_batch_host")
        return out["status"].astype(np.int8), out["remaining"].copy()

    def submit_param_batch_ordered(self, events, verdicts=None, seq=None, stream=None):
        """submit_param_batch with decide-order output (sentinel_submit_param_batch_ordered): returns
        (verdicts, seq) device tensors; verdicts[j] answers the request at arrival position seq[j]."""
        import torch
        n = int(events.shape[0])
        if verdicts is None:
            verdicts = torch.empty(n, dtype=torch.int64, device=events.device)
        if seq is None:
            seq = torch.empty(n, dtype=torch.int32, device=events.device)
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        check(self._L.sentinel_submit_param_batch_ordered(self._h, n, C.c_void_p(events.data_ptr()),
                                                          C.c_void_p(verdicts.data_ptr()), C.c_void_p(seq.data_ptr()),
                                                          None if s is None else C.c_void_p(s)),
              "submit_param_batch_ordered")
        return verdicts, seq

    def submit_param_batch_ordered_host(self, rule_idx, acquire, param_key, ts):
        """(status, remaining, seq) in decide order: entry j answers the request at arrival position seq[j]."""
        ev = self.pack_param_events(rule_idx, acquire, param_key, ts)
        out = np.empty(len(ev), dtype=_lib.VERDICT_DTYPE)
        seq = np.empty(len(ev), dtype=np.uint32)
        check(self._L.sentinel_submit_param_batch_ordered_host(self._h, len(ev), _p(ev), _p(out), _p(seq)),
              "submit_param_batch_ordered_host")
        return out["status"].astype(np.int8), out["remaining"].copy(), seq

    @staticmethod
    def pack_multi_events(rule_idx, acquire, ts, value_begin, value_count) -> np.ndarray:
        ev = np.empty(len(ts), dtype=_lib.MULTI_EVENT_DTYPE)
        ev["rule_idx"] = rule_idx
        ev["acquire"] = acquire
        ev["ts"] = ts
        ev["value_begin"] = value_begin
        ev["value_count"] = value_count
        return ev

    def submit_param_multi_batch_host(self, rule_idx, acquire, ts, value_begin, value_count, values):
        """requestParamToken with value lists (host arrays in, (status, remaining) out)."""
        ev = self.pack_multi_events(rule_idx, acquire, ts, value_begin, value_count)
        vals = np.ascontiguousarray(values, dtype=np.uint64)
        out = np.empty(len(ev), dtype=_lib.VERDICT_DTYPE)
        check(self._L.sentinel_submit_param_multi_batch_host(self._h, len(ev), _p(ev), _p(vals) if len(vals) else None,
                                                             len(vals), _p(out)), "submit_param_multi_batch_host")
        return out["status"].astype(np.int8), out["remaining"].copy()

    def submit_param_multi_batch(self, events, values, verdicts=None, stream=None):
        """Device tensors: events int64 (n, 3) of sentinel_param_multi_event_t, values uint64/int64 (m,)."""
        import torch
        n = int(events.shape[0])
        if verdicts is None:
            verdicts = torch.empty(n, dtype=torch.int64, device=events.device)
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        check(self._L.sentinel_submit_param_multi_batch(self._h, n, C.c_void_p(events.data_ptr()),
                                                        C.c_void_p(values.data_ptr()), int(values.shape[0]),
                                                        C.c_void_p(verdicts.data_ptr()), None if s is None else C.c_void_p(s)),
              "submit_param_multi_batch")
        return verdicts

    def set_param_mode(self, mode: int, depth: int = 4, width: int = 1024):
        """SENTINEL_PARAM_EXACT (0) or SENTINEL_PARAM_COUNT_MIN (1); clears the param counters."""
        check(self._L.sentinel_set_param_mode(self._h, int(mode), int(depth), int(width)), "set_param_mode")

    def load_local_param_rules(self, rules: Sequence[LocalParamRule]):
        """Local ParamFlowRules (index = position); every token bucket restarts."""
        arr = (_lib.LocalParamRuleC * max(len(rules), 1))()
        keys, counts = [], []
        for i, r in enumerate(rules):
            arr[i] = _lib.LocalParamRuleC(float(r.count), int(r.burst_count), int(r.duration_in_sec), len(keys),
                                          len(r.hot_items))
            for k, c in r.hot_items.items():
                keys.append(k)
                counts.append(c)
        hk = np.array(keys or [0], dtype=np.uint64)
        hc = np.array(counts or [0], dtype=np.int32)
        check(self._L.sentinel_load_local_param_rules(self._h, arr, len(rules), _p(hk), _p(hc), len(keys)),
              "load_local_param_rules")

    def submit_local_param_batch_host(self, rule_idx, acquire, ts, value_begin, value_count, values):
        """ParamFlowChecker.passLocalCheck per event; returns the status array (OK / BLOCKED / ...)."""
        ev = self.pack_multi_events(rule_idx, acquire, ts, value_begin, value_count)
        vals = np.ascontiguousarray(values, dtype=np.uint64)
        out = np.empty(len(ev), dtype=_lib.VERDICT_DTYPE)
        check(self._L.sentinel_submit_local_param_batch_host(self._h, len(ev), _p(ev), _p(vals) if len(vals) else None,
                                                             len(vals), _p(out)), "submit_local_param_batch_host")
        return out["status"].astype(np.int8)

    def set_local_param_grades(self, grades):
        """ParamFlowRule.grade per loaded local rule: 1 QPS (default), 0 THREAD."""
        g = np.ascontiguousarray(grades, dtype=np.int32)
        check(self._L.sentinel_set_local_param_grades(self._h, _p(g), len(g)), "set_local_param_grades")

    def submit_local_param_batch_ex_host(self, rule_idx, acquire, ts, value_begin, value_count, values, kinds=None):
        """As submit_local_param_batch_host, kinds[i] == 1 marking Entry.exit events (thread counts drop)."""
        ev = self.pack_multi_events(rule_idx, acquire, ts, value_begin, value_count)
        vals = np.ascontiguousarray(values, dtype=np.uint64)
        k = None if kinds is None else np.ascontiguousarray(kinds, dtype=np.uint8)
        out = np.empty(len(ev), dtype=_lib.VERDICT_DTYPE)
        check(self._L.sentinel_submit_local_param_batch_ex_host(self._h, len(ev), _p(ev), _p(k),
                                                                _p(vals) if len(vals) else None, len(vals), _p(out)),
              "submit_local_param_batch_ex_host")
        return out["status"].astype(np.int8)

    def local_param_state(self, key: int):
        last, tok = C.c_int64(), C.c_int64()
        rc = self._L.sentinel_local_param_state(self._h, int(key), C.byref(last), C.byref(tok))
        check(rc, "local_param_state")
        return last.value, tok.value

    # ---------------------------------------------------------------- local SphU.entry (DefaultController)
    def load_local_resources(self, counts, sample_count: int = 2, interval_ms: int = 1000):
        """Local resources (index = position): the smallest QPS rule count per resource, or None for
        a resource without flow rules; the StatisticNode window config (SampleCountProperty,
        IntervalProperty)."""
        arr = (_lib.LocalResourceC * max(len(counts), 1))()
        for i, c in enumerate(counts):
            arr[i] = _lib.LocalResourceC(0.0 if c is None else float(c), 0 if c is None else 1, 0)
        check(self._L.sentinel_load_local_resources(self._h, arr, len(counts), int(sample_count), int(interval_ms)),
              "load_local_resources")

    def load_local_resources_ex(self, qps_counts, thread_counts, thread_first=None, sample_count: int = 2,
                                interval_ms: int = 1000):
        """Resources with a QPS and / or a THREAD grade rule (None: no rule of that grade);
        thread_first[i]: the THREAD rule is checked before the QPS one."""
        n = len(qps_counts)
        arr = (_lib.LocalResourceExC * max(n, 1))()
        for i in range(n):
            q, t = qps_counts[i], thread_counts[i]
            f = (0 if q is None else _lib.LOCAL_QPS) | (0 if t is None else _lib.LOCAL_THREAD)
            if thread_first is not None and thread_first[i]:
                f |= _lib.LOCAL_THREAD_FIRST
            arr[i] = _lib.LocalResourceExC(0.0 if q is None else float(q), 0.0 if t is None else float(t), f, 0)
        check(self._L.sentinel_load_local_resources_ex(self._h, arr, n, int(sample_count), int(interval_ms)),
              "load_local_resources_ex")

    def submit_local_batch_host(self, resource_idx, acquire, ts, flags=None, rt=None):
        """Entries and exits (flags: LOCAL_PRIO / LOCAL_EXIT / LOCAL_ERROR; rt: exit response times)
        -> (status, waitInMs)."""
        ev = self.pack_events(resource_idx, acquire, ts)
        fl = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint8)
        r = None if rt is None else np.ascontiguousarray(rt, dtype=np.int64)
        out = np.empty(len(ev), dtype=_lib.VERDICT_DTYPE)
        check(self._L.sentinel_submit_local_batch_host(self._h, len(ev), _p(ev), _p(fl), _p(r), _p(out)),
              "submit_local_batch_host")
        return out["status"].astype(np.int8), out["wait_in_ms"].astype(np.int64)

    def local_node_metrics(self, resource_idx: int, ts: int) -> np.ndarray:
        """[second PASS, BLOCK, EXCEPTION, SUCCESS, RT, minRt, minute PASS, BLOCK, OCCUPIED_PASS,
        EXCEPTION, SUCCESS, RT, minRt, curThreadNum] of the resource's node at ts (read-only)."""
        out = np.zeros(14, dtype=np.int64)
        check(self._L.sentinel_local_node_metrics(self._h, int(resource_idx), int(ts), _p(out)), "local_node_metrics")
        return out

    def load_local_rules(self, rules, n_resources: int, n_origin_nodes: int, n_default_nodes: int,
                         sample_count: int = 2, interval_ms: int = 1000):
        """FlowRuleManager.loadRules over the local rule graph (FlowRuleChecker with every limitApp
        and strategy): `rules` is a LOCAL_RULE_DTYPE array (or records of its fields) in
        FlowRuleManager's order; invalid rules are dropped and the rules sorted as the reference's
        buildFlowRuleMap does.  Every node starts empty."""
        arr = np.zeros(len(rules), dtype=_lib.LOCAL_RULE_DTYPE)
        for i, r in enumerate(rules):
            arr[i] = tuple(r) if not isinstance(r, np.void) else r
        check(self._L.sentinel_load_local_rules(self._h, _p(arr) if len(arr) else None, len(arr), int(n_resources),
                                                int(n_origin_nodes), int(n_default_nodes), int(sample_count),
                                                int(interval_ms)), "load_local_rules")

    def submit_local_graph_batch_host(self, resource_idx, acquire, ts, ctx, flags=None, rt=None):
        """Entries / exits with their contexts (LOCAL_CTX_DTYPE: origin, origin_node, context,
        default_node) -> (status, waitInMs)."""
        ev = self.pack_events(resource_idx, acquire, ts)
        cx = np.ascontiguousarray(ctx, dtype=_lib.LOCAL_CTX_DTYPE)
        if len(cx) != len(ev):
            raise ValueError("one context per event")
        fl = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint8)
        r = None if rt is None else np.ascontiguousarray(rt, dtype=np.int64)
        out = np.empty(len(ev), dtype=_lib.VERDICT_DTYPE)
        check(self._L.sentinel_submit_local_graph_batch_host(self._h, len(ev), _p(ev), _p(cx), _p(fl), _p(r), _p(out)),
              "submit_local_graph_batch_host")
        return out["status"].astype(np.int8), out["wait_in_ms"].astype(np.int64)

    def local_graph_node_metrics(self, kind: int, idx: int, ts: int) -> np.ndarray:
        """local_node_metrics of a ClusterNode (NODE_CLUSTER), origin node or DefaultNode."""
        out = np.zeros(14, dtype=np.int64)
        check(self._L.sentinel_local_graph_node_metrics(self._h, int(kind), int(idx), int(ts), _p(out)),
              "local_graph_node_metrics")
        return out

    def set_statistic_max_rt(self, ms: int):
        check(self._L.sentinel_set_statistic_max_rt(self._h, int(ms)), "set_statistic_max_rt")

    def submit_local_entry_batch_host(self, resource_idx, acquire, ts, prioritized=None, with_wait=False):
        """SphU.entry (SphU.entryWithPriority where `prioritized`) for a batch -> status array (OK =
        entry, BLOCKED = FlowException); with_wait also returns waitInMs (> 0: an occupied pass,
        the PriorityWaitException wait)."""
        ev = self.pack_events(resource_idx, acquire, ts)
        pr = None if prioritized is None else np.ascontiguousarray(prioritized, dtype=np.uint8)
        out = np.empty(len(ev), dtype=_lib.VERDICT_DTYPE)
        check(self._L.sentinel_submit_local_entry_batch_host(self._h, len(ev), _p(ev), _p(pr), _p(out)),
              "submit_local_entry_batch_host")
        st = out["status"].astype(np.int8)
        return (st, out["wait_in_ms"].astype(np.int64)) if with_wait else st

    def set_occupy_timeout(self, ms: int):
        """OccupyTimeoutProperty.updateTimeout (ignored when < 0 or above the node interval)."""
        check(self._L.sentinel_set_occupy_timeout(self._h, int(ms)), "set_occupy_timeout")

    def local_node_stats(self, resource_idx: int, ts: int) -> np.ndarray:
        """{second PASS, second BLOCK, minute PASS, minute BLOCK, minute OCCUPIED_PASS, waiting} of
        the resource's node at ts (read-only)."""
        out = np.zeros(6, dtype=np.int64)
        check(self._L.sentinel_local_node_stats(self._h, int(resource_idx), int(ts), _p(out)), "local_node_stats")
        return out

    def synchronize(self):
        check(self._L.sentinel_synchronize(self._h), "synchronize")

    # ---------------------------------------------------------------- observability
    def flow_window(self, idx: int):
        """(sampleCount, intervalMs) of the metric behind flow idx (a reload keeps a surviving flowId's
        metric, so this can differ from its current rule's window)."""
        n, iv = C.c_int32(), C.c_int32()
        check(self._L.sentinel_flow_window(self._h, int(idx), C.byref(n), C.byref(iv)), "flow_window")
        return n.value, iv.value

    def metric_count(self) -> int:
        """ClusterMetricStatistics.METRIC_MAP.size() (orphaned metrics included)."""
        return int(self._L.sentinel_metric_count(self._h))

    def reset_metrics(self, sample_count: int, interval_ms: int):
        """Server window change: every flow / param metric restarts with this window
        (ClusterServerConfigManager.java:333-343)."""
        check(self._L.sentinel_reset_metrics(self._h, int(sample_count), int(interval_ms)), "reset_metrics")

    def param_table_stats(self):
        """{capacity, live slots after the last rebuild, rebuilds} of the exact param slot table."""
        out = np.zeros(3, dtype=np.int64)
        check(self._L.sentinel_param_table_stats(self._h, _p(out)), "param_table_stats")
        return dict(capacity=int(out[0]), live=int(out[1]), rebuilds=int(out[2]))

    def param_cm_stats(self):
        """{key_walk, overflow, block}: shared count-min batches decided by the key walk / by the per-rule
        lanes, and the key-walk batches decided by the block-owned walk (k_pp_cm_block)."""
        out = np.zeros(2, dtype=np.int64)
        check(self._L.sentinel_param_cm_stats(self._h, _p(out)), "param_cm_stats")
        blk = np.zeros(1, dtype=np.int64)
        check(self._L.sentinel_param_cm_block_batches(self._h, _p(blk)), "param_cm_block_batches")
        return dict(key_walk=int(out[0]), overflow=int(out[1]), block=int(blk[0]))

    def flow_path_stats(self):
        """Flow batches so far by pipeline: {small, sorted, partition, ordered (of the partition batches, those
        with decide-order output: sentinel_submit_flow_batch_ordered)}."""
        out = np.zeros(4, dtype=np.int64)
        check(self._L.sentinel_flow_path_stats(self._h, _p(out)), "flow_path_stats")
        return dict(small=int(out[0]), sorted=int(out[1]), partition=int(out[2]), ordered=int(out[3]))

    def param_top_values(self, ts: int, number: int = _lib.TOP_PARAMS):
        """getTopValues(number) of every param rule at ts -> list (per rule index) of [(key, avg)]."""
        n_rules = self.param_count()
        cnt = np.zeros(max(n_rules, 1), dtype=np.int32)
        keys = np.zeros(max(n_rules, 1) * number, dtype=np.uint64)
        avgs = np.zeros(max(n_rules, 1) * number, dtype=np.float64)
        check(self._L.sentinel_param_top_values(self._h, int(ts), int(number), _p(cnt), _p(keys), _p(avgs)),
              "param_top_values")
        return [[(int(keys[r * number + k]), float(avgs[r * number + k])) for k in range(int(cnt[r]))]
                for r in range(n_rules)]

    def param_snapshot_device(self, ts: int, out_tensor, stream=None):
        """paramToMetricNode records (flowId, top-5 params) of every param rule into a device tensor
        of len(rules) * 96 bytes (PARAM_SNAPSHOT_DTYPE layout)."""
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        check(self._L.sentinel_param_snapshot_device(self._h, int(ts), C.c_void_p(out_tensor.data_ptr()),
                                                     None if s is None else C.c_void_p(s)), "param_snapshot_device")
        return out_tensor

    def dump_flow(self, idx: int, sample_count: Optional[int] = None) -> np.ndarray:
        """Window dump of flow idx (oracle layout); the window is the metric's (flow_window)."""
        sample_count = self.flow_window(idx)[0]
        out = np.zeros(sample_count * 8 + 8, dtype=np.int64)
        check(self._L.sentinel_dump_flow(self._h, int(idx), _p(out), len(out)), "dump_flow")
        return out

    def param_sum(self, rule_idx: int, key: int, ts: int) -> int:
        v = C.c_int64()
        check(self._L.sentinel_param_sum(self._h, rule_idx, key, ts, C.byref(v)), "param_sum")
        return v.value

    def snapshot(self, ts: int) -> np.ndarray:
        n = self.flow_count()
        out = np.zeros(n, dtype=[("flow_id", "<i8"), ("pass_qps", "<f8"), ("block_qps", "<f8")])
        check(self._L.sentinel_snapshot(self._h, int(ts), C.c_void_p(out.ctypes.data)), "snapshot")
        return out

    def snapshot_device(self, ts: int, out_tensor, stream=None):
        s = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        check(self._L.sentinel_snapshot_device(self._h, int(ts), C.c_void_p(out_tensor.data_ptr()),
                                               None if s is None else C.c_void_p(s)), "snapshot_device")
        return out_tensor


class GpuTokenCluster:
    """One TokenService over several engines of one node (sentinel_cluster_*): the flowId space
    partitioned shard = splitmix64(flowId) mod n, one engine per entry of device_ids (a device may
    repeat).  Rule tables are split by shard, config is broadcast, host batches are routed and
    decided concurrently, verdicts come back at the arrival positions."""

    def __init__(self, device_ids: Sequence[int], exceed_count: float = 1.0, max_occupy_ratio: float = 1.0):
        self._L = _lib.load()
        self._h = C.c_void_p()
        ids = np.ascontiguousarray(device_ids, dtype=np.int32)
        cfg = _lib.ServerConfig(exceed_count, max_occupy_ratio)
        check(self._L.sentinel_cluster_create(_p(ids), len(ids), C.byref(cfg), C.byref(self._h)), "cluster_create")
        _LIVE_ENGINES.add(self)
        self.n = len(ids)

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._L.sentinel_cluster_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def shard_of(self, flow_id: int) -> int:
        return int(self._L.sentinel_shard_of(int(flow_id), self.n))

    def set_namespaces(self, namespaces: Sequence[ServerNamespace]):
        arr = (_lib.Namespace * max(len(namespaces), 1))()
        for i, ns in enumerate(namespaces):
            arr[i] = _lib.Namespace(int(ns.connected_count), int(bool(ns.has_limiter)), float(ns.max_allowed_qps))
        check(self._L.sentinel_cluster_set_namespaces(self._h, arr, len(namespaces)), "cluster_set_namespaces")

    def load_rules_array(self, flow_ids, counts, threshold_type=1, sample_count=10, window_interval_ms=1000,
                         namespace=0, checker=0):
        n = len(flow_ids)
        rec = np.zeros(n, dtype=[("flow_id", "<i8"), ("count", "<f8"), ("threshold_type", "<i4"),
                                 ("sample_count", "<i4"), ("window_interval_ms", "<i4"),
                                 ("namespace_idx", "<i4"), ("checker", "<i4"), ("reserved", "<i4")])
        rec["flow_id"] = flow_ids
        rec["count"] = counts
        rec["threshold_type"] = threshold_type
        rec["sample_count"] = sample_count
        rec["window_interval_ms"] = window_interval_ms
        rec["namespace_idx"] = namespace
        rec["checker"] = checker
        check(self._L.sentinel_cluster_load_flow_rules(self._h, C.c_void_p(rec.ctypes.data), n), "cluster_load_flow_rules")

    def flow_count(self) -> int:
        return int(self._L.sentinel_cluster_flow_count(self._h))

    def submit_host(self, flow_ids, acquire, ts, flags=None):
        """requestToken per (flowId, acquire, ts[, prioritized flag]) -> (status, remaining, waitInMs)."""
        ids = np.ascontiguousarray(flow_ids, dtype=np.int64)
        a = np.ascontiguousarray(acquire, dtype=np.int32)
        t = np.ascontiguousarray(ts, dtype=np.int64)
        fl = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint8)
        out = np.empty(len(ids), dtype=_lib.VERDICT_DTYPE)
        check(self._L.sentinel_cluster_submit_host(self._h, len(ids), _p(ids), _p(a), _p(t), _p(fl), _p(out)),
              "cluster_submit_host")
        return out["status"].astype(np.int8), out["remaining"].copy(), out["wait_in_ms"].astype(np.int32)

    def snapshot(self, ts: int) -> np.ndarray:
        n = self.flow_count()
        out = np.zeros(max(n, 1), dtype=[("flow_id", "<i8"), ("pass_qps", "<f8"), ("block_qps", "<f8")])
        got = C.c_int64()
        check(self._L.sentinel_cluster_snapshot(self._h, int(ts), C.c_void_p(out.ctypes.data), len(out), C.byref(got)),
              "cluster_snapshot")
        return out[:got.value]

    def start_batchers(self, max_batch: int = 4096, max_wait_us: int = 50):
        check(self._L.sentinel_cluster_batchers_create(self._h, int(max_batch), int(max_wait_us)), "cluster_batchers_create")

    def request_token(self, rule_id, acquire_count, prioritized=False, ts=None) -> TokenResult:
        out = _lib.TokenResultC()
        fid = 0 if rule_id is None else int(rule_id)
        check(self._L.sentinel_cluster_request_token(self._h, fid, int(acquire_count), int(bool(prioritized)),
                                                     _now_ms() if ts is None else int(ts), C.byref(out)),
              "cluster_request_token")
        return TokenResult(out.status, out.remaining, out.wait_in_ms)


class TokenBatcher:
    """Concurrent per-call front door: thread-safe request_token that is batched on the GPU
    (sentinel_batcher_*).  ctypes releases the GIL during the call, so Python threads really wait
    in parallel; the Java shim uses the same entry point from Netty worker threads."""

    def __init__(self, svc: "GpuTokenService", max_batch: int = 4096, max_wait_us: int = 50):
        self._svc = svc
        self._L = svc._L
        self._b = C.c_void_p()
        check(self._L.sentinel_batcher_create(svc.handle, max_batch, max_wait_us, C.byref(self._b)), "batcher_create")
        _LIVE_BATCHERS.add(self)

    def request_token(self, rule_id, acquire_count, prioritized=False, ts=None) -> TokenResult:
        out = _lib.TokenResultC()
        fid = 0 if rule_id is None else int(rule_id)
        check(self._L.sentinel_batcher_request_token(self._b, fid, int(acquire_count), int(bool(prioritized)),
                                                     _now_ms() if ts is None else int(ts), C.byref(out)),
              "batcher_request_token")
        return TokenResult(out.status, out.remaining, out.wait_in_ms)

    def stats(self):
        b, r = C.c_int64(), C.c_int64()
        check(self._L.sentinel_batcher_stats(self._b, C.byref(b), C.byref(r)), "batcher_stats")
        return b.value, r.value

    def close(self):
        if self._b.value:
            self._L.sentinel_batcher_destroy(self._b)
            self._b = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def decode_verdicts(v):
    """Packed int64 verdicts (torch or numpy) -> (status int16, remaining int32, wait uint16) numpy."""
    a = v.cpu().numpy() if hasattr(v, "cpu") else np.asarray(v)
    a = a.view(_lib.VERDICT_DTYPE)
    return a["status"], a["remaining"], a["wait_in_ms"]


def device_events(flow_idx, acquire, ts):
    """Build the (n, 2) int64 device tensor of sentinel_event_t records from torch tensors."""
    import torch
    w0 = (acquire.to(torch.int64) << 32) | (flow_idx.to(torch.int64) & 0xFFFFFFFF)
    return torch.stack([w0, ts.to(torch.int64)], dim=1).contiguous()


def device_count() -> int:
    return int(_lib.load().sentinel_device_count())
