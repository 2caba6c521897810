"""ctypes binding for the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: the parity checker and bench.py's ``cpu_baseline`` leg.  The product
package ``sentinel_amd`` never imports this module.  The restatement itself lives in
``oracle/sentinel_oracle.c`` (every function cites the reference Java file:line it follows).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

# ClusterFlowEvent ordinals (ClusterFlowEvent.java:22-52)
PASS, BLOCK, PASS_REQUEST, BLOCK_REQUEST, OCCUPIED_PASS, OCCUPIED_BLOCK, WAITING = range(7)
NEVENTS = 7

# TokenResultStatus (core/cluster/TokenResultStatus.java:27-69)
BAD_REQUEST, TOO_MANY_REQUEST, FAIL, OK, BLOCKED, SHOULD_WAIT, NO_RULE_EXISTS = -4, -2, -1, 0, 1, 2, 3


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


class FlowRule(C.Structure):
    _fields_ = [("flow_id", C.c_int64), ("count", C.c_double), ("threshold_type", C.c_int32),
                ("sample_count", C.c_int32), ("window_interval_ms", C.c_int32),
                ("namespace_idx", C.c_int32), ("checker", C.c_int32), ("reserved", C.c_int32)]


class Namespace(C.Structure):
    _fields_ = [("connected_count", C.c_int32), ("has_limiter", C.c_int32), ("max_allowed_qps", C.c_double)]


class ServerConfig(C.Structure):
    _fields_ = [("exceed_count", C.c_double), ("max_occupy_ratio", C.c_double)]


class ParamRule(C.Structure):
    _fields_ = [("flow_id", C.c_int64), ("count", C.c_double), ("threshold_type", C.c_int32),
                ("sample_count", C.c_int32), ("window_interval_ms", C.c_int32),
                ("namespace_idx", C.c_int32), ("hot_begin", C.c_int32), ("hot_n", C.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
            os.path.join(_HERE, "sentinel_oracle.c")):
        build()
    L = C.CDLL(_LIB_PATH)
    vp, i32, i64, u64, dbl = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_double
    sig = {
        "orc_cm_new": (vp, [C.c_int, C.c_int]),
        "orc_cm_free": (None, [vp]),
        "orc_cm_add": (None, [vp, i64, C.c_int, i64]),
        "orc_cm_get_sum": (i64, [vp, i64, C.c_int]),
        "orc_cm_get_current_count": (i64, [vp, i64, C.c_int]),
        "orc_cm_get_avg": (dbl, [vp, i64, C.c_int]),
        "orc_cm_try_occupy_next": (C.c_int, [vp, i64, C.c_int, C.c_int, dbl]),
        "orc_cm_dump": (None, [vp, vp]),
        "orc_cm_list_count": (C.c_int, [vp, i64]),
        "orc_cm_first_count": (i64, [vp, i64, C.c_int]),
        "orc_cm_window_start": (i64, [vp, i64]),
        "orc_limiter_new": (vp, [dbl]),
        "orc_limiter_free": (None, [vp]),
        "orc_limiter_add": (None, [vp, i64, C.c_int]),
        "orc_limiter_get_sum": (i64, [vp, i64]),
        "orc_limiter_get_qps": (dbl, [vp, i64]),
        "orc_limiter_can_pass": (C.c_int, [vp, i64]),
        "orc_limiter_try_pass": (C.c_int, [vp, i64]),
        "orc_pm_new": (vp, [C.c_int, C.c_int, C.c_int]),
        "orc_pm_free": (None, [vp]),
        "orc_pm_add_value": (None, [vp, i64, u64, C.c_int]),
        "orc_pm_get_sum": (i64, [vp, i64, u64]),
        "orc_pm_get_avg": (dbl, [vp, i64, u64]),
        "orc_pm_top_values": (C.c_int, [vp, i64, C.c_int, vp, vp]),
        "orc_engine_new": (vp, [vp, vp, C.c_int]),
        "orc_engine_free": (None, [vp]),
        "orc_engine_load_flow_rules": (C.c_int, [vp, vp, C.c_int]),
        "orc_engine_set_connected_count": (None, [vp, C.c_int32, C.c_int32]),
        "orc_request_token": (None, [vp, i32, i32, C.c_int, i64, vp, vp, vp]),
        "orc_flow_replay": (None, [vp, i64, vp, vp, vp, vp, vp, vp, vp]),
        "orc_flow_replay_mt": (C.c_int, [vp, i64, vp, vp, vp, vp, vp, vp, vp, C.c_int]),
        "orc_engine_dump_flow": (C.c_int, [vp, i32, vp]),
        "orc_engine_reset_metrics": (C.c_int, [vp, C.c_int, C.c_int]),
        "orc_engine_flow_window": (C.c_int, [vp, i32, vp]),
        "orc_engine_metric_count": (i64, [vp]),
        "orc_engine_param_top_values": (C.c_int, [vp, i32, i64, C.c_int, vp, vp]),
        "orc_engine_param_window": (C.c_int, [vp, i32, vp]),
        "orc_engine_limiter_sum": (i64, [vp, i32, i64]),
        "orc_engine_load_param_rules": (C.c_int, [vp, vp, C.c_int, vp, vp, C.c_int]),
        "orc_request_param_token": (None, [vp, i32, i32, i64, vp, C.c_int, vp, vp]),
        "orc_param_replay": (None, [vp, i64, vp, vp, vp, vp, vp, vp]),
        "orc_param_replay_mt": (C.c_int, [vp, i64, vp, vp, vp, vp, vp, vp, C.c_int]),
        "orc_engine_param_sum": (i64, [vp, i32, i64, u64]),
        "orc_engine_param_overflowed": (C.c_int, [vp]),
        "orc_node_new": (vp, [C.c_int, C.c_int]),
        "orc_node_free": (None, [vp]),
        "orc_node_pass_qps": (dbl, [vp, i64]),
        "orc_node_pass_sum": (i64, [vp, i64]),
        "orc_node_block_sum": (i64, [vp, i64]),
        "orc_node_total_pass": (i64, [vp, i64]),
        "orc_node_minute_block": (i64, [vp, i64]),
        "orc_node_add_pass_request": (None, [vp, i64, C.c_int]),
        "orc_node_increase_block_qps": (None, [vp, i64, C.c_int]),
        "orc_default_controller_can_pass": (C.c_int, [vp, dbl, C.c_int, C.c_int, i32, i64]),
        "orc_default_controller_check": (C.c_int, [dbl, dbl, C.c_int, C.c_int]),
        "orc_local_replay": (None, [vp, dbl, i64, vp, vp, vp]),
        "orc_local_replay_prio": (None, [vp, dbl, i64, vp, vp, vp, vp, vp]),
        "orc_local_entry": (C.c_int, [vp, dbl, C.c_int, C.c_int, i64, vp]),
        "orc_node_set_occupy_timeout": (None, [vp, C.c_int]),
        "orc_node_set_max_rt": (None, [vp, i64]),
        "orc_local_entry_ex": (C.c_int, [vp, dbl, dbl, C.c_int, C.c_int, C.c_int, i64, vp]),
        "orc_local_exit": (None, [vp, C.c_int, i64, C.c_int, i64]),
        "orc_node_metrics": (None, [vp, i64, vp]),
        "orc_lgraph_new": (vp, [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
        "orc_lgraph_free": (None, [vp]),
        "orc_lgraph_set_occupy_timeout": (None, [vp, C.c_int]),
        "orc_lgraph_n_rules": (C.c_int, [vp, C.c_int]),
        "orc_lgraph_replay": (None, [vp, i64, vp, vp, vp, vp, vp, vp, vp, vp]),
        "orc_lgraph_node_metrics": (C.c_int, [vp, C.c_int, C.c_int, i64, vp]),
        "orc_node_waiting": (i64, [vp, i64]),
        "orc_node_minute_occupied": (i64, [vp, i64]),
        "orc_node_try_occupy_next": (i64, [vp, i64, C.c_int, dbl]),
        "orc_node_add_waiting": (None, [vp, i64, C.c_int]),
        "orc_node_add_occupied_pass": (None, [vp, i64, C.c_int]),
        "orc_node_sec_window_pass": (i64, [vp, i64]),
        "orc_node_sec_window_add_pass": (None, [vp, i64, C.c_int]),
        "orc_node_sec_values": (i64, [vp, i64, vp]),
        "orc_pbucket_new": (vp, []),
        "orc_pbucket_free": (None, [vp]),
        "orc_pbucket_pass_default": (C.c_int, [vp, u64, i64, i64, i64, C.c_int, i64]),
        "orc_param_multi_replay": (None, [vp, i64, vp, vp, vp, vp, vp, vp, i64, vp, vp]),
        "orc_param_cm_audit": (None, [vp, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "orc_lparam_new": (vp, [vp, C.c_int, vp, vp, C.c_int]),
        "orc_lparam_free": (None, [vp]),
        "orc_lparam_replay": (None, [vp, i64, vp, vp, vp, vp, vp, vp, i64, vp]),
        "orc_lparam_state": (C.c_int, [vp, i32, u64, vp, vp]),
        "orc_lparam_set_grades": (None, [vp, vp, C.c_int]),
        "orc_lparam_replay_ex": (None, [vp, i64, vp, vp, vp, vp, vp, vp, i64, vp, vp]),
        "orc_lparam_thread_count": (C.c_int, [vp, i32, u64]),
        "orc_concurrent_replay": (None, [vp, i64, vp, vp, vp, vp]),
        "orc_concurrent_replay_mt": (C.c_int, [vp, i64, vp, vp, vp, vp, C.c_int]),
        "orc_concurrent_now_calls": (i32, [vp, i32]),
        "orc_concurrent_token_count": (i64, [vp]),
        "orc_concurrent_expire_all": (i64, [vp]),
        "orc_java_d2i": (i32, [dbl]),
        "orc_java_string_hash": (i32, [vp, i64]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _p(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class ClusterMetric:
    """ClusterMetric(sampleCount, intervalInMs) (ClusterMetric.java:32-37)."""

    def __init__(self, sample_count: int, interval_ms: int):
        self.n = sample_count
        self.h = lib().orc_cm_new(sample_count, interval_ms)
        if not self.h:
            raise ValueError("invalid ClusterMetric arguments")

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_cm_free(self.h)

    def add(self, t, event, count): lib().orc_cm_add(self.h, t, event, count)
    def get_sum(self, t, event): return lib().orc_cm_get_sum(self.h, t, event)
    def get_current_count(self, t, event): return lib().orc_cm_get_current_count(self.h, t, event)
    def get_avg(self, t, event): return lib().orc_cm_get_avg(self.h, t, event)
    def try_occupy_next(self, t, event, acquire, threshold): return lib().orc_cm_try_occupy_next(self.h, t, event, acquire, threshold)
    def list_count(self, t): return lib().orc_cm_list_count(self.h, t)
    def first_count(self, t, event): return lib().orc_cm_first_count(self.h, t, event)
    def window_start(self, t): return lib().orc_cm_window_start(self.h, t)

    def dump(self) -> np.ndarray:
        out = np.zeros(self.n * 8 + 8, dtype=np.int64)
        lib().orc_cm_dump(self.h, _p(out))
        return out


class RequestLimiter:
    """RequestLimiter(qpsAllowed) (RequestLimiter.java:35-37)."""

    def __init__(self, qps_allowed: float):
        self.h = lib().orc_limiter_new(qps_allowed)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_limiter_free(self.h)

    def add(self, t, x): lib().orc_limiter_add(self.h, t, x)
    def get_sum(self, t): return lib().orc_limiter_get_sum(self.h, t)
    def get_qps(self, t): return lib().orc_limiter_get_qps(self.h, t)
    def can_pass(self, t): return bool(lib().orc_limiter_can_pass(self.h, t))
    def try_pass(self, t): return bool(lib().orc_limiter_try_pass(self.h, t))


class ClusterParamMetric:
    """ClusterParamMetric(sampleCount, intervalMs, maxCapacity) (ClusterParamMetric.java:35-44)."""

    def __init__(self, sample_count: int, interval_ms: int, max_capacity: int = 4000):
        self.h = lib().orc_pm_new(sample_count, interval_ms, max_capacity)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_pm_free(self.h)

    def add_value(self, t, key, count): lib().orc_pm_add_value(self.h, t, key, count)
    def get_sum(self, t, key): return lib().orc_pm_get_sum(self.h, t, key)
    def get_avg(self, t, key): return lib().orc_pm_get_avg(self.h, t, key)

    def top_values(self, t, number):
        keys = np.zeros(max(number, 1), dtype=np.uint64)
        avgs = np.zeros(max(number, 1), dtype=np.float64)
        k = lib().orc_pm_top_values(self.h, t, number, _p(keys), _p(avgs))
        if k < 0:
            raise ValueError("number must be positive")
        return {int(keys[i]): float(avgs[i]) for i in range(k)}


LR_QPS, LR_THREAD, LR_THREAD_FIRST = 1, 2, 4


class StatisticNode:
    def __init__(self, sample_count: int = 2, interval_ms: int = 1000):
        self.h = lib().orc_node_new(sample_count, interval_ms)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_node_free(self.h)

    def pass_qps(self, t): return lib().orc_node_pass_qps(self.h, t)
    def pass_sum(self, t): return lib().orc_node_pass_sum(self.h, t)
    def block_sum(self, t): return lib().orc_node_block_sum(self.h, t)
    def total_pass(self, t): return lib().orc_node_total_pass(self.h, t)
    def minute_block(self, t): return lib().orc_node_minute_block(self.h, t)
    def add_pass_request(self, t, c): lib().orc_node_add_pass_request(self.h, t, c)
    def increase_block_qps(self, t, c): lib().orc_node_increase_block_qps(self.h, t, c)

    def can_pass(self, count, acquire, t, grade=1, cur_thread_num=0):
        return bool(lib().orc_default_controller_can_pass(self.h, count, grade, acquire, cur_thread_num, t))

    def replay(self, count, acquire: np.ndarray, ts: np.ndarray) -> np.ndarray:
        acquire = np.ascontiguousarray(acquire, dtype=np.int32)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        out = np.zeros(len(ts), dtype=np.uint8)
        lib().orc_local_replay(self.h, count, len(ts), _p(acquire), _p(ts), _p(out))
        return out

    def replay_prio(self, count, acquire: np.ndarray, ts: np.ndarray, prio: np.ndarray):
        """(passed u8, waitInMs i64) per entry, prioritized entries included."""
        acquire = np.ascontiguousarray(acquire, dtype=np.int32)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        prio = np.ascontiguousarray(prio, dtype=np.uint8)
        out = np.zeros(len(ts), dtype=np.uint8)
        wait = np.zeros(len(ts), dtype=np.int64)
        lib().orc_local_replay_prio(self.h, count, len(ts), _p(acquire), _p(ts), _p(prio), _p(out), _p(wait))
        return out, wait

    def entry(self, count, acquire, t, prioritized=False):
        w = C.c_int64(0)
        ok = lib().orc_local_entry(self.h, count, acquire, int(prioritized), t, C.byref(w))
        return bool(ok), int(w.value)

    def set_occupy_timeout(self, ms): lib().orc_node_set_occupy_timeout(self.h, ms)
    def set_max_rt(self, ms): lib().orc_node_set_max_rt(self.h, ms)

    # QPS / THREAD grade rules (flags: LR_QPS | LR_THREAD | LR_THREAD_FIRST) and exits
    def entry_ex(self, qps_count, thread_count, flags, acquire, t, prioritized=False):
        w = C.c_int64(0)
        ok = lib().orc_local_entry_ex(self.h, qps_count, thread_count, flags, acquire, int(prioritized), t, C.byref(w))
        return bool(ok), int(w.value)

    def exit(self, count, rt, t, error=False):
        lib().orc_local_exit(self.h, count, rt, int(error), t)

    def metrics(self, t) -> np.ndarray:
        """[sec PASS, BLOCK, EXCEPTION, SUCCESS, RT, minRt, min PASS, BLOCK, OCCUPIED_PASS, EXCEPTION,
        SUCCESS, RT, minRt, curThreadNum] at t (read-only, no roll)."""
        out = np.zeros(14, dtype=np.int64)
        lib().orc_node_metrics(self.h, t, _p(out))
        return out
    def waiting(self, t): return lib().orc_node_waiting(self.h, t)
    def minute_occupied(self, t): return lib().orc_node_minute_occupied(self.h, t)
    def try_occupy_next(self, t, acquire, threshold): return lib().orc_node_try_occupy_next(self.h, t, acquire, threshold)
    def add_waiting(self, future_t, c): lib().orc_node_add_waiting(self.h, future_t, c)
    def add_occupied_pass(self, t, c): lib().orc_node_add_occupied_pass(self.h, t, c)
    # OccupiableBucketLeapArray surface (rollingCounterInSecond's array) for the reference's own tests
    def window_pass(self, t): return lib().orc_node_sec_window_pass(self.h, t)
    def window_add_pass(self, t, c): lib().orc_node_sec_window_add_pass(self.h, t, c)

    def values(self, t):
        s = C.c_int64(0)
        k = lib().orc_node_sec_values(self.h, t, C.byref(s))
        return int(k), int(s.value)


class ParamTokenBucket:
    """ParameterMetric token/time counters for one rule (ParamFlowChecker.java:127-202)."""

    def __init__(self):
        self.h = lib().orc_pbucket_new()

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_pbucket_free(self.h)

    def pass_default(self, key, token_count, burst, duration_sec, acquire, t):
        return lib().orc_pbucket_pass_default(self.h, key, token_count, burst, duration_sec, acquire, t)


class LocalParamRule(C.Structure):
    _fields_ = [("count", C.c_double), ("burst_count", C.c_int64), ("duration_in_sec", C.c_int64),
                ("hot_begin", C.c_int32), ("hot_n", C.c_int32)]


def _multi_args(rule_idx, acquire, ts, vbegin, vcount, values):
    return (np.ascontiguousarray(rule_idx, dtype=np.int32), np.ascontiguousarray(acquire, dtype=np.int32),
            np.ascontiguousarray(ts, dtype=np.int64), np.ascontiguousarray(vbegin, dtype=np.int32),
            np.ascontiguousarray(vcount, dtype=np.int32), np.ascontiguousarray(values, dtype=np.uint64))


class LocalParamOracle:
    """ParamFlowChecker.passLocalCheck replay, one ParameterMetric per rule (ParamFlowChecker.java:78-202).
    rules: [(count, burst_count, duration_in_sec, {key: hot_count})]; rule index = position."""

    def __init__(self, rules, grades=None):
        arr = (LocalParamRule * max(len(rules), 1))()
        keys, counts = [], []
        for i, (count, burst, dur, hot) in enumerate(rules):
            arr[i] = LocalParamRule(float(count), int(burst), int(dur), len(keys), len(hot))
            for k, c in hot.items():
                keys.append(k)
                counts.append(c)
        hk = np.array(keys or [0], dtype=np.uint64)
        hc = np.array(counts or [0], dtype=np.int32)
        self.h = lib().orc_lparam_new(arr, len(rules), _p(hk), _p(hc), len(keys))
        if grades is not None:     # 0 THREAD, 1 QPS (default)
            g = np.ascontiguousarray(grades, dtype=np.int32)
            lib().orc_lparam_set_grades(self.h, _p(g), len(g))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_lparam_free(self.h)

    def replay(self, rule_idx, acquire, ts, vbegin, vcount, values, kinds=None) -> np.ndarray:
        """kinds[i] == 1: an exit (thread counts drop), else a check."""
        r, a, t, b, c, v = _multi_args(rule_idx, acquire, ts, vbegin, vcount, values)
        status = np.zeros(len(t), dtype=np.int8)
        k = None if kinds is None else np.ascontiguousarray(kinds, dtype=np.uint8)
        lib().orc_lparam_replay_ex(self.h, len(t), _p(r), _p(a), _p(t), _p(b), _p(c), _p(v) if len(v) else None,
                                   len(v), _p(k) if k is not None else None, _p(status))
        return status

    def thread_count(self, rule_idx, key) -> int:
        """-1 when the value has no entry in the thread-count map."""
        return lib().orc_lparam_thread_count(self.h, int(rule_idx), int(key))

    def state(self, rule_idx, key):
        last, tok = C.c_int64(), C.c_int64()
        lib().orc_lparam_state(self.h, int(rule_idx), int(key), C.byref(last), C.byref(tok))
        return last.value, tok.value


def default_controller_check(node_value, count, grade, acquire) -> bool:
    return bool(lib().orc_default_controller_check(node_value, count, grade, acquire))


def java_string_hash(s: str) -> int:
    u = np.frombuffer(s.encode("utf-16-le"), dtype=np.uint16).copy()
    return int(lib().orc_java_string_hash(_p(u), len(u)))


def rules_array(rules) -> "C.Array":
    arr = (FlowRule * max(len(rules), 1))()
    for i, r in enumerate(rules):
        arr[i] = FlowRule(int(r["flow_id"]), float(r["count"]), int(r.get("threshold_type", 1)),
                          int(r.get("sample_count", 10)), int(r.get("window_interval_ms", 1000)),
                          int(r.get("namespace_idx", 0)), int(r.get("checker", 0)), 0)
    return arr


class TokenServiceOracle:
    """Sequential DefaultTokenService replay (DefaultTokenService.java:37-62) with an injected clock."""

    def __init__(self, rules, namespaces=None, exceed_count=1.0, max_occupy_ratio=1.0, param_rules=None,
                 hot_items=None):
        namespaces = namespaces if namespaces is not None else [dict(connected_count=0, has_limiter=0, max_allowed_qps=30000.0)]
        ns = (Namespace * max(len(namespaces), 1))()
        for i, n in enumerate(namespaces):
            ns[i] = Namespace(int(n.get("connected_count", 0)), int(n.get("has_limiter", 0)),
                              float(n.get("max_allowed_qps", 30000.0)))
        cfg = ServerConfig(exceed_count, max_occupy_ratio)
        self.h = lib().orc_engine_new(C.byref(cfg), ns, len(namespaces))
        self.rules = list(rules)
        self._rules_c = rules_array(self.rules)
        lib().orc_engine_load_flow_rules(self.h, self._rules_c, len(self.rules))
        if param_rules is not None:
            self.load_param_rules(param_rules, hot_items or {})

    @classmethod
    def from_arrays(cls, flow_id, count, threshold_type, sample_count, window_interval_ms, namespace, checker,
                    namespaces=None, exceed_count=1.0, max_occupy_ratio=1.0):
        """Vectorised constructor for large rule tables (the FlowRule struct is filled from numpy)."""
        self = cls.__new__(cls)
        namespaces = namespaces if namespaces is not None else [dict(connected_count=0, has_limiter=0, max_allowed_qps=30000.0)]
        ns = (Namespace * max(len(namespaces), 1))()
        for i, n in enumerate(namespaces):
            ns[i] = Namespace(int(n.get("connected_count", 0)), int(n.get("has_limiter", 0)),
                              float(n.get("max_allowed_qps", 30000.0)))
        cfg = ServerConfig(exceed_count, max_occupy_ratio)
        self.h = lib().orc_engine_new(C.byref(cfg), ns, len(namespaces))
        n = len(flow_id)
        rec = np.zeros(n, dtype=[("flow_id", "<i8"), ("count", "<f8"), ("threshold_type", "<i4"),
                                 ("sample_count", "<i4"), ("window_interval_ms", "<i4"),
                                 ("namespace_idx", "<i4"), ("checker", "<i4"), ("reserved", "<i4")])
        rec["flow_id"], rec["count"], rec["threshold_type"] = flow_id, count, threshold_type
        rec["sample_count"], rec["window_interval_ms"] = sample_count, window_interval_ms
        rec["namespace_idx"], rec["checker"] = namespace, checker
        self._rec = rec
        self.rules = None
        self._sample_count = np.asarray(sample_count)
        lib().orc_engine_load_flow_rules(self.h, C.c_void_p(rec.ctypes.data), n)
        return self

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_engine_free(self.h)

    def load_param_rules(self, param_rules, hot_items):
        """hot_items: {rule_index: [(key, count), ...]}"""
        keys, counts = [], []
        arr = (ParamRule * max(len(param_rules), 1))()
        for i, r in enumerate(param_rules):
            items = hot_items.get(i, [])
            arr[i] = ParamRule(int(r["flow_id"]), float(r["count"]), int(r.get("threshold_type", 1)),
                               int(r.get("sample_count", 10)), int(r.get("window_interval_ms", 1000)),
                               int(r.get("namespace_idx", 0)), len(keys), len(items))
            for k, c in items:
                keys.append(k)
                counts.append(c)
        hk = np.array(keys if keys else [0], dtype=np.uint64)
        hc = np.array(counts if counts else [0], dtype=np.int32)
        self._param_c = arr
        lib().orc_engine_load_param_rules(self.h, arr, len(param_rules), _p(hk), _p(hc), len(keys))

    def request_token(self, flow_idx, acquire, prioritized, t):
        st, rem, wt = C.c_int8(), C.c_int32(), C.c_int32()
        lib().orc_request_token(self.h, flow_idx, acquire, int(bool(prioritized)), t,
                                C.byref(st), C.byref(rem), C.byref(wt))
        return st.value, rem.value, wt.value

    def replay(self, flow_idx, acquire, ts, flags=None):
        n = len(ts)
        flow_idx = np.ascontiguousarray(flow_idx, dtype=np.int32)
        acquire = np.ascontiguousarray(acquire, dtype=np.int32)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        flags = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint8)
        status = np.zeros(n, dtype=np.int8)
        remaining = np.zeros(n, dtype=np.int32)
        wait = np.zeros(n, dtype=np.int32)
        lib().orc_flow_replay(self.h, n, _p(flow_idx), _p(acquire), _p(flags), _p(ts),
                              _p(status), _p(remaining), _p(wait))
        return status, remaining, wait

    def replay_mt(self, flow_idx, acquire, ts, nthreads, flags=None):
        """Flow-sharded multi-threaded replay; returns (status, remaining, wait, threads_used)."""
        n = len(ts)
        flow_idx = np.ascontiguousarray(flow_idx, dtype=np.int32)
        acquire = np.ascontiguousarray(acquire, dtype=np.int32)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        flags = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint8)
        status = np.zeros(n, dtype=np.int8)
        remaining = np.zeros(n, dtype=np.int32)
        wait = np.zeros(n, dtype=np.int32)
        used = lib().orc_flow_replay_mt(self.h, n, _p(flow_idx), _p(acquire), _p(flags), _p(ts), _p(status),
                                        _p(remaining), _p(wait), int(nthreads))
        return status, remaining, wait, used

    def request_param_token(self, rule_idx, acquire, t, values):
        v = np.ascontiguousarray(values, dtype=np.uint64)
        st, rem = C.c_int8(), C.c_int32()
        lib().orc_request_param_token(self.h, rule_idx, acquire, t, _p(v), len(v), C.byref(st), C.byref(rem))
        return st.value, rem.value

    def set_connected_count(self, ns, connected):
        lib().orc_engine_set_connected_count(self.h, int(ns), int(connected))

    def param_replay(self, rule_idx, acquire, keys, ts):
        n = len(ts)
        rule_idx = np.ascontiguousarray(rule_idx, dtype=np.int32)
        acquire = np.ascontiguousarray(acquire, dtype=np.int32)
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        status = np.zeros(n, dtype=np.int8)
        remaining = np.zeros(n, dtype=np.int32)
        lib().orc_param_replay(self.h, n, _p(rule_idx), _p(acquire), _p(keys), _p(ts), _p(status), _p(remaining))
        return status, remaining

    def param_replay_mt(self, rule_idx, acquire, keys, ts, nthreads):
        """Rule-sharded multi-threaded param replay; returns (status, remaining, threads_used)."""
        n = len(ts)
        rule_idx = np.ascontiguousarray(rule_idx, dtype=np.int32)
        acquire = np.ascontiguousarray(acquire, dtype=np.int32)
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        status = np.zeros(n, dtype=np.int8)
        remaining = np.zeros(n, dtype=np.int32)
        used = lib().orc_param_replay_mt(self.h, n, _p(rule_idx), _p(acquire), _p(keys), _p(ts), _p(status),
                                         _p(remaining), int(nthreads))
        return status, remaining, used

    def param_multi_replay(self, rule_idx, acquire, ts, vbegin, vcount, values):
        r, a, t, b, c, v = _multi_args(rule_idx, acquire, ts, vbegin, vcount, values)
        status = np.zeros(len(t), dtype=np.int8)
        remaining = np.zeros(len(t), dtype=np.int32)
        lib().orc_param_multi_replay(self.h, len(t), _p(r), _p(a), _p(t), _p(b), _p(c), _p(v) if len(v) else None,
                                     len(v), _p(status), _p(remaining))
        return status, remaining

    def param_cm_audit(self, rule_idx, acquire, ts, vbegin, vcount, values, status_cm):
        """(violations, false_blocks, decided) of count-min verdicts replayed on exact counters."""
        r, a, t, b, c, v = _multi_args(rule_idx, acquire, ts, vbegin, vcount, values)
        st = np.ascontiguousarray(status_cm, dtype=np.int8)
        viol, fb, dec = C.c_int64(), C.c_int64(), C.c_int64()
        lib().orc_param_cm_audit(self.h, len(t), _p(r), _p(a), _p(t), _p(b), _p(c), _p(v), _p(st),
                                 C.byref(viol), C.byref(fb), C.byref(dec))
        return viol.value, fb.value, dec.value

    def param_sum(self, rule_idx, t, key):
        return lib().orc_engine_param_sum(self.h, rule_idx, t, key)

    def param_overflowed(self):
        return bool(lib().orc_engine_param_overflowed(self.h))

    def flow_window(self, idx):
        """(sampleCount, intervalMs) of the metric behind dense flow index idx (its window, which a
        reload keeps even when the rule's window changed)."""
        w = np.zeros(2, dtype=np.int32)
        if lib().orc_engine_flow_window(self.h, int(idx), _p(w)) < 0:
            raise ValueError("no metric for flow index %d" % idx)
        return int(w[0]), int(w[1])

    def dump_flow(self, idx) -> np.ndarray:
        n = self.flow_window(idx)[0]
        out = np.zeros(n * 8 + 8, dtype=np.int64)
        w = lib().orc_engine_dump_flow(self.h, idx, _p(out))
        if w < 0:
            raise ValueError("no metric for flow index %d" % idx)
        return out

    def reload_flow_rules(self, rules):
        """ClusterFlowRuleManager.loadRules again: surviving flowIds keep their ClusterMetric (old
        window and counters) and nowCalls; returns the number of dense flows."""
        self.rules = None
        self._rules_c = rules_array(list(rules))
        return lib().orc_engine_load_flow_rules(self.h, self._rules_c, len(rules))

    def reset_metrics(self, sample_count, interval_ms):
        """Server window change (ClusterServerConfigManager.java:333-343): every metric restarts."""
        return lib().orc_engine_reset_metrics(self.h, int(sample_count), int(interval_ms))

    def metric_count(self):
        return lib().orc_engine_metric_count(self.h)

    def param_top_values(self, rule_idx, t, number=5):
        keys = np.zeros(max(number, 1), dtype=np.uint64)
        avgs = np.zeros(max(number, 1), dtype=np.float64)
        k = lib().orc_engine_param_top_values(self.h, int(rule_idx), int(t), int(number), _p(keys), _p(avgs))
        return [(int(keys[i]), float(avgs[i])) for i in range(k)]

    def param_window(self, idx):
        w = np.zeros(2, dtype=np.int32)
        if lib().orc_engine_param_window(self.h, int(idx), _p(w)) < 0:
            raise ValueError("no param metric for rule index %d" % idx)
        return int(w[0]), int(w[1])

    CONC_EVENT = np.dtype([("flow_idx", "<i4"), ("acquire", "<i4"), ("token_id", "<i8"), ("kind", "<i4"),
                           ("flags", "<u4")])

    def concurrent_replay(self, events: np.ndarray, new_ids):
        """ConcurrentClusterFlowChecker replay; events in CONC_EVENT layout; returns (status, token_id)."""
        ev = np.ascontiguousarray(events, dtype=self.CONC_EVENT)
        ids = np.ascontiguousarray(new_ids, dtype=np.int64)
        st = np.zeros(len(ev), dtype=np.int8)
        tok = np.zeros(len(ev), dtype=np.int64)
        lib().orc_concurrent_replay(self.h, len(ev), _p(ev), _p(ids), _p(st), _p(tok))
        return st, tok

    def concurrent_replay_mt(self, events: np.ndarray, new_ids, nthreads):
        """Flow-sharded multi-threaded concurrency replay on a fresh oracle (own token cache per thread,
        releases routed to the thread that issued their token); returns (status, token_id, threads_used)."""
        ev = np.ascontiguousarray(events, dtype=self.CONC_EVENT)
        ids = np.ascontiguousarray(new_ids, dtype=np.int64)
        st = np.zeros(len(ev), dtype=np.int8)
        tok = np.zeros(len(ev), dtype=np.int64)
        used = lib().orc_concurrent_replay_mt(self.h, len(ev), _p(ev), _p(ids), _p(st), _p(tok), int(nthreads))
        return st, tok, used

    def concurrent_now_calls(self, idx): return lib().orc_concurrent_now_calls(self.h, idx)
    def concurrent_token_count(self): return lib().orc_concurrent_token_count(self.h)
    def concurrent_expire_all(self): return lib().orc_concurrent_expire_all(self.h)

    def limiter_sum(self, ns, t):
        return lib().orc_engine_limiter_sum(self.h, ns, t)


class LocalGraph:
    """orc_lgraph: FlowRuleChecker node selection over ClusterNode / origin / DefaultNode
    (FlowRuleChecker.java:44-145, StatisticSlot.java:55-164)."""

    RULE_DTYPE = np.dtype([("resource", "<i4"), ("grade", "<i4"), ("count", "<f8"), ("strategy", "<i4"),
                           ("limit_app", "<i4"), ("ref", "<i4"), ("reserved", "<i4")])
    CTX_DTYPE = np.dtype([("origin", "<i4"), ("origin_node", "<i4"), ("context", "<i4"), ("default_node", "<i4")])

    def __init__(self, rules, n_res, n_origin_nodes, n_default_nodes, sample_count=2, interval_ms=1000):
        arr = np.ascontiguousarray(rules, dtype=self.RULE_DTYPE)
        self.h = lib().orc_lgraph_new(_p(arr) if len(arr) else None, len(arr), n_res, n_origin_nodes,
                                      n_default_nodes, sample_count, interval_ms)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_lgraph_free(self.h)
            self.h = None

    def set_occupy_timeout(self, ms): lib().orc_lgraph_set_occupy_timeout(self.h, ms)
    def n_rules(self, res): return lib().orc_lgraph_n_rules(self.h, res)

    def replay(self, res, acquire, ts, ctx, flags=None, rt=None):
        res = np.ascontiguousarray(res, dtype=np.int32)
        acquire = np.ascontiguousarray(acquire, dtype=np.int32)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        cx = np.ascontiguousarray(ctx, dtype=self.CTX_DTYPE)
        fl = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint8)
        r = None if rt is None else np.ascontiguousarray(rt, dtype=np.int64)
        st = np.zeros(len(res), dtype=np.int8)
        wait = np.zeros(len(res), dtype=np.int32)
        lib().orc_lgraph_replay(self.h, len(res), _p(res), _p(acquire), _p(ts), _p(cx), _p(fl), _p(r), _p(st), _p(wait))
        return st, wait.astype(np.int64)

    def node_metrics(self, kind, idx, t) -> np.ndarray:
        out = np.zeros(14, dtype=np.int64)
        if lib().orc_lgraph_node_metrics(self.h, kind, idx, t, _p(out)) != 0:
            raise IndexError("bad node")
        return out
