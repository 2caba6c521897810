"""ctypes binding of libsentinel_amd.so (the C ABI declared in include/sentinel_amd.h).

The product path: there is no CPU fallback.  If the HIP library is missing or cannot load, every
entry point raises -- it never routes through the oracle.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SENTINEL_LIB") or os.path.join(_HERE, "libsentinel_amd.so")

STATUS_BAD_REQUEST = -4
STATUS_TOO_MANY_REQUEST = -2
STATUS_FAIL = -1
STATUS_OK = 0
STATUS_BLOCKED = 1
STATUS_SHOULD_WAIT = 2
STATUS_NO_RULE_EXISTS = 3

IDX_NO_RULE = -1
IDX_BAD_ID = -2

THRESHOLD_AVG_LOCAL = 0
THRESHOLD_GLOBAL = 1
CHECKER_CLUSTER = 0
CHECKER_SIMPLE = 1
FLAG_PRIORITIZED = 1

# every symbol include/sentinel_amd.h declares
EXPORTS = [
    "sentinel_engine_create", "sentinel_engine_destroy", "sentinel_last_error", "sentinel_device_count",
    "sentinel_set_server_config", "sentinel_set_namespaces", "sentinel_set_connected_count",
    "sentinel_load_flow_rules", "sentinel_load_param_rules", "sentinel_flow_count",
    "sentinel_lookup_flow_idx", "sentinel_lookup_param_idx",
    "sentinel_submit_flow_batch", "sentinel_submit_flow_batch_host", "sentinel_submit_flow_stream_host",
    "sentinel_submit_flow_batch_ordered", "sentinel_submit_flow_batch_ordered_host",
    "sentinel_submit_param_batch", "sentinel_submit_param_batch_host",
    "sentinel_submit_param_batch_ordered", "sentinel_submit_param_batch_ordered_host",
    "sentinel_request_token", "sentinel_request_param_token",
    "sentinel_synchronize", "sentinel_dump_flow", "sentinel_param_sum",
    "sentinel_snapshot", "sentinel_snapshot_device", "sentinel_engine_stream",
    "sentinel_profile_enable", "sentinel_profile_read",
    "sentinel_batcher_create", "sentinel_batcher_destroy", "sentinel_batcher_request_token", "sentinel_batcher_stats",
    "sentinel_submit_param_multi_batch", "sentinel_submit_param_multi_batch_host", "sentinel_set_param_mode",
    "sentinel_load_local_param_rules", "sentinel_submit_local_param_batch", "sentinel_submit_local_param_batch_host",
    "sentinel_local_param_state",
    "sentinel_submit_concurrent_batch_host", "sentinel_submit_concurrent_batch", "sentinel_concurrent_now_calls",
    "sentinel_concurrent_token_count",
    "sentinel_concurrent_expire",
    "sentinel_load_local_resources", "sentinel_submit_local_entry_batch", "sentinel_submit_local_entry_batch_host",
    "sentinel_local_node_stats", "sentinel_set_occupy_timeout", "sentinel_profile_select", "sentinel_profile_gate", "sentinel_set_flow_path",
    "sentinel_param_top_values", "sentinel_param_snapshot_device", "sentinel_flow_window", "sentinel_metric_count",
    "sentinel_reset_metrics", "sentinel_param_table_stats", "sentinel_param_cm_stats", "sentinel_param_cm_block_batches", "sentinel_flow_path_stats", "sentinel_param_count",
    "sentinel_batcher_request_token_async", "sentinel_submit_flow_batches", "sentinel_profile_every",
    "sentinel_set_local_param_grades", "sentinel_submit_local_param_batch_ex", "sentinel_submit_local_param_batch_ex_host",
    "sentinel_load_local_resources_ex", "sentinel_submit_local_batch", "sentinel_submit_local_batch_host",
    "sentinel_local_node_metrics", "sentinel_set_statistic_max_rt",
    "sentinel_load_local_rules", "sentinel_submit_local_graph_batch", "sentinel_submit_local_graph_batch_host",
    "sentinel_local_graph_node_metrics",
    "sentinel_shard_of", "sentinel_cluster_create", "sentinel_cluster_destroy", "sentinel_cluster_size",
    "sentinel_cluster_engine", "sentinel_cluster_set_server_config", "sentinel_cluster_set_namespaces",
    "sentinel_cluster_set_connected_count", "sentinel_cluster_load_flow_rules", "sentinel_cluster_load_param_rules",
    "sentinel_cluster_submit_host", "sentinel_cluster_flow_count", "sentinel_cluster_snapshot",
    "sentinel_cluster_batchers_create", "sentinel_cluster_request_token",
    "sentinel_batcher_request_tokens_async", "sentinel_batcher_set_batch_hook",
    "sentinel_param_interner_create", "sentinel_param_interner_destroy", "sentinel_param_interner_key",
    "sentinel_param_interner_key_at", "sentinel_param_interner_set_limits", "sentinel_param_interner_stats", "sentinel_param_interner_scans",
    "sentinel_wire_server_create", "sentinel_wire_server_port", "sentinel_wire_server_stats",
    "sentinel_wire_server_destroy",
]

STATUS_RELEASE_OK = 6
STATUS_ALREADY_RELEASE = 7
CONCURRENT_ACQUIRE = 0
CONCURRENT_RELEASE = 1

PARAM_EXACT = 0
PARAM_COUNT_MIN = 1
PARAM_COUNT_MIN_SHARED = 2


class ServerConfig(C.Structure):
    _fields_ = [("exceed_count", C.c_double), ("max_occupy_ratio", C.c_double)]


CLOCK_FN = C.CFUNCTYPE(C.c_int64, C.c_void_p)


class WireConfig(C.Structure):
    _fields_ = [("host", C.c_char_p), ("port", C.c_int32), ("io_threads", C.c_int32), ("max_batch", C.c_int32),
                ("max_wait_us", C.c_int32), ("namespaces", C.POINTER(C.c_char_p)), ("n_namespaces", C.c_int32),
                ("interner", C.c_void_p), ("clock", CLOCK_FN), ("clock_ctx", C.c_void_p)]


class Namespace(C.Structure):
    _fields_ = [("connected_count", C.c_int32), ("has_limiter", C.c_int32), ("max_allowed_qps", C.c_double)]


class FlowRuleC(C.Structure):
    _fields_ = [("flow_id", C.c_int64), ("count", C.c_double), ("threshold_type", C.c_int32),
                ("sample_count", C.c_int32), ("window_interval_ms", C.c_int32),
                ("namespace_idx", C.c_int32), ("checker", C.c_int32), ("reserved", C.c_int32)]


class ParamRuleC(C.Structure):
    _fields_ = [("flow_id", C.c_int64), ("count", C.c_double), ("threshold_type", C.c_int32),
                ("sample_count", C.c_int32), ("window_interval_ms", C.c_int32),
                ("namespace_idx", C.c_int32), ("hot_begin", C.c_int32), ("hot_n", C.c_int32)]


class LocalParamRuleC(C.Structure):
    _fields_ = [("count", C.c_double), ("burst_count", C.c_int64), ("duration_in_sec", C.c_int64),
                ("hot_begin", C.c_int32), ("hot_n", C.c_int32)]


class LocalResourceExC(C.Structure):
    _fields_ = [("qps_count", C.c_double), ("thread_count", C.c_double), ("flags", C.c_int32),
                ("reserved", C.c_int32)]


LOCAL_QPS, LOCAL_THREAD, LOCAL_THREAD_FIRST = 1, 2, 4
LOCAL_PRIO, LOCAL_EXIT, LOCAL_ERROR = 1, 2, 4


class LocalResourceC(C.Structure):
    _fields_ = [("count", C.c_double), ("has_rule", C.c_int32), ("reserved", C.c_int32)]


class TokenResultC(C.Structure):
    _fields_ = [("status", C.c_int32), ("remaining", C.c_int32), ("wait_in_ms", C.c_int32), ("reserved", C.c_int32)]


class FlowSnapshotC(C.Structure):
    _fields_ = [("flow_id", C.c_int64), ("pass_qps", C.c_double), ("block_qps", C.c_double)]


# AoS records of include/sentinel_amd.h
EVENT_DTYPE = np.dtype([("flow_idx", "<i4"), ("acquire", "<i4"), ("ts", "<i8")])
PARAM_EVENT_DTYPE = np.dtype([("rule_idx", "<i4"), ("acquire", "<i4"), ("ts", "<i8"), ("param_key", "<u8")])
MULTI_EVENT_DTYPE = np.dtype([("rule_idx", "<i4"), ("acquire", "<i4"), ("ts", "<i8"), ("value_begin", "<i4"),
                              ("value_count", "<i4")])
CONC_EVENT_DTYPE = np.dtype([("flow_idx", "<i4"), ("acquire", "<i4"), ("token_id", "<i8"), ("kind", "<i4"),
                             ("flags", "<u4")])
CONC_RESULT_DTYPE = np.dtype([("token_id", "<i8"), ("status", "<i4"), ("reserved", "<i4")])
VERDICT_DTYPE = np.dtype([("remaining", "<i4"), ("status", "<i2"), ("wait_in_ms", "<u2")])
# sentinel_local_rule_t / sentinel_local_ctx_t (local rule graph)
LOCAL_RULE_DTYPE = np.dtype([("resource", "<i4"), ("grade", "<i4"), ("count", "<f8"), ("strategy", "<i4"),
                             ("limit_app", "<i4"), ("ref", "<i4"), ("reserved", "<i4")])
LOCAL_CTX_DTYPE = np.dtype([("origin", "<i4"), ("origin_node", "<i4"), ("context", "<i4"), ("default_node", "<i4")])
LIMIT_APP_DEFAULT, LIMIT_APP_OTHER = 0, 1
STRATEGY_DIRECT, STRATEGY_RELATE, STRATEGY_CHAIN = 0, 1, 2
NODE_CLUSTER, NODE_ORIGIN, NODE_DEFAULT = 0, 1, 2
TOP_PARAMS = 5
PARAM_SNAPSHOT_DTYPE = np.dtype([("flow_id", "<i8"), ("n_top", "<i4"), ("reserved", "<i4"),
                                 ("key", "<u8", (TOP_PARAMS,)), ("avg", "<f8", (TOP_PARAMS,))])


class SentinelError(RuntimeError):
    pass


_lib = None


def load():
    """Load the HIP engine; raises SentinelError when it is absent (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    try:   # share one HIP runtime with PyTorch when it is present (both sonames are libamdhip64.so.7)
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise SentinelError(f"{LIB_PATH} not built: run `python __graft_entry__.py build` (hipcc, gfx950)")
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64
    sig = {
        "sentinel_engine_create": (C.c_int, [C.c_int, vp, C.POINTER(vp)]),
        "sentinel_engine_destroy": (C.c_int, [vp]),
        "sentinel_last_error": (C.c_char_p, []),
        "sentinel_device_count": (C.c_int, []),
        "sentinel_set_server_config": (C.c_int, [vp, vp]),
        "sentinel_set_namespaces": (C.c_int, [vp, vp, i32]),
        "sentinel_set_connected_count": (C.c_int, [vp, i32, i32]),
        "sentinel_load_flow_rules": (C.c_int, [vp, vp, i32]),
        "sentinel_load_param_rules": (C.c_int, [vp, vp, i32, vp, vp, i32]),
        "sentinel_flow_count": (i32, [vp]),
        "sentinel_lookup_flow_idx": (C.c_int, [vp, i64, vp, vp]),
        "sentinel_lookup_param_idx": (C.c_int, [vp, i64, vp, vp]),
        "sentinel_submit_flow_batch": (C.c_int, [vp, i64, vp, vp, vp, vp]),
        "sentinel_submit_flow_batch_host": (C.c_int, [vp, i64, vp, vp, vp]),
        "sentinel_submit_flow_batch_ordered": (C.c_int, [vp, i64, vp, vp, vp, vp, vp]),
        "sentinel_submit_flow_batch_ordered_host": (C.c_int, [vp, i64, vp, vp, vp, vp]),
        "sentinel_submit_flow_stream_host": (C.c_int, [vp, i64, vp, vp, vp, i64, vp]),
        "sentinel_submit_param_batch": (C.c_int, [vp, i64, vp, vp, vp]),
        "sentinel_submit_param_batch_host": (C.c_int, [vp, i64, vp, vp]),
        "sentinel_submit_param_batch_ordered": (C.c_int, [vp, i64, vp, vp, vp, vp]),
        "sentinel_submit_param_batch_ordered_host": (C.c_int, [vp, i64, vp, vp, vp]),
        "sentinel_request_token": (C.c_int, [vp, i64, i32, i32, i64, vp]),
        "sentinel_request_param_token": (C.c_int, [vp, i64, i32, u64, i64, vp]),
        "sentinel_synchronize": (C.c_int, [vp]),
        "sentinel_dump_flow": (C.c_int, [vp, i32, vp, i32]),
        "sentinel_param_sum": (C.c_int, [vp, i32, u64, i64, vp]),
        "sentinel_snapshot": (C.c_int, [vp, i64, vp]),
        "sentinel_snapshot_device": (C.c_int, [vp, i64, vp, vp]),
        "sentinel_engine_stream": (vp, [vp]),
        "sentinel_profile_enable": (C.c_int, [vp, C.c_int]),
        "sentinel_profile_read": (C.c_int, [vp, C.c_int, vp, vp, vp, vp]),
        "sentinel_batcher_create": (C.c_int, [vp, i32, i32, C.POINTER(vp)]),
        "sentinel_batcher_destroy": (C.c_int, [vp]),
        "sentinel_batcher_request_token": (C.c_int, [vp, i64, i32, i32, i64, vp]),
        "sentinel_batcher_stats": (C.c_int, [vp, vp, vp]),
        "sentinel_submit_param_multi_batch": (C.c_int, [vp, i64, vp, vp, i64, vp, vp]),
        "sentinel_submit_param_multi_batch_host": (C.c_int, [vp, i64, vp, vp, i64, vp]),
        "sentinel_set_param_mode": (C.c_int, [vp, i32, i32, i32]),
        "sentinel_load_local_param_rules": (C.c_int, [vp, vp, i32, vp, vp, i32]),
        "sentinel_submit_local_param_batch": (C.c_int, [vp, i64, vp, vp, i64, vp, vp]),
        "sentinel_submit_local_param_batch_host": (C.c_int, [vp, i64, vp, vp, i64, vp]),
        "sentinel_local_param_state": (C.c_int, [vp, u64, vp, vp]),
        "sentinel_submit_concurrent_batch_host": (C.c_int, [vp, i64, vp, vp]),
        "sentinel_submit_concurrent_batch": (C.c_int, [vp, i64, vp, vp, vp]),
        "sentinel_concurrent_now_calls": (C.c_int, [vp, i32, vp]),
        "sentinel_concurrent_token_count": (C.c_int, [vp, vp]),
        "sentinel_concurrent_expire": (C.c_int, [vp, i64, vp]),
        "sentinel_load_local_resources": (C.c_int, [vp, vp, i32, i32, i32]),
        "sentinel_submit_local_entry_batch": (C.c_int, [vp, i64, vp, vp, vp, vp]),
        "sentinel_submit_local_entry_batch_host": (C.c_int, [vp, i64, vp, vp, vp]),
        "sentinel_local_node_stats": (C.c_int, [vp, i32, i64, vp]),
        "sentinel_set_occupy_timeout": (C.c_int, [vp, i32]),
        "sentinel_set_local_param_grades": (C.c_int, [vp, vp, i32]),
        "sentinel_submit_local_param_batch_ex": (C.c_int, [vp, i64, vp, vp, vp, i64, vp, vp]),
        "sentinel_submit_local_param_batch_ex_host": (C.c_int, [vp, i64, vp, vp, vp, i64, vp]),
        "sentinel_load_local_resources_ex": (C.c_int, [vp, vp, i32, i32, i32]),
        "sentinel_submit_local_batch": (C.c_int, [vp, i64, vp, vp, vp, vp, vp]),
        "sentinel_submit_local_batch_host": (C.c_int, [vp, i64, vp, vp, vp, vp]),
        "sentinel_local_node_metrics": (C.c_int, [vp, i32, i64, vp]),
        "sentinel_load_local_rules": (C.c_int, [vp, vp, i32, i32, i32, i32, i32, i32]),
        "sentinel_submit_local_graph_batch": (C.c_int, [vp, i64, vp, vp, vp, vp, vp, vp]),
        "sentinel_submit_local_graph_batch_host": (C.c_int, [vp, i64, vp, vp, vp, vp, vp]),
        "sentinel_local_graph_node_metrics": (C.c_int, [vp, i32, i32, i64, vp]),
        "sentinel_set_statistic_max_rt": (C.c_int, [vp, i64]),
        "sentinel_submit_flow_batches": (C.c_int, [vp, i32, vp, vp, vp, vp, vp]),
        "sentinel_profile_every": (C.c_int, [vp, i32]),
        "sentinel_shard_of": (i32, [i64, i32]),
        "sentinel_cluster_create": (C.c_int, [vp, i32, vp, vp]),
        "sentinel_cluster_destroy": (C.c_int, [vp]),
        "sentinel_cluster_size": (i32, [vp]),
        "sentinel_cluster_engine": (C.c_int, [vp, i32, vp]),
        "sentinel_cluster_set_server_config": (C.c_int, [vp, vp]),
        "sentinel_cluster_set_namespaces": (C.c_int, [vp, vp, i32]),
        "sentinel_cluster_set_connected_count": (C.c_int, [vp, i32, i32]),
        "sentinel_cluster_load_flow_rules": (C.c_int, [vp, vp, i32]),
        "sentinel_cluster_load_param_rules": (C.c_int, [vp, vp, i32, vp, vp, i32]),
        "sentinel_cluster_submit_host": (C.c_int, [vp, i64, vp, vp, vp, vp, vp]),
        "sentinel_cluster_flow_count": (i32, [vp]),
        "sentinel_cluster_snapshot": (C.c_int, [vp, i64, vp, i64, vp]),
        "sentinel_cluster_batchers_create": (C.c_int, [vp, i32, i32]),
        "sentinel_cluster_request_token": (C.c_int, [vp, i64, i32, i32, i64, vp]),
        "sentinel_profile_select": (C.c_int, [vp, C.c_char_p]),
        "sentinel_profile_gate": (C.c_int, [vp, C.c_int]),
        "sentinel_set_flow_path": (C.c_int, [vp, C.c_int]),
        "sentinel_param_top_values": (C.c_int, [vp, i64, i32, vp, vp, vp]),
        "sentinel_param_snapshot_device": (C.c_int, [vp, i64, vp, vp]),
        "sentinel_flow_window": (C.c_int, [vp, i32, vp, vp]),
        "sentinel_metric_count": (i64, [vp]),
        "sentinel_reset_metrics": (C.c_int, [vp, i32, i32]),
        "sentinel_param_table_stats": (C.c_int, [vp, vp]),
        "sentinel_param_cm_stats": (C.c_int, [vp, vp]),
        "sentinel_flow_path_stats": (C.c_int, [vp, vp]),
        "sentinel_param_cm_block_batches": (C.c_int, [vp, vp]),
        "sentinel_param_count": (i32, [vp]),
        "sentinel_batcher_request_token_async": (C.c_int, [vp, i64, i32, i32, i64, vp, vp, C.c_uint64]),
        "sentinel_param_interner_create": (C.c_int, [C.POINTER(vp)]),
        "sentinel_param_interner_destroy": (C.c_int, [vp]),
        "sentinel_param_interner_key": (C.c_int, [vp, i64, i32, vp, i32, C.POINTER(C.c_uint64)]),
        "sentinel_param_interner_key_at": (C.c_int, [vp, i64, i32, vp, i32, i64, C.POINTER(C.c_uint64)]),
        "sentinel_param_interner_set_limits": (C.c_int, [vp, i64, i64]),
        "sentinel_param_interner_stats": (C.c_int, [vp, C.POINTER(i64), C.POINTER(i64)]),
        "sentinel_param_interner_scans": (C.c_int, [vp, C.POINTER(i64)]),
        "sentinel_wire_server_create": (C.c_int, [vp, C.POINTER(WireConfig), C.POINTER(vp)]),
        "sentinel_wire_server_port": (i32, [vp]),
        "sentinel_wire_server_stats": (C.c_int, [vp, vp, vp, vp, vp]),
        "sentinel_wire_server_destroy": (C.c_int, [vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc < 0:
        msg = load().sentinel_last_error()
        raise SentinelError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
