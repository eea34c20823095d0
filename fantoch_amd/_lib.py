"""ctypes binding of libfantoch_hip.so (the C ABI in include/fantoch_hip.h).

The product path is the HIP library: there is no CPU fallback.  If the shared
library is missing or fails to load this module raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libfantoch_hip.so")

FH_OK, FH_EINVAL, FH_EHIP, FH_EOOM, FH_EINVARIANT, FH_ECAP, FH_ENOTIMPL = range(7)
FH_STREAM_ELEMENT_LOGS = 1  # fh_stream_desc.flags (include/fantoch_hip.h)
FH_REPLY_INFO, FH_REPLY_EXECUTED = 0, 1  # RequestReply kinds (include/fantoch_hip.h)
# execution-log event kinds (include/fantoch_hip.h)
FH_LOG_ADD, FH_LOG_REQUEST, FH_LOG_REPLY_INFO, FH_LOG_REPLY_EXECUTED, FH_LOG_EXECUTED = range(5)
STATUS_NAMES = ["FH_OK", "FH_EINVAL", "FH_EHIP", "FH_EOOM", "FH_EINVARIANT", "FH_ECAP",
                "FH_ENOTIMPL"]


class FhError(RuntimeError):
    def __init__(self, status: int, msg: str):
        name = STATUS_NAMES[status] if 0 <= status < len(STATUS_NAMES) else str(status)
        super().__init__(f"{name}: {msg}")
        self.status = status


class fh_config(C.Structure):
    _fields_ = [("n", C.c_uint32), ("f", C.c_uint32), ("shard_count", C.c_uint32),
                ("device", C.c_int32), ("key_space", C.c_uint64)]


class fh_stream_desc(C.Structure):
    _fields_ = [("n", C.c_size_t), ("keys_per_cmd", C.c_uint32), ("views", C.c_uint32),
                ("nproc", C.c_uint32), ("flags", C.c_uint32)]


class fh_workload(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("n", C.c_uint32), ("keys_per_cmd", C.c_uint32),
                ("kind", C.c_uint32), ("conflict_rate", C.c_uint32), ("pool_size", C.c_uint32),
                ("clients", C.c_uint32), ("zipf_s", C.c_double), ("key_count", C.c_uint64),
                ("views", C.c_uint32), ("window", C.c_uint32),
                ("shards", C.c_uint32), ("pad", C.c_uint32)]


V, S, P = C.c_void_p, C.c_size_t, C.POINTER

# name -> (restype, argtypes); every symbol declared in include/fantoch_hip.h
SIGNATURES = {
    "fh_version": (C.c_char_p, []),
    "fh_last_error": (C.c_char_p, []),
    "fh_device_count": (C.c_int, [P(C.c_int)]),
    "fh_keydeps_create": (C.c_int, [C.c_uint64, P(fh_config), P(V)]),
    "fh_keydeps_destroy": (C.c_int, [V]),
    "fh_keydeps_add_batch": (C.c_int, [V, S, V, V, V, V, V, V, V, V, S, P(S)]),
    "fh_keydeps_cmd_deps": (C.c_int, [V, S, V, V, S, P(S)]),
    "fh_keydeps_noop_deps": (C.c_int, [V, V, S, P(S)]),
    "fh_dep_union": (C.c_int, [C.c_int, S, S, V, V, V, V, P(S), V]),
    "fh_keydeps_add_batch_device": (C.c_int, [V, S, S, V, V, V, V, V, S, P(S), V]),
    "fh_keydeps_add_batch_rw": (C.c_int, [V, S, V, V, V, V, V, V, V, V, V, S, P(S)]),
    "fh_keyclocks_create": (C.c_int, [C.c_uint32, C.c_uint64, P(fh_config), P(V)]),
    "fh_keyclocks_destroy": (C.c_int, [V]),
    "fh_keyclocks_clock_next": (C.c_int, [V, P(C.c_uint64)]),
    "fh_keyclocks_clock_join": (C.c_int, [V, C.c_uint64]),
    "fh_keyclocks_add": (C.c_int, [V, S, V, V, V, V]),
    "fh_keyclocks_remove": (C.c_int, [V, S, V, V, V]),
    "fh_keyclocks_predecessors": (C.c_int, [V, S, V, V, V, V, V, V, S, P(S), V, V, S, P(S)]),
    "fh_keyclocks_len": (C.c_int, [V, P(S)]),
    "fh_pred_create": (C.c_int, [C.c_uint32, C.c_uint64, P(fh_config), P(V)]),
    "fh_pred_destroy": (C.c_int, [V]),
    "fh_pred_add_batch": (C.c_int, [V, S, V, V, V, V]),
    "fh_pred_drain": (C.c_int, [V, V, S, P(S)]),
    "fh_pred_pending": (C.c_int, [V, P(S)]),
    "fh_graph_create": (C.c_int, [C.c_uint32, C.c_uint64, P(fh_config), P(V)]),
    "fh_graph_destroy": (C.c_int, [V]),
    "fh_graph_add_batch": (C.c_int, [V, S, V, V, V, V, V]),
    "fh_graph_drain": (C.c_int, [V, V, V, S, P(S)]),
    "fh_graph_mark_executed": (C.c_int, [V, S, V]),
    "fh_graph_set_executed_frontier": (C.c_int, [V, C.c_uint32, C.c_uint64]),
    "fh_graph_pending": (C.c_int, [V, P(S)]),
    "fh_graph_set_time": (C.c_int, [V, C.c_uint64]),
    "fh_graph_monitor_pending": (C.c_int, [V, C.c_uint64, V, V, V, S, P(S)]),
    "fh_graph_take_metrics": (C.c_int, [V, V, S, V, S, P(S), P(S)]),
    "fh_graph_passes": (C.c_int, [V, P(C.c_uint64), P(C.c_uint64)]),
    "fh_graph_missing": (C.c_int, [V, V, S, P(S)]),
    "fh_graph_inject_small_delay": (C.c_int, [V, C.c_uint32, C.c_uint32]),
    "fh_selftest_poll_deadline": (C.c_int, [C.c_uint32]),
    "fh_graph_add_batch_sharded": (C.c_int, [V, S, V, V, V, V, V, V, V]),
    "fh_graph_requests": (C.c_int, [V, V, V, S, P(S)]),
    "fh_graph_handle_requests": (C.c_int, [V, C.c_uint64, S, V]),
    "fh_graph_cleanup": (C.c_int, [V]),
    "fh_graph_request_replies": (C.c_int, [V, S, V, V, V, V, V, S, V, V, P(S), P(S)]),
    "fh_execlog_parse": (C.c_int, [V, S, C.c_uint64, P(V)]),
    "fh_execlog_destroy": (C.c_int, [V]),
    "fh_execlog_sizes": (C.c_int, [V, P(S), P(S), P(S), P(S), P(S)]),
    "fh_execlog_events": (C.c_int, [V, V, V, V, V, V, V, V, V, V, V, V]),
    "fh_execlog_key": (C.c_int, [V, C.c_uint64, V, S, P(S)]),
    "fh_execlog_replay": (C.c_int, [V, V, S, P(S)]),
    "fh_engine_create": (C.c_int, [P(fh_config), P(V)]),
    "fh_engine_destroy": (C.c_int, [V]),
    "fh_engine_reset": (C.c_int, [V]),
    "fh_engine_stage": (C.c_int, [V, P(fh_stream_desc), V, V, V, V]),
    "fh_engine_stage_many": (C.c_int, [V, P(fh_stream_desc), S, V, V, V, V]),
    "fh_engine_stage_logs": (C.c_int, [V, P(fh_stream_desc), S, V, V, V, V]),
    "fh_engine_run": (C.c_int, [V, P(C.c_float)]),
    "fh_engine_results": (C.c_int, [V, V, V, S, P(S), V, V, V, V]),
    "fh_engine_kernel_times": (C.c_int, [V, P(C.c_char_p), P(C.c_float), S, P(S)]),
    "fh_engine_set_profiling": (C.c_int, [V, C.c_int]),
    "fh_engine_set_deps_only": (C.c_int, [V, C.c_int]),
    "fh_engine_forget_tuning": (C.c_int, [V]),
    "fh_engine_set_probe": (C.c_int, [V, C.c_char_p]),
    "fh_engine_probe_stats": (C.c_int, [V, P(C.c_float), P(S), P(C.c_double)]),
    "fh_engine_probe_stats_for": (C.c_int, [V, C.c_char_p, P(C.c_float), P(S), P(C.c_double)]),
    "fh_multi_create": (C.c_int, [P(fh_config), S, V, P(V)]),
    "fh_multi_destroy": (C.c_int, [V]),
    "fh_multi_stage_logs": (C.c_int, [V, P(fh_stream_desc), V, V, V, V]),
    "fh_multi_rewind": (C.c_int, [V]),
    "fh_multi_sync": (C.c_int, [V]),
    "fh_multi_run": (C.c_int, [V, P(C.c_float)]),
    "fh_multi_results": (C.c_int, [V, V, V, S, P(S), V, V, V, V]),
    "fh_multi_shard_size": (C.c_int, [V, S, P(S)]),
    "fh_multi_owners": (C.c_int, [V, V]),
    "fh_key_owners_balanced": (C.c_int, [V, S, C.c_uint32, V]),
    "fh_workload_key_space": (C.c_uint64, [P(fh_workload)]),
    "fh_workload_generate": (C.c_int, [P(fh_workload), C.c_uint64, S, V, V, V, V]),
    "fh_workload_generate_logs": (C.c_int, [P(fh_workload), C.c_uint64, S, V, V]),
    "fh_workload_generate_element_logs": (C.c_int, [P(fh_workload), C.c_uint64, S, V, V]),
    "fh_workload_generate_shard": (C.c_int, [P(fh_workload), C.c_uint64, S, C.c_uint32,
                                             C.c_uint32, P(S), V, V, V, V]),
    "fh_workload_generate_shard_owned": (C.c_int, [P(fh_workload), C.c_uint64, S, V,
                                                   C.c_uint32, C.c_uint32, P(S), V, V, V, V]),
    "fh_workload_key_histogram": (C.c_int, [P(fh_workload), C.c_uint64, S, V]),
    "fh_dgraph_create": (C.c_int, [P(fh_config), C.c_uint32, C.c_uint32, P(V)]),
    "fh_dgraph_destroy": (C.c_int, [V]),
    "fh_dgraph_stage": (C.c_int, [V, P(fh_stream_desc), C.c_uint32, V, V, V, V, V, V, V]),
    "fh_dgraph_keydeps": (C.c_int, [V, V]),
    "fh_dgraph_local": (C.c_int, [V, V, V]),
    "fh_dgraph_queries": (C.c_int, [V, V]),
    "fh_dgraph_answer": (C.c_int, [V, S, V, V]),
    "fh_dgraph_condense": (C.c_int, [V, V, P(C.c_uint64), P(C.c_uint64)]),
    "fh_dgraph_condensed_part": (C.c_int, [V, V, V]),
    "fh_dgraph_solve": (C.c_int, [V, S, V, S, V, V]),
    "fh_dgraph_elements": (C.c_int, [V, V]),
    "fh_dgraph_per_key": (C.c_int, [V, S, V]),
    "fh_dgraph_results": (C.c_int, [V, V, V, S, P(S), V, V, V, P(S)]),
    "fh_dgraph_set_profiling": (C.c_int, [V, C.c_int]),
    "fh_dgraph_stage_times": (C.c_int, [V, P(C.c_char_p), P(C.c_float), S, P(S)]),
    "fh_engine_rewind": (C.c_int, [V]),
    "fh_engine_sync": (C.c_int, [V]),
}

_lib = None


def load(path: str = LIB_PATH):
    """Load the HIP library (raises if it is missing: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found: build it with `python -m fantoch_amd.build` "
            "(the HIP engine has no CPU fallback)")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status: int) -> None:
    if status != FH_OK:
        msg = load().fh_last_error()
        raise FhError(status, msg.decode() if msg else "")


def ptr(a):
    """numpy array -> void* (None for empty/None)."""
    if a is None:
        return None
    return a.ctypes.data_as(V)
