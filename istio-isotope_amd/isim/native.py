"""ctypes binding of libisim.so (include/isim.h).

The library is built in-tree (``istio-isotope_amd/isim/libisim.so``) by
``__graft_entry__.build()``.  There is no fallback: if the library is missing
or fails to load, every entry point raises.

torch is imported (when available) BEFORE the library is loaded: torch ships
its own ``libamdhip64.so`` (SONAME ``libamdhip64.so.7``); loading it first
makes libisim's ``libamdhip64.so.7`` dependency resolve to the same runtime
instead of a second copy from /opt/rocm.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ISIM_LIB") or os.path.join(_HERE, "libisim.so")

# isim_status
OK, EINVAL, ENOMEM, EHIP, EPARSE, ECYCLE, EDEPTH, ERANGE, ENOTFOUND, ENODEV, ECOMM = range(11)
STATUS_NAMES = {0: "OK", 1: "EINVAL", 2: "ENOMEM", 3: "EHIP", 4: "EPARSE", 5: "ECYCLE",
                6: "EDEPTH", 7: "ERANGE", 8: "ENOTFOUND", 9: "ENODEV",
                10: "ECOMM"}
MODE_A, MODE_B = 0, 1
ABI_VERSION = 10  # include/isim.h ISIM_ABI_VERSION
FLAG_NO_STREAM = 1
FLAG_NO_SVC_DUR = 2
FLAG_WALK_ALL = 4  # draw-free static walks: walk every trace (default: one walk, then a fill)
FLAG_BIT_STACK = 8  # mode B on the draw stream: the bit-stack kernel (kind 5/4) instead of the close list (6)
FLAG_DYNAMIC = 16  # every walk on the general (dynamic) kernels, kind 7 (or 2/3)
FLAG_WAVE_WALK = 32  # dynamic walks on the wave-walk interpreter (kinds 2/3) instead of the lane tree walk (7)
FLAG_CLOSE_LIST = 64  # mode B on the draw stream: the close list (kind 6) instead of sparse ancestor marking (8)
# independent-check paths (isim.h): the same results by a different algorithm
FLAG_TREE_WIDE = 128  # the wide lane-tree format for any dynamic walk
FLAG_DES_SCAN_BY_KEY = 256  # DES items: queues by rocPRIM's scan by key (not k_qscan)
FLAG_DES_SORT_ALL = 512  # DES items, cyclic schedules: sort every round of every pass
FLAG_DES_TWO_SORTS = 1024  # DES items: two stable sorts per sorted queue round
FLAG_TREE_DAG = 2048  # the lane walk over the site graph for any dynamic walk

# stats layout (isim.h)
ST_N_TRACES, ST_SUM_LATENCY, ST_SUM_HOPS, ST_SUM_ERR_HOPS, ST_N_500 = 0, 1, 2, 3, 4
ST_NOT_MIN_LATENCY, ST_MAX_LATENCY = 5, 6
ST_DES_RETRY = 7  # DES batches not accumulated (32-bit rows overflowed): rerun with DES_FLAG_WIDE
N_PROM, N_LOG2 = 33, 64
ST_PROM = 8
ST_LOG2 = ST_PROM + 2 * N_PROM
ST_SITES = ST_LOG2 + 2 * N_LOG2
SVC_DUR_WORDS = 2 * N_PROM + 2
# DES table row (isim.h ISIM_DES_*)
DES_COUNT, DES_SUM_WAIT, DES_MAX_WAIT, DES_SUM_HOLD = SVC_DUR_WORDS, SVC_DUR_WORDS + 1, SVC_DUR_WORDS + 2, SVC_DUR_WORDS + 3
DES_ROW_WORDS = SVC_DUR_WORDS + 4
DES_FLAG_WIDE = 1  # isim_des_params.flags: 64-bit rows


class IsimError(RuntimeError):
    def __init__(self, code: int, msg: str):
        self.code = code
        self.status = STATUS_NAMES.get(code, str(code))
        super().__init__(f"{self.status}: {msg}")


class Params(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("hop_base_ns", C.c_uint64),
                ("req_ps_per_byte", C.c_uint64), ("resp_ps_per_byte", C.c_uint64),
                ("error_mode", C.c_uint32), ("max_depth", C.c_uint32),
                ("flags", C.c_uint32), ("reserved", C.c_uint32)]


class TraceRec(C.Structure):
    _fields_ = [("latency_ns", C.c_uint64), ("hops", C.c_uint32), ("status_err", C.c_uint32)]


class HandlerInfo(C.Structure):
    _fields_ = [("n_services", C.c_int32), ("n_sites", C.c_int32), ("n_slots", C.c_int32),
                ("entry", C.c_int32), ("max_depth", C.c_int32), ("static_walk", C.c_int32),
                ("time_bits", C.c_int32), ("program_len", C.c_int32),
                ("max_latency_ns", C.c_uint64), ("hops_upper", C.c_uint64),
                ("stats_words", C.c_uint64), ("svc_dur_rows", C.c_int32), ("n_reachable", C.c_int32),
                ("draw_groups", C.c_uint64)]


class LaunchInfo(C.Structure):
    _fields_ = [("wg_threads", C.c_int32), ("lds_bytes", C.c_int32), ("lds_counters", C.c_int32),
                ("blocks_per_cu", C.c_int32), ("max_blocks", C.c_int32), ("kernel_kind", C.c_int32),
                ("fill", C.c_int32), ("tree_wide", C.c_int32), ("max_launch_traces", C.c_uint64)]


class DesParams(C.Structure):
    _fields_ = [("mean_interarrival_ns", C.c_uint64), ("flags", C.c_uint32), ("reserved", C.c_uint32)]


class K8sParams(C.Structure):
    _fields_ = [("service_image", C.c_char_p), ("client_image", C.c_char_p), ("environment_name", C.c_char_p),
                ("service_node_selector", C.c_void_p), ("client_node_selector", C.c_void_p),
                ("n_service_node_selector", C.c_int32), ("n_client_node_selector", C.c_int32),
                ("service_max_idle_connections_per_host", C.c_int32), ("reserved", C.c_int32),
                ("creation_timestamp_s", C.c_int64), ("rbac_seed", C.c_uint64)]


class MultiId(C.Structure):
    _fields_ = [("internal", C.c_char * 128)]


class DesBatchStats(C.Structure):
    _fields_ = [("passes", C.c_uint32), ("syncs", C.c_uint32), ("items", C.c_uint64)]


class DesInfo(C.Structure):
    _fields_ = [("n_positions", C.c_int32), ("n_levels", C.c_int32), ("max_width", C.c_int32),
                ("table_rows", C.c_int32), ("n_fused", C.c_int32), ("cyclic", C.c_int32),
                ("row_reads", C.c_int32), ("row_writes", C.c_int32), ("items", C.c_int32)]


# every function declared in include/isim.h: name -> (restype, argtypes)
_VP = C.c_void_p
SIGNATURES = {
    "isim_last_error": (C.c_char_p, []),
    "isim_abi_version": (C.c_int, []),
    "isim_graph_unmarshal_json": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(_VP)]),
    "isim_graph_free": (None, [_VP]),
    "isim_graph_num_services": (C.c_int, [_VP]),
    "isim_graph_canonical_json": (C.c_int, [_VP, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "isim_graph_marshal_json": (C.c_int, [_VP, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "isim_graph_to_dot": (C.c_int, [_VP, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "isim_graph_to_k8s_manifests": (C.c_int, [_VP, C.c_void_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "isim_graph_marshal_yaml": (C.c_int, [_VP, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "isim_graph_service_index": (C.c_int, [_VP, C.c_char_p]),
    "isim_size_from_string": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint64)]),
    "isim_duration_parse": (C.c_int, [C.c_char_p, C.POINTER(C.c_int64)]),
    "isim_percentage_from_string": (C.c_int, [C.c_char_p, C.POINTER(C.c_double)]),
    "isim_handler_create": (C.c_int, [_VP, C.c_char_p, C.POINTER(Params), C.POINTER(_VP)]),
    "isim_handler_free": (None, [_VP]),
    "isim_handler_info_get": (C.c_int, [_VP, C.POINTER(HandlerInfo)]),
    "isim_handler_launch_info": (C.c_int, [_VP, C.c_int, C.POINTER(LaunchInfo)]),
    "isim_handler_slots": (C.c_int, [_VP, _VP, _VP]),
    "isim_serve_device": (C.c_int, [_VP, C.c_uint64, C.c_uint64, _VP, _VP, _VP]),
    "isim_serve": (C.c_int, [_VP, C.c_int, C.c_uint64, C.c_uint64, _VP, _VP]),
    "isim_stats_fold": (C.c_int, [_VP, _VP, _VP, _VP, _VP]),
    "isim_stats_fold_durations": (C.c_int, [_VP, _VP, _VP]),
    "isim_des_info_get": (C.c_int, [_VP, C.POINTER(DesInfo)]),
    "isim_des_last_batch": (C.c_int, [_VP, C.POINTER(DesBatchStats)]),
    "isim_des_workspace_bytes": (C.c_int, [_VP, C.c_uint64, C.POINTER(C.c_uint64)]),
    "isim_serve_des_device": (C.c_int, [_VP, C.POINTER(DesParams), C.c_uint64, C.c_uint64, _VP, _VP, _VP,
                                        _VP, C.c_uint64, _VP]),
    "isim_serve_des": (C.c_int, [_VP, C.c_int, C.POINTER(DesParams), C.c_uint64, C.c_uint64, _VP, _VP, _VP]),
    "isim_des_fold": (C.c_int, [_VP, _VP, _VP]),
    "isim_debug_set_spin_limit": (None, [C.c_uint32]),
    "isim_debug_spin_limit": (C.c_uint32, []),
    "isim_multi_get_id": (C.c_int, [C.POINTER(MultiId)]),
    "isim_multi_precheck": (C.c_int, [C.c_int]),
    "isim_multi_init_rank": (C.c_int, [C.POINTER(MultiId), C.c_int, C.c_int, C.c_int, C.POINTER(_VP)]),
    "isim_multi_init_all": (C.c_int, [C.POINTER(C.c_int), C.c_int, C.POINTER(_VP)]),
    "isim_multi_free": (None, [_VP]),
    "isim_multi_abort": (C.c_int, [_VP]),
    "isim_multi_info": (C.c_int, [_VP, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "isim_stats_allreduce_device": (C.c_int, [_VP, _VP, C.POINTER(_VP), C.POINTER(_VP)]),
    "isim_des_table_allreduce_device": (C.c_int, [_VP, _VP, C.POINTER(_VP), C.POINTER(_VP)]),
    "isim_serve_multi": (C.c_int, [_VP, _VP, C.c_uint64, C.c_uint64, _VP, _VP]),
    "isim_stats_merge": (C.c_int, [_VP, _VP, _VP]),
    "isim_des_table_merge": (C.c_int, [_VP, _VP, _VP]),
}

_lib = None


def load():
    """Load libisim.so (raises if absent: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401  (see module docstring)
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libisim.so not built: {LIB_PATH} (run __graft_entry__.build())")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.isim_abi_version() != ABI_VERSION:
        raise ImportError("libisim ABI version mismatch")
    _lib = lib
    return lib


def last_error() -> str:
    return load().isim_last_error().decode("utf-8", "replace")


def check(rc: int) -> None:
    if rc != OK:
        raise IsimError(rc, last_error())
