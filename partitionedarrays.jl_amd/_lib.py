"""ctypes binding of libpa_hip.so — the same C-ABI a Julia `HIPBackend` would
`ccall` (include/pa_hip.h).

There is no CPU fallback: if the shared library is missing, or no HIP device
is visible, every device operation raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# PA_HIP_LIB: another build of the same library (A/B tooling only)
LIB_PATH = os.environ.get("PA_HIP_LIB") or os.path.join(_HERE, "libpa_hip.so")

PA_F32, PA_F64, PA_C64, PA_C128 = 0, 1, 2, 3
PA_REPLACE, PA_ADD = 0, 1
TUNE_DROP = -(2 ** 31)  # pa_ctx_tune: drop a context's override (PA_TUNE_DROP)
PA_BCAST_F64, PA_BCAST_C128 = 8, 16  # pa_vec_axpby scalar kinds (Float64 / ComplexF64 scalars)

DTYPES = {
    np.dtype(np.float32): PA_F32,
    np.dtype(np.float64): PA_F64,
    np.dtype(np.complex64): PA_C64,
    np.dtype(np.complex128): PA_C128,
}
NP_OF = {v: k for k, v in DTYPES.items()}

_lib = None
_p = C.c_void_p
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)

# name: (argtypes)  — every function returns int status
_SIGS = {
    "pa_version": [],
    "pa_device_count": [C.POINTER(C.c_int)],
    "pa_tune": [C.c_char_p, C.c_int, C.POINTER(C.c_int)],
    "pa_ctx_tune": [_p, C.c_char_p, C.c_int, C.POINTER(C.c_int)],
    "pa_knob_selftest": [C.c_int, C.c_int, C.POINTER(C.c_int)],
    "pa_cg_variant_agree": [C.POINTER(C.c_float), _p, _p, C.POINTER(C.c_int)],
    "pa_cg_fuse_agree": [C.c_int, _p, _p, C.POINTER(C.c_int)],
    "pa_mat_cg_choice": [_p, C.POINTER(C.c_int)],
    "pa_hbm_probe": [C.c_int, C.c_int64, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)],
    "pa_issue_stats": [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int64)],
    "pa_hbm_probe_launch": [C.c_int, C.c_int64, C.c_int64, C.c_int, C.POINTER(C.c_double)],
    "pa_ctx_create": [C.c_int, C.c_int, C.c_int, C.POINTER(_p)],
    "pa_ctx_create_shared": [C.c_int, C.c_int, _p, C.POINTER(_p)],
    "pa_ctx_destroy": [_p],
    "pa_ctx_sync": [_p],
    "pa_comm_unique_id": [C.c_char_p],
    "pa_comm_init_rank": [_p, C.c_char_p],
    "pa_comm_init_all": [C.c_int, C.POINTER(_p)],
    "pa_comm_stats": [_p, _i64p, _i64p],
    "pa_comm_info": [_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_char_p, C.c_int,
                     C.POINTER(C.c_int), C.c_char_p, C.c_int],
    "pa_index_create": [_p, C.c_int64, C.c_int64, _i32p, C.c_int64, _i32p, C.POINTER(_p)],
    "pa_index_destroy": [_p],
    "pa_xchg_create": [_p, C.c_int32, _i32p, _i32p, _i32p, C.c_int32, _i32p, _i32p, _i32p, C.POINTER(_p)],
    "pa_xchg_destroy": [_p],
    "pa_vec_create": [_p, C.c_int, C.c_int64, C.POINTER(_p)],
    "pa_vec_destroy": [_p],
    "pa_vec_upload": [_p, _p, C.c_int64],
    "pa_vec_download": [_p, _p, C.c_int64],
    "pa_vec_device_ptr": [_p, _p],
    "pa_vec_fill": [_p, _p],
    "pa_vec_copy": [_p, _p, _p, _p, C.c_int],
    "pa_vec_axpby": [_p, _p, _p, _p, C.c_int, C.c_int],
    "pa_mat_from_csc": [_p, C.c_int, C.c_int, C.c_int64, C.c_int64, _p, _p, _p, _p, _p, C.POINTER(_p)],
    "pa_mat_from_csr": [_p, C.c_int, C.c_int, C.c_int, C.c_int64, C.c_int64, _p, _p, _p, _p, _p, C.POINTER(_p)],
    "pa_coo_create": [_p, C.c_int, C.c_int64, _i64p, _i64p, _p, C.POINTER(_p)],
    "pa_coo_destroy": [_p],
    "pa_coo_size": [_p, _i64p],
    "pa_coo_download": [_p, _i64p, _i64p, _p],
    "pa_coo_assemble_all": [C.c_int, C.POINTER(_p), C.POINTER(_p), C.POINTER(_p)],
    "pa_mat_from_dcoo": [_p, C.c_int, C.c_int64, C.c_int64, _p, _p, _i64p, _i64p, _i64p, C.POINTER(_p)],
    "pa_mat_from_coo": [_p, C.c_int, C.c_int, C.c_int, C.c_int64, C.c_int64, C.c_int64, _p, _p, _p, _p, _p, _i64p,
                        _i64p, _i64p, C.POINTER(_p)],
    "pa_mat_from_coo_csr": [_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int64, C.c_int64, C.c_int64, _p, _p, _p, _p,
                            _p, _i64p, _i64p, _i64p, C.POINTER(_p)],
    "pa_mat_from_dcoo_csr": [_p, C.c_int, C.c_int, C.c_int64, C.c_int64, _p, _p, _i64p, _i64p, _i64p,
                             C.POINTER(_p)],
    "pa_mat_fillstored": [_p, _p],
    "pa_index_set_gids": [_p, _i64p],
    "pa_add_gids": [_p, C.c_int64, _i64p, C.c_int64, _i64p, _i64p],
    "pa_index_to_lids": [_p, C.c_int64, _i64p],
    "pa_mat_set_values": [_p, _p],
    "pa_mat_get_values": [_p, _p],
    "pa_mat_xchg_create": [_p, C.c_int32, _i32p, _i32p, _i64p, C.c_int32, _i32p, _i32p, _i64p, C.POINTER(_p)],
    "pa_mat_exchange_all": [C.c_int, C.POINTER(_p), C.POINTER(_p), C.c_int, C.c_int, C.c_int],
    "pa_mat_destroy": [_p],
    "pa_mat_info": [_p, _i64p, _i64p, _i64p, _i64p, _i64p],
    "pa_mat_format_info": [_p, _i64p, _i64p, _i64p, _i64p],
    "pa_mat_delta16_info": [_p, _i64p],
    "pa_mat_triple_info": [_p, _i64p, _i64p, _i64p, _i64p],
    "pa_mat_pair_info": [_p, _i64p, _i64p],
    "pa_mat_long_rows": [_p, _i64p, _i64p],
    "pa_mat_stencil": [_p, C.c_int, C.c_int, _i64p, _i64p, _i64p, C.c_int64, _i32p, C.POINTER(C.c_double), C.c_int, C.POINTER(_p)],
    "pa_spmv_all": [C.c_int, C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), _p, _p],
    "pa_spmv_dot_all": [C.c_int, C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), _p, _p, _p],
    "pa_cg_update_all": [C.c_int, C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), _p, C.POINTER(C.c_double)],
    "pa_cg_solve_all": [C.c_int, C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.POINTER(_p),
                        C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.c_double, C.c_double, C.c_int64, C.c_int,
                        _i64p, C.POINTER(C.c_double), C.POINTER(C.c_double)],
    "pa_exchange_all": [C.c_int, C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.c_int, C.c_int, C.c_int],
    "pa_dot_all": [C.c_int, C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), _p],
    "pa_norm2_all": [C.c_int, C.POINTER(_p), C.POINTER(_p), _p],
    "pa_sum_all": [C.c_int, C.POINTER(_p), C.POINTER(_p), _p],
    "pa_ctx_last_kernel_ms": [_p, C.POINTER(C.c_float), C.POINTER(C.c_float)],
    "pa_ctx_kernel_times": [_p, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float),
                            C.POINTER(C.c_int)],
    "pa_mat_traffic": [_p, _i64p, _i64p, _i64p],
    "pa_mat_device_ptrs": [_p, _p],
    "pa_ctx_span": [_p, C.c_int],
    "pa_ctx_span_ms": [_p, C.POINTER(C.c_float)],
    "pa_ctx_set_timing": [_p, C.c_int],
}

EXPORTED = sorted(list(_SIGS) + ["pa_last_error"])


class PAError(RuntimeError):
    pass


def _prepare_runtime():
    # One HIP runtime per process: torch ships its own libamdhip64 with the
    # same soname; importing torch first makes the dynamic linker reuse it
    # for libpa_hip.so (two runtimes in one process would not share devices).
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PAError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    _prepare_runtime()
    L = C.CDLL(LIB_PATH)
    for name, args in _SIGS.items():
        if os.environ.get("PA_HIP_LIB") and not hasattr(L, name):
            continue  # another build (A/B tooling only) may lack newer entry points
        f = getattr(L, name)
        f.argtypes = args
        f.restype = C.c_int
    L.pa_last_error.argtypes = []
    L.pa_last_error.restype = C.c_char_p
    _lib = L
    return L


def call(name, *args):
    L = lib()
    rc = getattr(L, name)(*args)
    if rc != 0:
        raise PAError(f"{name}: {L.pa_last_error().decode(errors='replace')}")


def device_count() -> int:
    n = C.c_int(0)
    call("pa_device_count", C.byref(n))
    return n.value


def tune(key: str, value: int) -> int:
    """pa_tune: set a process-wide kernel knob, return the previous value."""
    prev = C.c_int(0)
    call("pa_tune", key.encode(), int(value), C.byref(prev))
    return prev.value


def knob_selftest(nthreads: int = 4, iters: int = 2000) -> int:
    """pa_knob_selftest: resolutions of concurrent calls' knobs that saw
    another call's context value (0 expected; no device needed)."""
    n = C.c_int(-1)
    call("pa_knob_selftest", int(nthreads), int(iters), C.byref(n))
    return n.value


ALLREDUCE_MAX_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_float), C.c_int, C.c_void_p)


def cg_variant_agree(local_ms, allreduce_max=None) -> int:
    """pa_cg_variant_agree: the device CG's auto u-update choice (1 fused,
    0 sweep, -1 none) from this rank's two batch times (ms per iteration:
    sweep, fused), reduced with `allreduce_max(list of 2 floats) -> list`
    over the ranks first (the library's RCCL reduction's role; None: one
    process)."""
    ms = (C.c_float * 2)(*[float(v) for v in local_ms])
    cb = None
    if allreduce_max is not None:
        def _cb(v, n, _user):
            try:
                out = allreduce_max([v[i] for i in range(n)])
                for i in range(n):
                    v[i] = float(out[i])
                return 0
            except Exception:  # reported as a PAError by the library
                return 1
        cb = ALLREDUCE_MAX_FN(_cb)
    ch = C.c_int(-3)
    call("pa_cg_variant_agree", ms, C.cast(cb, C.c_void_p) if cb else None, None, C.byref(ch))
    return ch.value


def cg_fuse_agree(local_can_fuse: bool, allreduce_max=None) -> bool:
    """pa_cg_fuse_agree: whether the device CG may run the fused u update,
    decided over the ranks (every rank's part must allow it: no long rows,
    no triple SELL); `allreduce_max` as in cg_variant_agree."""
    cb = None
    if allreduce_max is not None:
        def _cb(v, n, _user):
            try:
                out = allreduce_max([v[i] for i in range(n)])
                for i in range(n):
                    v[i] = float(out[i])
                return 0
            except Exception:  # reported as a PAError by the library
                return 1
        cb = ALLREDUCE_MAX_FN(_cb)
    ok = C.c_int(-1)
    call("pa_cg_fuse_agree", int(bool(local_can_fuse)), C.cast(cb, C.c_void_p) if cb else None, None, C.byref(ok))
    return ok.value == 1


def hbm_probe(device: int = 0, nbytes: int = 2 << 30, reps: int = 10):
    """pa_hbm_probe: (read GB/s, copy GB/s) attainable on `device` (calibration)."""
    r, c = C.c_double(), C.c_double()
    call("pa_hbm_probe", int(device), int(nbytes), int(reps), C.byref(r), C.byref(c))
    return r.value, c.value


def issue_stats(reset=True):
    """pa_issue_stats: (max µs, mean µs, count) of the issue jobs (one part's
    share of a threaded call) since the last reset"""
    mx, mean, n = C.c_double(), C.c_double(), C.c_int64()
    call("pa_issue_stats", int(bool(reset)), C.byref(mx), C.byref(mean), C.byref(n))
    return mx.value, mean.value, n.value


def hbm_probe_launch(device: int, bytes_per_launch: int, span: int = 2 << 30, reps: int = 40) -> float:
    """pa_hbm_probe_launch: read GB/s when each launch reads bytes_per_launch
    (rotating over `span` bytes, from HBM): one launch's ramp and drain
    included"""
    r = C.c_double()
    call("pa_hbm_probe_launch", int(device), int(bytes_per_launch), int(span), int(reps), C.byref(r))
    return r.value


def i32(a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    return a, a.ctypes.data_as(_i32p)


def ptr_array(handles):
    arr = (_p * len(handles))(*[h for h in handles])
    return arr


def scalar_buf(value, dtype):
    """host buffer holding `value` as dtype (for alpha/beta/fill)."""
    a = np.array([value], dtype=np.dtype(dtype))
    return a, a.ctypes.data_as(_p)
