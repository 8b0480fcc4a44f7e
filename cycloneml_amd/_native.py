"""ctypes binding of libcyclone.so (include/cyclone.h).

The library is built in-tree (cycloneml_amd/libcyclone.so, see
cycloneml_amd/csrc/Makefile).  There is no fallback: if the shared object is
missing or cannot be loaded this module raises, and every entry point refuses
to run without a gfx950 device (CYC_ERR_NO_DEVICE).
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# CYC_LIB_DIR: load the libraries from another directory (tools/asan_cpu.sh:
# the AddressSanitizer build of the host code)
LIB_DIR = os.environ.get("CYC_LIB_DIR") or _HERE
LIB_PATH = os.path.join(LIB_DIR, "libcyclone.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "cyclone.h")

CYC_OK = 0
CYC_ERR_INVALID_ARG = 1
CYC_ERR_HIP = 2
CYC_ERR_ALLOC = 3
CYC_ERR_UNSUPPORTED = 4
CYC_ERR_NO_DEVICE = 5
CYC_ERR_ASSERTION = 6

CYC_DISTANCE_EUCLIDEAN = 0
CYC_DISTANCE_COSINE = 1

_lib = None
_lock = threading.Lock()

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f64 = ctypes.c_double
_pi64 = ctypes.POINTER(ctypes.c_int64)
_pi32 = ctypes.POINTER(ctypes.c_int32)

# name -> (restype, argtypes).  Device pointers travel as c_void_p.
SIGNATURES = {
    "cyc_last_error": (ctypes.c_char_p, []),
    "cyc_version": (ctypes.c_int, []),
    "cyc_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "cyc_set_device": (ctypes.c_int, [ctypes.c_int]),
    "cyc_synchronize": (ctypes.c_int, [_vp]),
    "cyc_profile_enable": (ctypes.c_int, [ctypes.c_int]),
    "cyc_profile_query": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(_f64), _pi64]),
    "cyc_profile_only": (ctypes.c_int, [ctypes.c_char_p]),
    "cyc_row_norms_dev": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp]),
    "cyc_kmeans_plan_create": (ctypes.c_int, [_i32, _i32, _i64, ctypes.POINTER(_vp)]),
    "cyc_kmeans_plan_destroy": (ctypes.c_int, [_vp]),
    "cyc_kmeans_plan_set_distance_measure": (ctypes.c_int, [_vp, _i32]),
    "cyc_kmeans_silhouette_stats_dev": (ctypes.c_int, [_vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                                       _vp]),
    "cyc_kmeans_silhouette_score_dev": (ctypes.c_int, [_vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                                       _vp, _vp]),
    "cyc_kmeans_stats_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp]),
    "cyc_kmeans_assign_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp,
                                             _pi64, _vp]),
    "cyc_kmeans_point_cost_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                                 _vp, _vp]),
    "cyc_kmeans_point_cost_csr_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp,
                                                     _vp, _vp, _vp]),
    "cyc_kmeans_accumulate_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                                 _vp, _vp, _vp, _vp, _vp]),
    "cyc_kmeans_rows_create": (ctypes.c_int, [_vp, _vp, _i64, _vp, ctypes.POINTER(_vp)]),
    "cyc_kmeans_rows_destroy": (ctypes.c_int, [_vp]),
    "cyc_kmeans_rows_bytes": (_i64, [_vp]),
    "cyc_kmeans_rows_set_bounds": (ctypes.c_int, [_vp, _i32]),
    "cyc_kmeans_rows_bounds_info": (ctypes.c_int, [_vp, _pi64, _pi64]),
    "cyc_kmeans_rows_bounds_rechecked": (ctypes.c_int, [_vp, _pi64]),
    "cyc_kmeans_rows_set_incremental": (ctypes.c_int, [_vp, _i32]),
    "cyc_kmeans_rows_incremental_info": (ctypes.c_int, [_vp, _pi64, _pi64]),
    "cyc_kmeans_last_tiers": (ctypes.c_int, [_vp, _pi64, _pi64]),
    "cyc_kmeans_last_screen": (ctypes.c_int, [_vp, _pi64]),
    "cyc_kmeans_last_candidates": (ctypes.c_int, [_vp, _pi64]),
    "cyc_kmeans_last_candidates3": (ctypes.c_int, [_vp, _pi64]),
    "cyc_kmeans_last_refine": (ctypes.c_int, [_vp, _pi64, _pi64, _pi64]),
    "cyc_kmeans_parallel_sample_dev": (ctypes.c_int, [_vp, _pi64, _i32, _i32, _i32, _i32, _i32,
                                                      _f64, _vp, _vp]),
    "cyc_xorshift_hash_seed": (ctypes.c_uint64, [_i64]),
    "cyc_kmeans_update_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _f64, _vp, _vp]),
    "cyc_row_norms_csr_dev": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp]),
    "cyc_kmeans_assign_csr_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                                 _vp, _vp]),
    "cyc_kmeans_accumulate_csr_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp,
                                                     _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "cyc_gramian_plan_create": (ctypes.c_int, [_i32, ctypes.POINTER(_vp)]),
    "cyc_gramian_plan_destroy": (ctypes.c_int, [_vp]),
    "cyc_gramian_accumulate_dev": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp, _vp]),
    "cyc_col_sums_dev": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp]),
    "cyc_col_moments_dev": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp, _vp]),
    "cyc_gramian_accumulate_sums_dev": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp, _vp]),
    "cyc_triu_to_full_dev": (ctypes.c_int, [_i32, _vp, _vp, _vp]),
    "cyc_covariance_finalize_dev": (ctypes.c_int, [_i32, _vp, _i64, _vp, _vp]),
    "cyc_gramian_accumulate_csr_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp]),
    "cyc_col_sums_csr_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    "cyc_col_moments_csr_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp]),
    "cyc_rowmatrix_dense_rows_dev": (ctypes.c_int, [_vp, _vp, _vp, _i64, ctypes.c_int32, _vp,
                                                    _vp]),
    "cyc_sparse_covariance_finalize_dev": (ctypes.c_int, [ctypes.c_int32, _vp, _i64, _vp, _vp,
                                                          _vp]),
    "cyc_logistic_plan_create": (ctypes.c_int, [_i32, _i32, ctypes.c_int, ctypes.c_int,
                                                ctypes.POINTER(_vp)]),
    "cyc_logistic_plan_destroy": (ctypes.c_int, [_vp]),
    "cyc_binary_logistic_add_dense_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp,
                                                         _vp, _vp, _vp, _vp]),
    "cyc_binary_logistic_add_csr_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp,
                                                       _vp, _vp, _vp, _vp, _vp, _vp]),
    "cyc_hinge_plan_create": (ctypes.c_int, [_i32, ctypes.c_int, ctypes.POINTER(_vp)]),
    "cyc_hinge_add_dense_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp,
                                               _vp, _vp]),
    "cyc_hinge_add_csr_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                             _vp, _vp, _vp, _vp]),
    "cyc_huber_plan_create": (ctypes.c_int, [_i32, ctypes.c_int, _f64, ctypes.POINTER(_vp)]),
    "cyc_huber_add_dense_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp,
                                               _vp, _vp]),
    "cyc_huber_add_csr_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                             _vp, _vp, _vp, _vp]),
    "cyc_aft_plan_create": (ctypes.c_int, [_i32, ctypes.c_int, ctypes.POINTER(_vp)]),
    "cyc_aft_add_dense_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp,
                                             _vp, _vp]),
    "cyc_aft_add_csr_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                           _vp, _vp, _vp, _vp]),
    "cyc_least_squares_plan_create": (ctypes.c_int, [_i32, ctypes.c_int, _f64, _f64,
                                                     ctypes.POINTER(_vp)]),
    "cyc_least_squares_add_dense_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                                       _vp, _vp, _vp, _vp]),
    "cyc_least_squares_add_csr_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp,
                                                     _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "cyc_libsvm_parse": (ctypes.c_int, [ctypes.c_char_p, _i64, _i32, ctypes.c_int,
                                        ctypes.POINTER(_vp)]),
    "cyc_libsvm_load_file": (ctypes.c_int, [ctypes.c_char_p, _i32, ctypes.c_int,
                                            ctypes.POINTER(_vp)]),
    "cyc_libsvm_sizes": (ctypes.c_int, [_vp, _pi64, _pi64, ctypes.POINTER(_i32)]),
    "cyc_libsvm_copy": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "cyc_libsvm_upload": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "cyc_libsvm_destroy": (ctypes.c_int, [_vp]),
    "cyc_csc_build_dev": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _vp, ctypes.POINTER(_vp)]),
    "cyc_csc_destroy": (ctypes.c_int, [_vp]),
    "cyc_csc_rows": (_i64, [_vp]),
    "cyc_csc_blocks": (ctypes.c_int, [_vp, _pi64, _pi64]),
    "cyc_csc_arrays": (ctypes.c_int, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                                      ctypes.POINTER(_vp)]),
    "cyc_multinomial_logistic_add_dense_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp,
                                                              _vp, _vp, _vp, _vp, _vp]),
    "cyc_multinomial_logistic_add_csr_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64,
                                                            _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "cyc_softmax_exp_dev": (ctypes.c_int, [_vp, _i64, _vp, _vp]),
    "cyc_csc_features": (_i32, [_vp]),
    "cyc_tiles_create": (ctypes.c_int, [_i32, _i64, _i64, ctypes.POINTER(_vp)]),
    "cyc_tiles_append_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, _vp]),
    "cyc_tiles_set_format": (ctypes.c_int, [_vp, _i32]),
    "cyc_tiles_format": (_i32, [_vp]),
    "cyc_tiles_entries": (_i64, [_vp]),
    "cyc_tiles_destroy": (ctypes.c_int, [_vp]),
    "cyc_tiles_rows": (_i64, [_vp]),
    "cyc_tiles_nnz": (_i64, [_vp]),
    "cyc_tiles_features": (_i32, [_vp]),
    "cyc_tiles_bytes": (_i64, [_vp]),
    "cyc_tiles_row_block": (_i32, []),
    "cyc_binary_add_tiles_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                                _vp]),
    "cyc_summarizer_buffer_len": (_i64, [_i32]),
    "cyc_summarizer_dense_dev": (ctypes.c_int, [_vp, _vp, _i64, _i32, _i64, _vp, _vp]),
    "cyc_summarizer_csr_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp]),
    "cyc_summarizer_merge_dev": (ctypes.c_int, [_i32, _vp, _i64, _vp, _vp]),
    "cyc_summarizer_metrics_dev": (ctypes.c_int, [_i32, _vp, _vp, _vp]),
    "cyc_label_summarizer_dev": (ctypes.c_int, [_vp, _vp, _i64, _i64, _i32, _vp, _vp, _vp, _vp]),
    "cyc_scale_columns_dense_dev": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp]),
    "cyc_scale_columns_csr_dev": (ctypes.c_int, [_vp, _vp, _i64, _vp, _vp]),
    "cyc_blokify_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64, ctypes.c_int32, _i64, _vp, _vp,
                                        _vp, _vp]),
    # resident datasets: host pointers
    "cyc_dataset_dense_create": (ctypes.c_int, [_i32, _i64, ctypes.c_int, ctypes.c_int,
                                                ctypes.POINTER(_vp)]),
    "cyc_dataset_csr_create": (ctypes.c_int, [_i32, _i64, _i64, ctypes.c_int, ctypes.c_int,
                                              ctypes.POINTER(_vp)]),
    "cyc_dataset_destroy": (ctypes.c_int, [_vp]),
    "cyc_dataset_rows": (_i64, [_vp]),
    "cyc_dataset_append_dense": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i64]),
    "cyc_dataset_append_csr": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64]),
    "cyc_kmeans_iter": (ctypes.c_int, [_vp, _vp, _i32, _vp, _vp, _vp, _vp]),
    "cyc_kmeans_iter_measure": (ctypes.c_int, [_vp, _i32, _vp, _vp, _i32, _vp, _vp, _vp, _vp]),
    "cyc_svc_hinge_eval": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _vp, _vp, _vp, _vp]),
    "cyc_linreg_least_squares_eval": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int, _f64, _f64,
                                                     _vp, _vp, _vp, _vp]),
    "cyc_linreg_huber_eval": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _f64, _vp, _vp, _vp,
                                             _vp]),
    "cyc_aft_eval": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _vp, _vp, _vp, _vp]),
    "cyc_logreg_binary_eval": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, _vp, _vp,
                                              _vp, _vp]),
    "cyc_logreg_multinomial_eval": (ctypes.c_int, [_vp, _i32, _vp, ctypes.c_int, ctypes.c_int,
                                                   _vp, _vp, _vp, _vp]),
    "cyc_gramian": (ctypes.c_int, [_vp, _vp, _vp]),
    # the aggregation step over RCCL (cyc_comm_*)
    "cyc_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "cyc_comm_init": (ctypes.c_int, [ctypes.c_char_p, _i32, _i32, _i32, ctypes.POINTER(_vp)]),
    "cyc_comm_destroy": (ctypes.c_int, [_vp]),
    "cyc_comm_rank": (ctypes.c_int, [_vp, _pi32, _pi32]),
    "cyc_allreduce_sum_dev": (ctypes.c_int, [_vp, _vp, _i64, _vp]),
    "cyc_allreduce_max_dev": (ctypes.c_int, [_vp, _vp, _i64, _vp]),
    "cyc_broadcast_dev": (ctypes.c_int, [_vp, _vp, _i64, _i32, _vp]),
    "cyc_allgather_dev": (ctypes.c_int, [_vp, _vp, _vp, _i64, _vp]),
    "cyc_allreduce_sum": (ctypes.c_int, [_vp, _vp, _i64]),
    "cyc_broadcast": (ctypes.c_int, [_vp, _vp, _i64, _i32]),
    "cyc_col_sums": (ctypes.c_int, [_vp, _vp]),
}


class CycloneError(RuntimeError):
    """A libcyclone call failed (HIP error, allocation, unsupported shape)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[cyclone {code}] {msg}")
        self.code = code


class IllegalArgumentException(ValueError):
    """A reference `require` failed (Scala IllegalArgumentException)."""


class JavaAssertionError(AssertionError):
    """A reference `assert` failed (java.lang.AssertionError)."""


def load():
    """Load libcyclone.so; raises if it is missing (no silent fallback)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"libcyclone.so not found at {LIB_PATH}; build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` "
                    "(or make -C cycloneml_amd/csrc)")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def check(rc: int):
    if rc == CYC_OK:
        return
    msg = load().cyc_last_error().decode(errors="replace")
    if rc == CYC_ERR_INVALID_ARG:
        raise IllegalArgumentException(msg)
    if rc == CYC_ERR_ASSERTION:
        raise JavaAssertionError(msg)
    raise CycloneError(rc, msg)


def header_symbols(path: str = HEADER_PATH):
    """Function names declared in include/cyclone.h."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(cyc_[a-z0-9_]+)\s*\(", txt)))


def profile_enable(on: bool):
    check(load().cyc_profile_enable(int(on)))


def profile_only(kernels):
    """Time only these kernel names (None: all)."""
    check(load().cyc_profile_only(None if kernels is None else ",".join(kernels).encode()))


def profile_query(kernel: str):
    """(total_ms, launches) of `kernel` since the last query (HIP events)."""
    ms = _f64()
    cnt = _i64()
    check(load().cyc_profile_query(kernel.encode(), ctypes.byref(ms), ctypes.byref(cnt)))
    return ms.value, cnt.value


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(stream=None) -> int | None:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
