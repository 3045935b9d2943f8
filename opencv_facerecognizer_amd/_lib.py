"""ctypes binding of libocvf_hip.so (the gfx950 C ABI declared in include/ofr.h).

torch is imported FIRST so that its bundled HIP runtime (soname
libamdhip64.so.7) is the one our library binds to: device pointers and
streams handed over from torch tensors are then valid in our kernels.

The product path has no CPU fallback: every compute entry point raises if the
library is missing or no gfx950 device is visible.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OFR_LIB", os.path.join(_HERE, "libocvf_hip.so"))

METRIC_EUCLIDEAN = 0
METRIC_COSINE = 1
METRIC_CHISQUARE = 2
MAX_K = 16
DT_U8, DT_U16, DT_U32, DT_F32, DT_F64 = 0, 1, 2, 3, 4

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_vp = ctypes.c_void_p
c_dbl = ctypes.c_double
c_sz = ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/ofr.h
SIGNATURES = {
    "ofr_version": (c_int, []),
    "ofr_last_error": (ctypes.c_char_p, []),
    "ofr_device_check": (c_int, [c_int]),
    "ofr_qproj_bytes": (c_sz, [c_i64, c_i64]),
    "ofr_qproj_prepare": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp]),
    "ofr_project_u8_exact": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp,
                                     c_i64, c_int]),
    "ofr_project_u8_exact_tiles": (c_i64, [c_i64, c_i64]),
    "ofr_project_u8_exact_range": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp,
                                           c_vp, c_i64, c_int, c_i64, c_i64]),
    "ofr_center_round_f64": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64]),
    "ofr_row_aux": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "ofr_col_mean": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "ofr_sub_rows": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "ofr_knn_workspace_bytes": (c_sz, [c_i64, c_i64, c_int]),
    "ofr_knn_f32": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_int, c_i64,
                            c_vp, c_vp, c_vp, c_sz]),
    "ofr_knn_tiles_f32": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_int, c_i64,
                                  c_vp, c_vp, c_vp, c_sz]),
    "ofr_knn_merge_f32": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_int, c_i64,
                                  c_vp, c_vp, c_vp, c_sz]),
    "ofr_q8_quantize_rows": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "ofr_knn_q8_workspace_bytes": (c_sz, [c_i64, c_i64]),
    "ofr_knn_q8": (c_int, [c_vp, c_int, c_int, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64,
                           c_vp, c_i64, c_vp, c_vp, c_vp, c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz]),
    "ofr_normalize_rows_f32": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64]),
    "ofr_cosine_pairs": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_int, c_vp, c_vp]),
    "ofr_f6_tiles_bytes": (c_sz, [c_i64, c_i64]),
    "ofr_f6_quantize_rows_at": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_sz, c_vp, c_vp, c_vp]),
    "ofr_q8_maxima": (c_int, [c_vp, c_vp, c_vp, c_i64, c_vp]),
    "ofr_knn_f6_workspace_bytes": (c_sz, [c_i64, c_i64]),
    "ofr_knn_f6_merge_evals_offset": (c_sz, [c_i64, c_i64]),
    "ofr_f6_sieve_kernel": (ctypes.c_char_p, []),
    "ofr_f6p_sieve_kernel": (ctypes.c_char_p, [c_int]),
    "ofr_knn_f6_sieve_counts_offset": (c_sz, [c_i64, c_i64]),
    "ofr_knn_f6_set_thresholds": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_sz]),
    "ofr_f6_quantize_rows": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_sz, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "ofr_knn_f6": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp,
                           c_vp, c_vp, c_vp, c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ofr_knn_f6_sampled": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp,
                                   c_vp, c_vp, c_vp, c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp,
                                   c_vp, c_sz, c_vp]),
    "ofr_f6_quantize_rows_prefix": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_int, c_vp, c_sz, c_vp, c_vp, c_vp]),
    "ofr_f6p_tiles_bytes": (c_sz, [c_i64, c_int]),
    "ofr_f6p_quantize_rows_at": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_int, c_vp, c_sz, c_vp, c_vp, c_vp]),
    "ofr_f6p_quantize_rows": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_int, c_vp, c_sz, c_vp, c_vp, c_vp, c_vp,
                                      c_vp]),
    "ofr_knn_f6p_sampled": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp,
                                    c_vp, c_vp, c_vp, c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp,
                                    c_vp, c_sz, c_vp, c_int]),
    "ofr_knn_deep_workspace_bytes": (c_sz, [c_i64, c_i64]),
    "ofr_knn_deep": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_int, c_vp, c_i64, c_i64, c_int, c_i64, c_dbl, c_int,
                             c_i64, c_vp, c_vp, c_vp, c_sz]),
    "ofr_f6_sample_step": (c_i64, []),
    "ofr_f6_block_sumsq": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "ofr_f6_block_scales": (c_int, [c_vp, c_vp, c_i64, c_vp]),
    "ofr_f6_sample_rows": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_sz, c_vp, c_vp,
                                   c_vp, c_vp]),
    "ofr_knn_f6_merge_pruned": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                        c_i64, c_vp, c_vp, c_vp, c_vp, c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                        c_vp, c_sz]),
    "ofr_knn_f6p_merge_pruned": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                         c_i64, c_vp, c_vp, c_vp, c_vp, c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                         c_vp, c_sz, c_int]),
    "ofr_f6x2_quantize_rows": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_sz, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "ofr_f6x2_quantize_rows_at": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_sz, c_vp, c_vp, c_vp]),
    "ofr_knn_f6x2": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64,
                             c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ofr_f6x2_sample_rows": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_sz, c_vp, c_vp, c_vp]),
    "ofr_knn_f6x2_sampled": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                     c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                     c_vp, c_i64, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ofr_class_sums_f64": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "ofr_class_between_f64": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "ofr_class_sub_f64": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "ofr_topk_merge": (c_int, [c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_vp]),
    "ofr_elbp_codes": (c_int, [c_vp, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_vp, c_int, c_int, c_int, c_int,
                               c_vp]),
    "ofr_elbp_hist_geom": (c_int, [c_vp, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_vp, c_int, c_int, c_int, c_int,
                                   c_int, c_int, c_vp, c_int]),
    "ofr_elbp_hist": (c_int, [c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_int, c_int, c_int, c_vp]),
    "ofr_chi2_workspace_bytes": (c_sz, [c_i64, c_i64, c_int]),
    "ofr_chi2_mfma_bound": (c_dbl, [c_i64]),
    "ofr_chi2_table": (None, [c_vp]),
    "ofr_chi2_knn": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_dbl, c_int, c_i64, c_vp,
                             c_vp, c_vp, c_sz, c_vp]),
    "ofr_chi2_knn_exact": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_dbl, c_int, c_i64,
                                   c_vp, c_vp, c_vp, c_sz, c_vp]),
    "ofr_gemm_f64": (c_int, [c_vp, c_int, c_int, c_i64, c_i64, c_i64, c_dbl, c_vp, c_i64, c_vp, c_i64, c_dbl, c_vp,
                             c_i64]),
    "ofr_center_u8_f64": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64]),
    "ofr_col_mean_u8": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "ofr_col_mean_f64": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "ofr_sub_mean_f64": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64]),
    "ofr_normalize_cols_f64": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64]),
    "ofr_pad_u8": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_int, c_vp, c_i64]),
    "ofr_gram_u8": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_i64]),
    "ofr_class_sums_u8": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_int, c_vp, c_vp]),
    "ofr_row_dot_u8": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "ofr_center_gram_f64": (c_int, [c_vp, c_vp, c_i64, c_i64, c_vp, c_dbl, c_dbl]),
    "ofr_scatter_combine_f64": (c_int, [c_vp, c_vp, c_vp, c_vp, c_dbl, c_i64, c_i64, c_vp, c_vp]),
    "ofr_rank1_f64": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_dbl]),
    "ofr_row_div_f64": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64]),
    "ofr_comm_init_all": (c_int, [c_int, c_vp, c_vp]),
    "ofr_comm_destroy": (c_int, [c_vp]),
    "ofr_comm_size": (c_int, [c_vp]),
    "ofr_knn_sharded_workspace_bytes": (c_sz, [c_i64, c_i64, c_i64, c_int, c_int]),
    "ofr_knn_sharded": (c_int, [c_vp, c_vp, c_i64, c_i64, c_int]),
    "ofr_topk_merge_certify": (c_int, [c_vp, c_vp, c_int, c_i64, c_int, c_vp, c_vp, c_vp]),
    "ofr_topk_pack": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp]),
    "ofr_kth_bound": (c_int, [c_vp, c_vp, c_int, c_i64, c_int, c_vp]),
    "ofr_open_rows": (c_int, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    "ofr_eig_workspace_bytes": (c_sz, [c_i64, c_i64]),
    "ofr_ctx_create": (c_int, [c_int, c_vp]),
    "ofr_ctx_destroy": (c_int, [c_vp]),
    "ofr_project_u8": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_int]),
    "ofr_gram": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_int, c_int, c_vp]),
    "ofr_scatter": (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_vp]),
    "ofr_knn": (c_int, [c_vp, c_vp, c_int, c_vp, c_i64, c_vp, c_vp, c_i64, c_i64, c_int, c_i64, c_vp, c_vp]),
    "ofr_eigh_f64": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_sz]),
    "ofr_sygv_f64": (c_int, [c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_sz]),
    "ofr_ingest_faces": (c_int, [c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_vp]),
    "ofr_class_center_f64": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                     c_vp]),
}


class KnnShard(ctypes.Structure):
    """struct ofr_knn_shard (include/ofr.h): one device's part of ofr_knn_sharded."""
    _fields_ = [("stream", c_vp), ("Q", c_vp), ("ldq", c_i64), ("Qt", c_vp), ("qscale", c_vp), ("qstats", c_vp),
                ("G", c_vp), ("N", c_i64), ("ldg", c_i64), ("Gt", c_vp), ("gscale", c_vp), ("aux", c_vp),
                ("gmax", c_vp), ("index_base", c_i64), ("workspace", c_vp), ("workspace_bytes", c_sz),
                ("out_d", c_vp), ("out_i", c_vp), ("cert", c_vp),
                ("Gt2", c_vp), ("gscale2", c_vp), ("gmax2", c_vp), ("G8", c_vp), ("ld8", c_i64), ("gscale8", c_vp),
                ("gmax8", c_vp), ("tier_counts", c_vp), ("St", c_vp), ("Ns", c_i64), ("sscale", c_vp), ("saux", c_vp),
                ("St2", c_vp), ("bscale", c_vp),
                ("pstages", c_int), ("Qtp", c_vp), ("qscalep", c_vp), ("qstatsp", c_vp), ("paux", c_vp),
                ("spaux", c_vp), ("prefix_open", c_vp), ("Gtp", c_vp), ("gscalep", c_vp), ("gmaxp", c_vp)]


class OfrError(RuntimeError):
    """A libocvf_hip call failed (message from ofr_last_error()); .code = the ofr_status."""

    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


E_UNSUPPORTED, E_NUMERIC = -2, -4
OFR_FP64_ACC, OFR_PROJ_REUSE_W = 1, 2          # ofr_project_u8 flags


_lib = None
_lock = threading.Lock()
_checked_devices = set()


def load():
    """Load the shared library (no GPU needed) and bind every declared symbol."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise OfrError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def check(rc, what=""):
    if rc != 0:
        msg = load().ofr_last_error().decode(errors="replace")
        raise OfrError(f"{what or 'ofr'} failed ({rc}): {msg}", rc)


def device():
    """The torch device the kernels run on (raises without a gfx950 GPU)."""
    if not torch.cuda.is_available():
        raise OfrError("ocvfacerec (MI355X build): no HIP device visible — this implementation has no CPU path")
    idx = torch.cuda.current_device()
    if idx not in _checked_devices:
        check(load().ofr_device_check(idx), "ofr_device_check")
        _checked_devices.add(idx)
    return torch.device("cuda", idx)


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def call(name, *args):
    check(getattr(load(), name)(*args), name)
