"""ctypes binding of libcwq (include/cobweb_query.h).

The library is built in-tree (``__graft_entry__.build()`` / ``python -m
rag_cobweb_amd.build``) as ``rag-cobweb_amd/libcwq.so``.  There is no fallback: if
the library is missing or fails to load, every query entry point raises.
"""
import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CWQ_LIB") or os.path.join(HERE, "libcwq.so")   # CWQ_LIB: A/B experiments only

CWQ_OK = 0
CWQ_ERR_ARG = -1
CWQ_ERR_HIP = -2
CWQ_ERR_OOM = -3
CWQ_ERR_NOT_FOUND = -4

# symbol -> (restype, argtypes); mirrors include/cobweb_query.h
_c = ctypes
_P = _c.c_void_p
_I64 = _c.c_int64
_I32 = _c.c_int32
SIGNATURES = {
    "cwq_version": (_c.c_int, []),
    "cwq_build_id": (_c.c_char_p, []),
    "cwq_last_error": (_c.c_char_p, []),
    "cwq_index_create": (_c.c_int, [_c.c_int, _I64, _I32, _P, _P, _P, _P, _I64, _P, _I32, _P, _c.POINTER(_P)]),
    "cwq_index_create_cv": (_c.c_int, [_c.c_int, _I64, _I32, _P, _P, _P, _I64, _P, _P, _P, _I64, _P, _I32, _P,
                                       _c.POINTER(_P)]),
    "cwq_index_destroy": (_c.c_int, [_P]),
    "cwq_index_info": (_c.c_int, [_P, _P]),
    "cwq_index_filter_info": (_c.c_int, [_P, _P]),
    "cwq_index_cut_info": (_c.c_int, [_P, _P]),
    "cwq_last_lazy_stats": (_c.c_int, [_P, _P]),
    "cwq_score_topk": (_c.c_int, [_P, _P, _I64, _I32, _P, _P, _P]),
    "cwq_rank_scores": (_c.c_int, [_P, _P, _I64, _P, _P]),
    "cwq_node_logprob": (_c.c_int, [_P, _P, _I64, _I32, _P, _P]),
    "cwq_prefix_bounds": (_c.c_int, [_P, _P, _I64, _P, _P, _P, _P]),
    "cwq_categorize": (_c.c_int, [_P, _P, _I64, _I32, _I64, _P, _P, _P, _P]),
    "cwq_set_timing": (_c.c_int, [_P, _c.c_int]),
    "cwq_last_timing": (_c.c_int, [_P, _P]),
    "cwq_set_filter": (_c.c_int, [_P, _c.c_int]),
    "cwq_last_stats": (_c.c_int, [_P, _P]),
    "cwq_last_prune_stats": (_c.c_int, [_P, _P]),
    "cwq_score_topk_host": (_c.c_int, [_P, _P, _I64, _I32, _P, _P, _P]),
    "cwq_categorize_host": (_c.c_int, [_P, _P, _I64, _I32, _I64, _P, _P, _P, _P]),
    "cwq_whiten": (_c.c_int, [_P, _I64, _I32, _P, _P, _I32, _P, _P, _I32, _P, _P, _P]),
    "cwq_fit_kl": (_c.c_int, [_P, _P, _P, _I32, _P, _c.c_float, _I32, _P, _I32, _P, _P]),
    "cwq_fit_node_op": (_c.c_int, [_I32, _P, _P, _P, _I32, _I32, _I32, _P, _P, _P]),
    "cwq_welford_groups": (_c.c_int, [_P, _I64, _I32, _P, _P, _I64, _P, _P, _P, _P]),
    "cwq_fit_create": (_c.c_int, [_c.c_int, _I32, _c.c_float, _I32, _c.POINTER(_P)]),
    "cwq_fit_destroy": (_c.c_int, [_P]),
    "cwq_fit_load": (_c.c_int, [_P, _I32, _I32, _P, _P, _P, _P, _P, _P, _P, _P]),
    "cwq_fit_insert": (_c.c_int, [_P, _P, _I64, _P, _P, _P]),
    "cwq_fit_export": (_c.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "cwq_fit_last_error": (_c.c_char_p, []),
    "cwq_mt19937_draw": (_c.c_int, [_P, _I64, _P]),
    "cwq_mt19937_words": (_c.c_int, [_P, _I64, _P]),
    "cwq_mt19937_skip": (_c.c_int, [_P, _I64]),
}

_lock = threading.Lock()
_lib = None


class CwqError(RuntimeError):
    """A libcwq call returned an error status."""

    def __init__(self, rc, msg):
        super().__init__(f"libcwq error {rc}: {msg}")
        self.rc = rc


def load_library(path, strict=True):
    """A configured CDLL for a libcwq build at ``path``.  strict=False (A/B scripts
    loading older builds only) skips entry points the build does not export."""
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: build it with __graft_entry__.build()")
    L = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        if not strict and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def lib():
    """Load libcwq.so (once).  Raises ImportError when it is not built, or when it was
    built from other sources than the ones in csrc/ (stale binary: rebuild it)."""
    global _lib
    with _lock:
        if _lib is None:
            L = load_library(LIB_PATH)
            if not os.environ.get("CWQ_LIB"):
                from .build import source_id
                # the same extra flags build_library() stamps into the id (CWQ_HIPCC_FLAGS)
                got, want = L.cwq_build_id().decode(), source_id(os.environ.get("CWQ_HIPCC_FLAGS", "").split())
                if got != want:
                    raise ImportError(f"{LIB_PATH} was built from other sources (build id {got}, sources {want}): "
                                      f"rebuild it with __graft_entry__.build()")
            _lib = L
    return _lib


def check(rc):
    if rc != CWQ_OK:
        raise CwqError(rc, lib().cwq_last_error().decode(errors="replace"))
