"""ctypes loader for oracle/build/liboracle_knn.so — TEST INFRASTRUCTURE ONLY.

Used by tests/ (checker at sizes where numpy is slow) and by bench.py's
``cpu_baseline`` leg (the timed "port" of the reference's flat search,
``rust_lib/src/lance_manager.rs:393-451``).  Never imported by the product.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle_knn.so")
_lib = None

METRIC_IDS = {"l2": 0, "dot": 1, "cosine": 2}


def build() -> str:
    import subprocess

    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        L.oracle_flat_search_batch.argtypes = [P, ctypes.c_int64, ctypes.c_int32, P, P, P, ctypes.c_int32,
                                               ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                               P, P, P]
        L.oracle_flat_search_batch.restype = ctypes.c_int
        L.oracle_distances.argtypes = [P, ctypes.c_int64, ctypes.c_int32, P, ctypes.c_int32, P]
        L.oracle_distances.restype = None
        I32, I64 = ctypes.c_int32, ctypes.c_int64
        L.oracle_ivf_search_batch.argtypes = [P, I32, P, P, P, I32, P, I64, P, P, I32, P, P, P, I32, I32, I32, I32,
                                              I32, I32, I32, I32, P, P, P]
        L.oracle_ivf_search_batch.restype = ctypes.c_int
        L.oracle_set_tie.argtypes = [ctypes.c_int32]
        L.oracle_set_tie.restype = None
        _lib = L
    return _lib


def _set_tie(tie):
    """The final order's tie rule for the next call (flat_knn.tie_desc:
    label_desc by default, LANCE_HIP_TIE / tie="label_asc" otherwise)."""
    t = tie or os.environ.get("LANCE_HIP_TIE") or "label_desc"
    if t not in ("label_desc", "desc", "label_asc", "asc"):
        raise ValueError(f"tie must be 'label_desc' or 'label_asc', got {t!r}")
    lib().oracle_set_tie(1 if t in ("label_desc", "desc") else 0)


def _ptr(a):
    return None if a is None else a.ctypes.data


def flat_search_batch(base, Q, k, metric="l2", live=None, labels=None, acc64=True, nthreads=0, tie=None):
    base = np.ascontiguousarray(base, dtype=np.float32)
    Q = np.ascontiguousarray(Q, dtype=np.float32)
    n, d = base.shape
    nq = Q.shape[0]
    live_a = None if live is None else np.ascontiguousarray(live, dtype=np.uint8)
    lab_a = None if labels is None else np.ascontiguousarray(labels, dtype=np.int64)
    out_l = np.empty((nq, k), np.int64)
    out_d = np.empty((nq, k), np.float32)
    cnt = np.empty(nq, np.int32)
    _set_tie(tie)
    rc = lib().oracle_flat_search_batch(_ptr(base), n, d, _ptr(live_a), _ptr(lab_a), _ptr(Q), nq, k,
                                        METRIC_IDS[metric], 1 if acc64 else 0, int(nthreads),
                                        _ptr(out_l), _ptr(out_d), _ptr(cnt))
    if rc != 0:
        raise MemoryError("oracle_flat_search_batch failed")
    return out_l, out_d, cnt


def distances(base, q, metric="l2"):
    base = np.ascontiguousarray(base, dtype=np.float32)
    q = np.ascontiguousarray(q, dtype=np.float32)
    out = np.empty(base.shape[0], np.float32)
    lib().oracle_distances(_ptr(base), base.shape[0], base.shape[1], _ptr(q), METRIC_IDS[metric], _ptr(out))
    return out


class IvfLayout:
    """CSR list layout of the LIVE indexed slots + the unindexed live tail, built
    once from ``lance_hip_ivf_export`` output (slot lists / live flags)."""

    def __init__(self, lists, live, nlist):
        lists = np.asarray(lists, np.int64)
        live = np.asarray(live, bool)
        idx = np.nonzero(live & (lists >= 0))[0]
        order = np.argsort(lists[idx], kind="stable")
        self.lrows = np.ascontiguousarray(idx[order], np.int64)
        cnt = np.bincount(lists[idx], minlength=nlist)
        self.loff = np.zeros(nlist + 1, np.int64)
        np.cumsum(cnt, out=self.loff[1:])
        self.tail = np.ascontiguousarray(np.nonzero(live & (lists < 0))[0], np.int64)
        self.nlist = nlist


def ivf_search_batch(base, labels, layout, centroids, Q, k, nprobe, metric="l2", codes=None, codebook=None, T=None,
                     refine_factor=1, acc64=True, nthreads=0, lut="f32", query_fp8=False, tie=None):
    """IVF_FLAT (codes None) / IVF_PQ search of oracle/flat_knn.c over a given
    model and layout.  base / labels / codes are per slot.  l2 and dot only.
    lut "u8": the fast scan's 8-bit LUT; query_fp8: ADC tables from e4m3 queries
    (oracle/ivf.py's definitions)."""
    base = np.ascontiguousarray(base, np.float32)
    Q = np.ascontiguousarray(Q, np.float32)
    labels = np.ascontiguousarray(labels, np.int64)
    C = np.ascontiguousarray(centroids, np.float32)
    nq, d = Q.shape
    m = 0
    if codes is not None:
        codes = np.ascontiguousarray(codes, np.uint8)
        codebook = np.ascontiguousarray(codebook, np.float32)
        m = codes.shape[1]
        T = None if T is None else np.ascontiguousarray(T, np.float32)
    out_l = np.empty((nq, k), np.int64)
    out_d = np.empty((nq, k), np.float32)
    cnt = np.empty(nq, np.int32)
    _set_tie(tie)
    rc = lib().oracle_ivf_search_batch(_ptr(base), d, _ptr(labels), _ptr(layout.loff), _ptr(layout.lrows),
                                       layout.nlist, _ptr(layout.tail), len(layout.tail), _ptr(C), _ptr(codes), m,
                                       _ptr(codebook), _ptr(T), _ptr(Q), nq, k, nprobe, refine_factor,
                                       METRIC_IDS[metric], 1 if acc64 else 0,
                                       (1 if lut == "u8" else 0) | (2 if query_fp8 else 0), int(nthreads), _ptr(out_l),
                                       _ptr(out_d), _ptr(cnt))
    if rc != 0:
        raise ValueError(f"oracle_ivf_search_batch failed ({rc})")
    return out_l, out_d, cnt
