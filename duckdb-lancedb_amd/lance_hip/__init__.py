"""Host-side mirror of the reference's operator interface over the HIP C-ABI.

The reference's DuckDB operator layer (``src/*.cpp`` under ``/root/reference``)
cannot be compiled here (empty ``duckdb/`` submodule), so this
module restates the two C++ layers that sit on the hot path above the C-ABI,
with the reference's names, argument meaning and error behaviour:

* ``rust_ffi.cpp`` — one wrapper per C symbol, 2048-byte error buffer
  (``rust_ffi.cpp:44``), raising :class:`IOException` ``"Lance <op>: <msg>"``
  on a NULL / negative / non-zero return (``rust_ffi.cpp:53-55`` etc.);
* ``lance_index.cpp`` — :class:`LanceIndex` with ``Append`` / ``Delete`` /
  ``Search`` (dimension guard ``:444-446``, label -> row_id map ``:455-462``)
  and the ``metric`` / ``nprobes`` / ``refine_factor`` options
  (``lance_index.cpp:157-165``, defaults ``lance_index.hpp:90-92``).

The library is ``lib/liblancedb_hip.so`` next to this package (built by
``make -C duckdb-lancedb_amd``).  There is no fallback: if the library is
missing, importing :func:`lib` raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_PKG_DIR), "lib", "liblancedb_hip.so")
# development override (ablation builds); the shipped path is LIB_PATH
LIB_PATH = os.environ.get("LANCE_HIP_LIB") or LIB_PATH
ERR_BUF_LEN = 2048  # rust_ffi.cpp:44

_lib = None

c_void_p = ctypes.c_void_p
c_char_p = ctypes.c_char_p
c_int = ctypes.c_int
i32 = ctypes.c_int32
i64 = ctypes.c_int64

# (name, restype, argtypes) — exactly include/lancedb_hip.h
_SIGNATURES = [
    ("lance_create_detached", c_void_p, [c_char_p, i32, c_char_p, c_char_p, c_char_p, c_int]),
    ("lance_create_detached_from_arrow", c_void_p, [c_char_p, c_void_p, c_char_p, c_char_p, c_char_p, c_int]),
    ("lance_open_detached", c_void_p, [c_char_p, c_char_p, c_char_p, c_char_p, c_int]),
    ("lance_free_detached", None, [c_void_p]),
    ("lance_detached_has_extra_columns", i32, [c_void_p]),
    ("lance_detached_dimension", i32, [c_void_p]),
    ("lance_detached_add", i64, [c_void_p, c_void_p, i32, c_char_p, c_int]),
    ("lance_detached_add_batch", i32, [c_void_p, c_void_p, i32, i32, c_void_p, c_char_p, c_int]),
    ("lance_detached_add_batch_arrow", i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_char_p, c_int]),
    ("lance_detached_merge", i32, [c_void_p, c_void_p, c_void_p, i32, c_void_p, c_void_p, c_char_p, c_int]),
    ("lance_detached_search", i32, [c_void_p, c_void_p, i32, i32, i32, i32, c_void_p, c_void_p, c_char_p, c_int]),
    ("lance_detached_search_with_predicate", i32,
     [c_void_p, c_void_p, i32, i32, i32, i32, c_char_p, c_void_p, c_void_p, c_char_p, c_int]),
    ("lance_detached_search_batch", i32,
     [c_void_p, c_void_p, i32, i32, i32, i32, i32, c_char_p, c_void_p, c_void_p, c_void_p, c_char_p, c_int]),
    ("lance_detached_count", i64, [c_void_p, c_char_p, c_int]),
    ("lance_detached_delete", i32, [c_void_p, i64, c_char_p, c_int]),
    ("lance_detached_delete_batch", i32, [c_void_p, c_void_p, i32, c_char_p, c_int]),
    ("lance_detached_create_index", i32, [c_void_p, i32, i32, c_char_p, c_int]),
    ("lance_detached_create_hnsw_index", i32, [c_void_p, i32, i32, c_char_p, c_int]),
    ("lance_detached_compact", i32, [c_void_p, c_char_p, c_int]),
    ("lance_detached_get_vector", i32, [c_void_p, i64, c_void_p, i32, c_char_p, c_int]),
    ("lance_detached_get_all_vectors", i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_char_p, c_int]),
    ("lance_hip_version", c_char_p, []),
    ("lance_hip_device_count", i32, []),
    ("lance_hip_set_option", i32, [c_void_p, c_char_p, c_char_p, c_char_p, c_int]),
    ("lance_hip_last_search_stats", i32, [c_void_p, c_void_p, i32]),
    ("lance_hip_merge_topk", i32,
     [i32, i32, i32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_char_p, c_int]),
    ("lance_hip_add_batch_device", i64, [c_void_p, c_void_p, i64, i32, c_char_p, c_int]),
    ("lance_hip_search_batch_device", i32,
     [c_void_p, c_void_p, i32, i32, i32, i32, i32, c_void_p, c_void_p, c_void_p, c_char_p, c_int]),
    ("lance_hip_kernel_times", i32, [c_void_p, c_void_p, i32]),
    ("lance_hip_search_batch_device_async", i64,
     [c_void_p, c_void_p, i32, i32, i32, i32, i32, c_void_p, c_void_p, c_void_p, c_char_p, c_int]),
    ("lance_hip_search_wait", i32, [c_void_p, i64, c_char_p, c_int]),
    ("lance_hip_stream_after", i32, [c_void_p, c_void_p, c_char_p, c_int]),
    ("lance_hip_merge_topk_device", i32,
     [i32, i32, i32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_char_p, c_int]),
    ("lance_hip_merge_packed_stride", i64, [i32, i32]),
    ("lance_hip_merge_topk_packed", i32,
     [i32, i32, i32, c_void_p, i64, c_void_p, c_void_p, c_void_p, c_char_p, c_int]),
    ("lance_hip_ivf_info", i32, [c_void_p, c_void_p, i32]),
    ("lance_hip_ivf_export", i32,
     [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_char_p, c_int]),
    ("lance_hip_ivf_set_model", i32, [c_void_p, i32, i32, i32, c_void_p, c_void_p, c_char_p, c_int]),
    ("lance_hip_predicate_mask", i64,
     [c_void_p, c_void_p, c_void_p, c_void_p, c_char_p, c_char_p, c_void_p, c_char_p, c_int]),
    ("lance_detached_create_scalar_index", i32, [c_void_p, c_char_p, c_char_p, c_char_p, c_int]),
]

EXPORTED_SYMBOLS = [s[0] for s in _SIGNATURES]


class IOException(RuntimeError):
    """DuckDB ``IOException`` raised by the reference's ``rust_ffi.cpp`` wrappers."""


def lib():
    """Load ``liblancedb_hip.so`` (raises if it was not built — no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built; run `make -C duckdb-lancedb_amd` (or __graft_entry__.build())")
        # ONE HIP runtime per process: torch's wheel bundles its own libamdhip64 /
        # libhsa-runtime64 (soname libamdhip64.so.7, but torch NEEDs it as
        # "libamdhip64.so"), so loading this library first maps /opt/rocm's copy
        # and a later `import torch` maps a second one; two HSA runtimes in one
        # process leave the second to initialise without a device.  With torch
        # loaded first, this library's libamdhip64.so.7 resolves to torch's copy.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in _SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _err():
    return ctypes.create_string_buffer(ERR_BUF_LEN)


def _b(s: Optional[str]):
    return None if s is None else s.encode()


def _f32(a, dim=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a


def version() -> str:
    return lib().lance_hip_version().decode()


def device_count() -> int:
    return int(lib().lance_hip_device_count())


# ---------------------------------------------------------------------------
# rust_ffi.cpp wrappers (same names, same error behaviour)
# ---------------------------------------------------------------------------
def LanceCreateDetached(db_path: str, dimension: int, metric: str, table_name: str):
    e = _err()
    h = lib().lance_create_detached(_b(db_path), int(dimension), _b(metric), _b(table_name), e, ERR_BUF_LEN)
    if not h:
        raise IOException("Lance create: " + e.value.decode())
    return h


def LanceCreateDetachedFromArrow(db_path: str, arrow_schema, metric: str, table_name: str):
    e = _err()
    h = lib().lance_create_detached_from_arrow(_b(db_path), arrow_schema, _b(metric), _b(table_name), e, ERR_BUF_LEN)
    if not h:
        raise IOException("Lance create_from_arrow: " + e.value.decode())
    return h


def LanceOpenDetached(db_path: str, table_name: str, metric: str):
    e = _err()
    h = lib().lance_open_detached(_b(db_path), _b(table_name), _b(metric), e, ERR_BUF_LEN)
    if not h:
        raise IOException("Lance open: " + e.value.decode())
    return h


def LanceFreeDetached(handle) -> None:
    lib().lance_free_detached(handle)


def LanceDetachedHasExtraColumns(handle) -> bool:
    return lib().lance_detached_has_extra_columns(handle) != 0


def LanceDetachedDimension(handle) -> int:
    return int(lib().lance_detached_dimension(handle))


def LanceDetachedAdd(handle, vector, dimension: int) -> int:
    v = _f32(vector)
    e = _err()
    label = lib().lance_detached_add(handle, v.ctypes.data, int(dimension), e, ERR_BUF_LEN)
    if label < 0:
        raise IOException("Lance add: " + e.value.decode())
    return int(label)


def LanceDetachedAddBatch(handle, vectors, num: int, dim: int) -> np.ndarray:
    v = _f32(vectors)
    out = np.empty(max(int(num), 0), np.int64)
    e = _err()
    n = lib().lance_detached_add_batch(handle, v.ctypes.data, int(num), int(dim), out.ctypes.data, e, ERR_BUF_LEN)
    if n < 0:
        raise IOException("Lance add_batch: " + e.value.decode())
    return out[:n]


def LanceDetachedAddBatchArrow(handle, arrow_schema, arrow_array) -> np.ndarray:
    """arrow_schema / arrow_array: addresses of Arrow C Data Interface structs
    (ArrowC.export); the array is taken over by the library."""
    e = _err()
    n_rows = ctypes.c_int64.from_address(int(arrow_array)).value  # ArrowArray.length
    out = np.empty(max(n_rows, 1), np.int64)
    n = lib().lance_detached_add_batch_arrow(handle, arrow_schema, arrow_array, out.ctypes.data, e, ERR_BUF_LEN)
    if n < 0:
        raise IOException("Lance add_batch_arrow: " + e.value.decode())
    return out[:n]


class _ArrowSchemaC(ctypes.Structure):
    _fields_ = [("format", ctypes.c_char_p), ("name", ctypes.c_char_p), ("metadata", ctypes.c_char_p),
                ("flags", ctypes.c_int64), ("n_children", ctypes.c_int64), ("children", ctypes.c_void_p),
                ("dictionary", ctypes.c_void_p), ("release", ctypes.c_void_p), ("private_data", ctypes.c_void_p)]


class _ArrowArrayC(ctypes.Structure):
    _fields_ = [("length", ctypes.c_int64), ("null_count", ctypes.c_int64), ("offset", ctypes.c_int64),
                ("n_buffers", ctypes.c_int64), ("n_children", ctypes.c_int64), ("buffers", ctypes.c_void_p),
                ("children", ctypes.c_void_p), ("dictionary", ctypes.c_void_p), ("release", ctypes.c_void_p),
                ("private_data", ctypes.c_void_p)]


_ARROW_RELEASE = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


class ArrowC:
    """Arrow C Data Interface structs of a pyarrow StructArray (what DuckDB's
    ArrowConverter hands the reference's FFI, lance_index.cpp:340-354).  The
    structs are released on close() unless the library took them over."""

    def __init__(self, struct_array):
        self.schema = _ArrowSchemaC()
        self.array = _ArrowArrayC()
        struct_array._export_to_c(ctypes.addressof(self.array), ctypes.addressof(self.schema))

    @property
    def schema_ptr(self):
        return ctypes.addressof(self.schema)

    @property
    def array_ptr(self):
        return ctypes.addressof(self.array)

    def close(self):
        for st in (self.array, self.schema):
            if st.release:
                _ARROW_RELEASE(st.release)(ctypes.addressof(st))

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def arrow_rows(vectors, extras=None, vector_name="vector"):
    """StructArray [vector FixedSizeList<float32>[d], extra columns...];
    extras: list of (name, pyarrow array or python list, pyarrow type or None)."""
    import pyarrow as pa

    v = np.ascontiguousarray(vectors, dtype=np.float32)
    n, d = v.shape
    vec = pa.FixedSizeListArray.from_arrays(pa.array(v.reshape(-1), pa.float32()), d)
    arrays, names = [vec], [vector_name]
    for name, vals, typ in (extras or []):
        arrays.append(vals if isinstance(vals, pa.Array) else pa.array(vals, typ))
        names.append(name)
    return pa.StructArray.from_arrays(arrays, names=names)


def LanceDetachedCreateScalarIndex(handle, column: str, index_type: str = "BTREE") -> None:
    """``LanceDetachedCreateScalarIndex`` as ``lance_index.cpp:481-486`` calls it."""
    e = _err()
    if lib().lance_detached_create_scalar_index(handle, _b(column), _b(index_type), e, ERR_BUF_LEN) != 0:
        raise IOException("Lance create_scalar_index: " + e.value.decode())


def LanceHipPredicateMask(struct_array, labels, live, predicate: str, indexed_columns=()) -> np.ndarray:
    """The library's predicate evaluator over a host Arrow batch (no device);
    indexed_columns go through a scalar index."""
    n = len(struct_array)
    lab = np.ascontiguousarray(labels, np.int64)
    lv = np.ascontiguousarray(live, np.uint8)
    out = np.zeros(max(n, 1), np.uint8)
    e = _err()
    with ArrowC(struct_array) as a:
        c = lib().lance_hip_predicate_mask(a.schema_ptr, a.array_ptr, lab.ctypes.data, lv.ctypes.data,
                                           _b(predicate), _b(",".join(indexed_columns)), out.ctypes.data, e,
                                           ERR_BUF_LEN)
    if c < 0:
        raise IOException("Lance predicate: " + e.value.decode())
    return out[:n].astype(bool)


def LanceDetachedMerge(target, source, live_source_labels):
    labs = np.ascontiguousarray(live_source_labels, dtype=np.int64)
    old = np.empty(max(labs.size, 1), np.int64)
    new = np.empty(max(labs.size, 1), np.int64)
    e = _err()
    n = lib().lance_detached_merge(target, source, labs.ctypes.data, int(labs.size), old.ctypes.data, new.ctypes.data,
                                   e, ERR_BUF_LEN)
    if n < 0:
        raise IOException("Lance merge: " + e.value.decode())
    return old[:n], new[:n]


def LanceDetachedSearch(handle, query, dim: int, k: int, nprobes: int = 20, refine_factor: int = 1,
                        predicate: Optional[str] = None):
    """``LanceDetachedSearch`` (``rust_ffi.cpp:130-139``); with ``predicate`` it
    is the intended 9-argument form called at ``lance_index.cpp:452-453``."""
    q = _f32(query)
    kk = max(int(k), 0)
    labels = np.empty(max(kk, 1), np.int64)
    dists = np.empty(max(kk, 1), np.float32)
    e = _err()
    if predicate is None:
        n = lib().lance_detached_search(handle, q.ctypes.data, int(dim), int(k), int(nprobes), int(refine_factor),
                                        labels.ctypes.data, dists.ctypes.data, e, ERR_BUF_LEN)
    else:
        n = lib().lance_detached_search_with_predicate(handle, q.ctypes.data, int(dim), int(k), int(nprobes),
                                                       int(refine_factor), _b(predicate), labels.ctypes.data,
                                                       dists.ctypes.data, e, ERR_BUF_LEN)
    if n < 0:
        raise IOException("Lance search: " + e.value.decode())
    return labels[:n], dists[:n]


def LanceDetachedSearchBatch(handle, queries, k: int, nprobes: int = 20, refine_factor: int = 1,
                             predicate: Optional[str] = None):
    Q = _f32(queries)
    if Q.ndim == 1:
        Q = Q[None, :]
    nq, dim = Q.shape
    labels = np.empty((nq, max(k, 1)), np.int64)
    dists = np.empty((nq, max(k, 1)), np.float32)
    counts = np.empty(max(nq, 1), np.int32)
    e = _err()
    n = lib().lance_detached_search_batch(handle, Q.ctypes.data, int(nq), int(dim), int(k), int(nprobes),
                                          int(refine_factor), _b(predicate), labels.ctypes.data, dists.ctypes.data,
                                          counts.ctypes.data, e, ERR_BUF_LEN)
    if n < 0:
        raise IOException("Lance search: " + e.value.decode())
    return labels[:, :k], dists[:, :k], counts[:nq]


def LanceDetachedCount(handle) -> int:
    e = _err()
    n = lib().lance_detached_count(handle, e, ERR_BUF_LEN)
    if n < 0:
        raise IOException("Lance count: " + e.value.decode())
    return int(n)


def LanceDetachedDelete(handle, label: int) -> None:
    e = _err()
    if lib().lance_detached_delete(handle, int(label), e, ERR_BUF_LEN) != 0:
        raise IOException("Lance delete: " + e.value.decode())


def LanceDetachedDeleteBatch(handle, labels) -> None:
    labs = np.ascontiguousarray(labels, dtype=np.int64)
    e = _err()
    if lib().lance_detached_delete_batch(handle, labs.ctypes.data, int(labs.size), e, ERR_BUF_LEN) != 0:
        raise IOException("Lance delete_batch: " + e.value.decode())


def LanceDetachedCreateIndex(handle, num_partitions: int, num_sub_vectors: int) -> None:
    e = _err()
    if lib().lance_detached_create_index(handle, int(num_partitions), int(num_sub_vectors), e, ERR_BUF_LEN) != 0:
        raise IOException("Lance create_index: " + e.value.decode())


def LanceDetachedCreateHnswIndex(handle, m: int, ef_construction: int) -> None:
    e = _err()
    if lib().lance_detached_create_hnsw_index(handle, int(m), int(ef_construction), e, ERR_BUF_LEN) != 0:
        raise IOException("Lance create_hnsw_index: " + e.value.decode())


def LanceDetachedCompact(handle) -> None:
    e = _err()
    if lib().lance_detached_compact(handle, e, ERR_BUF_LEN) != 0:
        raise IOException("Lance compact: " + e.value.decode())


def LanceDetachedGetVector(handle, label: int, capacity: int) -> np.ndarray:
    out = np.empty(max(int(capacity), 1), np.float32)
    e = _err()
    d = lib().lance_detached_get_vector(handle, int(label), out.ctypes.data, int(capacity), e, ERR_BUF_LEN)
    if d < 0:
        raise IOException("Lance get_vector: " + e.value.decode())
    return out[:d]


def LanceDetachedGetAllVectors(handle):
    cnt = ctypes.c_int64(0)
    e = _err()
    n = lib().lance_detached_get_all_vectors(handle, None, None, ctypes.byref(cnt), e, ERR_BUF_LEN)
    if n < 0:
        raise IOException("Lance get_all_vectors: " + e.value.decode())
    dim = LanceDetachedDimension(handle)
    labels = np.empty(max(cnt.value, 1), np.int64)
    vecs = np.empty((max(cnt.value, 1), dim), np.float32)
    n = lib().lance_detached_get_all_vectors(handle, labels.ctypes.data, vecs.ctypes.data, ctypes.byref(cnt), e,
                                             ERR_BUF_LEN)
    if n < 0:
        raise IOException("Lance get_all_vectors: " + e.value.decode())
    return labels[:n], vecs[:n]


def LanceHipSetOption(handle, key: str, value: str) -> None:
    e = _err()
    if lib().lance_hip_set_option(handle, _b(key), _b(str(value)), e, ERR_BUF_LEN) != 0:
        raise IOException("Lance set_option: " + e.value.decode())


def LanceHipLastSearchStats(handle) -> dict:
    out = np.zeros(6, np.int64)
    lib().lance_hip_last_search_stats(handle, out.ctypes.data, 6)
    return {"fallback_queries": int(out[0]), "refined": int(out[1]), "max_pool": int(out[2]),
            "dense_path": bool(out[3]), "small_exact": int(out[3]) == 2, "retried_queries": int(out[4]),
            "append_launches": int(out[5])}


def LanceHipKernelTimes(handle) -> dict:
    out = np.zeros(13, np.float64)
    lib().lance_hip_kernel_times(handle, out.ctypes.data, 13)
    return {"scan_ms_total": float(out[0]), "scan_launches": int(out[1]), "scan_rows": int(out[2]),
            "scan_qpad": int(out[3]), "dense_ms_total": float(out[4]), "dense_launches": int(out[5]),
            "scan_elem_bytes": int(out[6]), "ivf_scan_ms_total": float(out[7]), "ivf_scan_launches": int(out[8]),
            "ivf_scan_bytes": float(out[9]), "ivf_pair_rows": float(out[10]), "ivf_coarse_ms_total": float(out[11]),
            "scan_kernel": {2: "scan8_kernel"}.get(int(out[12]), "scan_kernel")}


IVF_TYPES = {-1: None, 0: "ivf_flat", 1: "ivf_pq"}


def LanceHipIvfInfo(handle) -> dict:
    """IVF state of a handle: type (None when the table has no index), nlist,
    m (sub-vectors), dsub, rows indexed, slots."""
    out = np.zeros(6, np.int64)
    lib().lance_hip_ivf_info(handle, out.ctypes.data, 6)
    return {"type": IVF_TYPES[int(out[0])], "nlist": int(out[1]), "m": int(out[2]), "dsub": int(out[3]),
            "n_indexed": int(out[4]), "n_slots": int(out[5])}


def LanceHipIvfExport(handle) -> dict:
    """Host copy of the IVF model and of the per-slot layout (for the oracle):
    centroids [nlist, dim], codebook [m, 256, dsub] (IVF_PQ), and per slot:
    label, live flag, list (-1 = not indexed yet), codes [m]."""
    info = LanceHipIvfInfo(handle)
    if info["type"] is None:
        raise IOException("Lance ivf_export: no IVF index")
    dim = LanceDetachedDimension(handle)
    ns = info["n_slots"]
    C = np.zeros((info["nlist"], dim), np.float32)
    pq = info["type"] == "ivf_pq"
    cb = np.zeros((info["m"], 256, info["dsub"]), np.float32) if pq else None
    labels = np.zeros(ns, np.int64)
    live = np.zeros(ns, np.uint8)
    lists = np.zeros(ns, np.int32)
    codes = np.zeros((ns, max(info["m"], 1)), np.uint8)
    e = _err()
    r = lib().lance_hip_ivf_export(handle, C.ctypes.data, cb.ctypes.data if pq else None, labels.ctypes.data,
                                   live.ctypes.data, lists.ctypes.data, codes.ctypes.data if pq else None, e,
                                   ERR_BUF_LEN)
    if r != 0:
        raise IOException("Lance ivf_export: " + e.value.decode())
    return {**info, "centroids": C, "codebook": cb, "labels": labels, "live": live.astype(bool), "lists": lists,
            "codes": codes if pq else None}


def LanceHipIvfSetModel(handle, index_type: str, centroids, codebook=None) -> None:
    """Install a trained IVF model (rank 0's, on every rank) and index this
    handle's rows with it."""
    C = np.ascontiguousarray(centroids, dtype=np.float32)
    t = {"ivf_flat": 0, "ivf_pq": 1}[index_type]
    cb = None if codebook is None else np.ascontiguousarray(codebook, dtype=np.float32)
    m = 0 if cb is None else cb.shape[0]
    e = _err()
    r = lib().lance_hip_ivf_set_model(handle, t, C.shape[0], m, C.ctypes.data, None if cb is None else cb.ctypes.data,
                                      e, ERR_BUF_LEN)
    if r != 0:
        raise IOException("Lance ivf_set_model: " + e.value.decode())


def LanceHipMergeTopk(part_labels, part_dists, part_counts):
    """Merge per-shard partial top-k (nshard x nq x k) into the global top-k."""
    pl = np.ascontiguousarray(part_labels, dtype=np.int64)
    pd = np.ascontiguousarray(part_dists, dtype=np.float32)
    pc = np.ascontiguousarray(part_counts, dtype=np.int32)
    nshard, nq, k = pl.shape
    ol = np.empty((nq, k), np.int64)
    od = np.empty((nq, k), np.float32)
    oc = np.empty(nq, np.int32)
    e = _err()
    n = lib().lance_hip_merge_topk(nshard, nq, k, pl.ctypes.data, pd.ctypes.data, pc.ctypes.data, ol.ctypes.data,
                                   od.ctypes.data, oc.ctypes.data, e, ERR_BUF_LEN)
    if n < 0:
        raise IOException("Lance merge_topk: " + e.value.decode())
    return ol, od, oc


# ---------------------------------------------------------------------------
# lance_index.cpp: LanceIndex (the BoundIndex) — hot-path subset
# ---------------------------------------------------------------------------
class LanceIndex:
    """Mirror of ``src/lance_index.cpp`` ``LanceIndex`` for the search path.

    ``options`` keys as in ``CREATE INDEX ... USING LANCE (...) WITH (...)``:
    ``metric`` (default ``"l2"``), ``nprobes`` (20), ``refine_factor`` (1).
    Row ids are DuckDB row ids supplied by the caller (``Append``), mapped to
    labels exactly as ``label_to_rowid_`` / ``rowid_to_label_`` do.
    """

    def __init__(self, name: str, dimension: int, options: Optional[dict] = None, lance_path: str = "",
                 table_name: str = "vectors", extra_columns=None):
        """extra_columns: [(name, pyarrow type)] of a multi-column index
        (``CREATE INDEX .. USING LANCE (embedding, lang, score)``,
        lance_index.cpp:283-312 ``has_extra_columns_``)."""
        options = dict(options or {})
        self.extra_columns_ = list(extra_columns or [])
        self.has_extra_columns_ = bool(self.extra_columns_)
        self.name = name
        self.metric_ = str(options.get("metric", "l2"))
        self.nprobes_ = int(options.get("nprobes", 20))
        self.refine_factor_ = int(options.get("refine_factor", 1))
        self.dimension_ = int(dimension)
        self.lance_path_ = lance_path
        self.table_name_ = table_name
        self.rust_handle_ = None
        self.label_to_rowid_: list[int] = []
        self.rowid_to_label_: dict[int, int] = {}
        self.has_pending_deletes_ = False

    # lance_index.cpp:273-383 (Append; lazily creates the dataset :283-312)
    def Append(self, vectors, row_ids, extras: Optional[dict] = None) -> None:
        """extras: {column name: values} of the extra columns (multi-column index)."""
        v = np.ascontiguousarray(vectors, dtype=np.float32).reshape(-1, self.dimension_)
        if v.shape[0] == 0:
            return
        if self.has_extra_columns_:
            # Arrow C Data Interface path (lance_index.cpp:322-360)
            cols = [(nm, (extras or {}).get(nm, [None] * v.shape[0]), typ) for nm, typ in self.extra_columns_]
            batch = arrow_rows(v, cols)
            if self.rust_handle_ is None:
                with ArrowC(batch) as sch:
                    self.rust_handle_ = LanceCreateDetachedFromArrow(self.lance_path_, sch.schema_ptr, self.metric_,
                                                                     self.table_name_)
            with ArrowC(batch) as a:
                labels = LanceDetachedAddBatchArrow(self.rust_handle_, a.schema_ptr, a.array_ptr)
        else:
            if self.rust_handle_ is None:
                self.rust_handle_ = LanceCreateDetached(self.lance_path_, self.dimension_, self.metric_,
                                                        self.table_name_)
            labels = LanceDetachedAddBatch(self.rust_handle_, v, v.shape[0], self.dimension_)
        for lab, rid in zip(labels.tolist(), list(row_ids)):
            while len(self.label_to_rowid_) <= lab:
                self.label_to_rowid_.append(-1)
            self.label_to_rowid_[lab] = int(rid)
            self.rowid_to_label_[int(rid)] = lab

    Insert = Append

    # lance_index.cpp:389-425
    def Delete(self, row_ids) -> None:
        labels = []
        for rid in row_ids:
            lab = self.rowid_to_label_.pop(int(rid), None)
            if lab is not None:
                labels.append(lab)
                if 0 <= lab < len(self.label_to_rowid_):
                    self.label_to_rowid_[lab] = -1
        if self.rust_handle_ is not None and labels:
            LanceDetachedDeleteBatch(self.rust_handle_, labels)
            self.has_pending_deletes_ = True

    # lance_index.cpp:442-465
    def Search(self, query, dimension: int, k: int, predicate: str = ""):
        if self.rust_handle_ is None or int(dimension) != self.dimension_:
            return []
        labels, dists = LanceDetachedSearch(self.rust_handle_, query, dimension, k, self.nprobes_,
                                            self.refine_factor_, predicate if predicate else None)
        out = []
        for lab, d in zip(labels.tolist(), dists.tolist()):
            if 0 <= lab < len(self.label_to_rowid_):
                out.append((self.label_to_rowid_[lab], d))
        return out

    # lance_index.cpp:467-479
    def CreateAnnIndex(self, num_partitions: int, num_sub_vectors: int) -> None:
        if self.rust_handle_ is None:
            raise IOException("Lance index not initialized")
        LanceDetachedCreateIndex(self.rust_handle_, num_partitions, num_sub_vectors)

    # lance_index.cpp:481-486
    def CreateScalarIndex(self, column: str, index_type: str) -> None:
        if self.rust_handle_ is None:
            raise IOException("Lance index not initialized")
        LanceDetachedCreateScalarIndex(self.rust_handle_, column, index_type)

    def CreateHnswIndex(self, m: int, ef_construction: int) -> None:
        if self.rust_handle_ is None:
            raise IOException("Lance index not initialized")
        LanceDetachedCreateHnswIndex(self.rust_handle_, m, ef_construction)

    def GetVectorCount(self) -> int:
        return LanceDetachedCount(self.rust_handle_) if self.rust_handle_ is not None else 0

    def GetDimension(self) -> int:
        return self.dimension_

    def GetMetric(self) -> str:
        return self.metric_

    # persistence: metadata serialised by DuckDB (lance_index.cpp:492-532),
    # vectors reopened from the table log (:534-587 -> LanceOpenDetached)
    def Serialize(self) -> dict:
        return {"table_name": self.table_name_, "label_to_rowid": list(self.label_to_rowid_),
                "dim": self.dimension_, "nprobes": self.nprobes_, "refine_factor": self.refine_factor_,
                "metric": self.metric_, "lance_path": self.lance_path_}

    @classmethod
    def LoadFromStorage(cls, name: str, meta: dict) -> "LanceIndex":
        ix = cls(name, meta["dim"], {"metric": meta["metric"], "nprobes": meta["nprobes"],
                                     "refine_factor": meta["refine_factor"]}, meta["lance_path"], meta["table_name"])
        ix.label_to_rowid_ = list(meta["label_to_rowid"])
        ix.rowid_to_label_ = {r: l for l, r in enumerate(ix.label_to_rowid_) if r >= 0}
        ix.rust_handle_ = LanceOpenDetached(ix.lance_path_, ix.table_name_, ix.metric_)
        return ix

    # lance_index.cpp:427-436 (CommitDrop)
    def CommitDrop(self) -> None:
        if self.rust_handle_ is not None:
            LanceFreeDetached(self.rust_handle_)
            self.rust_handle_ = None

    def __del__(self):
        try:
            self.CommitDrop()
        except Exception:
            pass
