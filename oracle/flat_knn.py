"""CPU ORACLE — test infrastructure only, never the product path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the *checker*.  The shipped search path
is the HIP library (``duckdb-lancedb_amd/csrc``) behind the C-ABI in
``include/lancedb_hip.h``; it never calls into ``oracle/``.

What it restates (reference paths relative to ``/root/reference``):

* ``rust_lib/src/lance_manager.rs:393-451`` — ``LanceIndex::search``: a flat
  (no ANN index) exact k-NN over every non-deleted row, ascending distance,
  ``label`` (Int64) + ``_distance`` (Float32) per hit, at most ``k`` hits.
  The query never sets ``distance_type`` (``:411-418``) so LanceDB ranks by its
  default, *squared* L2 (pinned by ``test/sql/lance_basic.test:33-42``:
  ``[1,0,0]`` vs ``[0,1,0]`` -> ``2.000000``).
* the distance definitions of the third-party ``lance-linalg 0.22.0``
  (``rust_lib/Cargo.lock:3048-3051``, source not in the container; restated
  from its published algorithm): ``l2 = sum((x-q)^2)`` (no sqrt),
  ``dot = 1 - x.q``, ``cosine = 1 - x.q / (|x| |q|)``.
* ``lance_manager.rs:227-242`` — labels are dense consecutive int64 starting at
  ``next_label``; ``:461-471`` deletes by label; ``:474-478`` counts live rows;
  ``:136-169`` + ``:662-696`` reopen with ``next_label = max(label) + 1``.
* ``src/lance_index.cpp:442-465`` — ``LanceIndex::Search``: dimension mismatch
  -> empty result (no error, ``lance_basic.test:55-59``), label -> row_id map,
  labels outside the map dropped.

Canonical numerics of this build (documented in DESIGN.md): every distance is
accumulated in float64 from the float32 inputs and rounded once to float32;
hits are ordered by (float32 distance ascending, label under the tie rule).  The
tie rule is label DESCENDING by default — the order the reference's own golden
shows at a tie (``test/sql/lance_optimizer_filter.test:36-44``: ids 3 and 4 tie
at d = 2.0 and LanceDB returns 4, the higher label) — or label ascending
(``tie="label_asc"``; ``LANCE_HIP_TIE`` sets the default, as it does for the
library's handles).  The reference's own f32 SIMD accumulation order is not
reproducible bit-for-bit, so distances are compared at 1e-4 relative
(BASELINE.json north_star) and ids bit-exactly under this order.
"""
from __future__ import annotations

import os

import numpy as np

METRICS = ("l2", "dot", "cosine")
TIES = ("label_desc", "label_asc")


def default_tie() -> str:
    """The tie rule a new handle gets: ``LANCE_HIP_TIE`` or label_desc."""
    return os.environ.get("LANCE_HIP_TIE") or "label_desc"


def tie_desc(tie: str | None) -> bool:
    t = tie or default_tie()
    if t in ("label_desc", "desc"):
        return True
    if t in ("label_asc", "asc"):
        return False
    raise ValueError(f"tie must be 'label_desc' or 'label_asc', got {t!r}")


def normalize_metric(metric: str) -> str:
    """Metric name mapping of ``lance_manager.rs:493-497`` / ``lance_optimizer.cpp:360-371``:
    ``cosine`` -> cosine, ``dot``/``ip`` -> dot, anything else -> l2."""
    m = (metric or "").lower()
    if m == "cosine":
        return "cosine"
    if m in ("dot", "ip"):
        return "dot"
    return "l2"


def exact_distances(base: np.ndarray, q: np.ndarray, metric: str = "l2") -> np.ndarray:
    """Exact distances (float64 accumulation, rounded once to float32) of every
    row of ``base`` [n, d] to the query ``q`` [d].  Direct form for l2."""
    metric = normalize_metric(metric)
    X = np.asarray(base, dtype=np.float32).astype(np.float64)
    qq = np.asarray(q, dtype=np.float32).astype(np.float64)
    if metric == "l2":
        diff = X - qq[None, :]
        d = np.einsum("ij,ij->i", diff, diff)
    elif metric == "dot":
        d = 1.0 - X @ qq
    else:
        xn = np.sqrt(np.einsum("ij,ij->i", X, X))
        qn = np.sqrt(qq @ qq)
        with np.errstate(divide="ignore", invalid="ignore"):
            d = 1.0 - (X @ qq) / (xn * qn)
    return d.astype(np.float32)


def _order(dist32: np.ndarray, labels: np.ndarray, tie: str | None = None) -> np.ndarray:
    """Indices sorting by (float32 distance asc, label under the tie rule); NaN sorts last."""
    key = np.where(np.isnan(dist32), np.float32(np.inf), dist32)
    nan_last = np.isnan(dist32).astype(np.int8)
    lab = np.asarray(labels, dtype=np.int64)
    return np.lexsort((-lab if tie_desc(tie) else lab, key, nan_last))


def flat_search(base: np.ndarray, labels: np.ndarray, live: np.ndarray, q: np.ndarray, k: int,
                metric: str = "l2", tie: str | None = None):
    """Exact flat top-k (restates ``lance_manager.rs:393-451``).

    Returns ``(labels int64[n_hit], distances float32[n_hit])`` with
    ``n_hit = min(k, live rows)``.
    """
    base = np.asarray(base, dtype=np.float32)
    labels = np.asarray(labels, dtype=np.int64)
    live = np.asarray(live, dtype=bool)
    if k <= 0 or base.shape[0] == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.float32)
    idx = np.nonzero(live)[0]
    if idx.size == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.float32)
    d = exact_distances(base[idx], q, metric)
    order = _order(d, labels[idx], tie)[:k]
    return labels[idx][order], d[order]


def flat_search_batch(base, labels, live, Q, k, metric="l2", prefilter_k=None, tie=None):
    """Batched exact top-k.  For large ``n`` the candidate set per query is first
    narrowed with a float64 expanded-form ranking (error ~1e-12 relative) and the
    survivors are re-scored with :func:`exact_distances`; the margin of
    ``prefilter_k`` extra rows makes the narrowing exact for continuous data."""
    base = np.asarray(base, dtype=np.float32)
    labels = np.asarray(labels, dtype=np.int64)
    live = np.asarray(live, dtype=bool)
    Q = np.asarray(Q, dtype=np.float32)
    metric = normalize_metric(metric)
    nq = Q.shape[0]
    out_l = np.full((nq, k), -1, np.int64)
    out_d = np.full((nq, k), np.nan, np.float32)
    counts = np.zeros(nq, np.int32)
    idx = np.nonzero(live)[0]
    if idx.size == 0 or k <= 0:
        return out_l, out_d, counts
    X = base[idx]
    L = labels[idx]
    n = X.shape[0]
    if prefilter_k is None:
        prefilter_k = k + 64
    if n <= 4 * prefilter_k:
        for i in range(nq):
            d = exact_distances(X, Q[i], metric)
            o = _order(d, L, tie)[:k]
            counts[i] = o.size
            out_l[i, :o.size] = L[o]
            out_d[i, :o.size] = d[o]
        return out_l, out_d, counts
    X64 = X.astype(np.float64)
    xn2 = np.einsum("ij,ij->i", X64, X64)
    for s in range(0, nq, 64):
        Qb = Q[s:s + 64].astype(np.float64)
        dots = Qb @ X64.T
        if metric == "l2":
            approx = xn2[None, :] - 2.0 * dots + np.einsum("ij,ij->i", Qb, Qb)[:, None]
        elif metric == "dot":
            approx = 1.0 - dots
        else:
            with np.errstate(divide="ignore", invalid="ignore"):
                approx = 1.0 - dots / (np.sqrt(xn2)[None, :] * np.sqrt(np.einsum("ij,ij->i", Qb, Qb))[:, None])
            approx = np.where(np.isnan(approx), np.inf, approx)
        m = min(prefilter_k, n)
        part = np.argpartition(approx, m - 1, axis=1)[:, :m]
        for j in range(Qb.shape[0]):
            cand = part[j]
            d = exact_distances(X[cand], Q[s + j], metric)
            o = _order(d, L[cand], tie)[:k]
            i = s + j
            counts[i] = o.size
            out_l[i, :o.size] = L[cand][o]
            out_d[i, :o.size] = d[o]
    return out_l, out_d, counts


def recall_at_k(found: np.ndarray, truth: np.ndarray, k: int) -> float:
    """mean |found[:k] ∩ truth[:k]| / k over queries (BASELINE.md formula)."""
    tot = 0.0
    for f, t in zip(found, truth):
        tot += len(set(f[:k].tolist()) & set(t[:k].tolist())) / float(k)
    return tot / max(1, len(found))


class DetachedIndexOracle:
    """State machine of one detached Lance table as seen through the C-ABI
    (``rust_lib/src/ffi.rs:37-541`` over ``lance_manager.rs``): dense labels,
    label deletes, live count, per-label vector lookup, reopen semantics."""

    def __init__(self, dim: int, metric: str = "l2", next_label: int = 0, tie: str | None = None):
        self.dim = int(dim)
        self.metric = metric
        self.tie = tie
        self.next_label = int(next_label)
        self.vectors: dict[int, np.ndarray] = {}

    # lance_manager.rs:227-242
    def add_batch(self, vectors: np.ndarray) -> np.ndarray:
        v = np.asarray(vectors, dtype=np.float32).reshape(-1, self.dim)
        labels = np.arange(self.next_label, self.next_label + v.shape[0], dtype=np.int64)
        self.next_label += v.shape[0]
        for lab, row in zip(labels, v):
            self.vectors[int(lab)] = row.copy()
        return labels

    # lance_manager.rs:461-471 (unknown labels are a no-op, as a SQL IN-delete is)
    def delete_batch(self, labels) -> None:
        for lab in labels:
            self.vectors.pop(int(lab), None)

    # lance_manager.rs:474-478
    def count(self) -> int:
        return len(self.vectors)

    # lance_manager.rs:136-169, :662-696
    def reopen(self) -> "DetachedIndexOracle":
        nxt = (max(self.vectors) + 1) if self.vectors else 0
        o = DetachedIndexOracle(self.dim, self.metric, nxt, self.tie)
        o.vectors = {k: v.copy() for k, v in self.vectors.items()}
        return o

    def arrays(self):
        labs = np.array(sorted(self.vectors), dtype=np.int64)
        if labs.size == 0:
            return np.zeros((0, self.dim), np.float32), labs
        return np.stack([self.vectors[int(l)] for l in labs]), labs

    # lance_manager.rs:393-451 (dimension mismatch is an error at this layer)
    def search(self, q, k: int, metric: str | None = None):
        q = np.asarray(q, dtype=np.float32)
        if q.shape[0] != self.dim:
            raise ValueError(f"expected query dimension {self.dim}, got {q.shape[0]}")
        X, L = self.arrays()
        return flat_search(X, L, np.ones(L.shape[0], bool), q, k, metric or self.metric, self.tie)


class LanceIndexOracle:
    """``src/lance_index.cpp`` semantics above the FFI: ``label_to_rowid_`` /
    ``rowid_to_label_`` maps, Search dim guard (``:442-465``), Delete (``:389-425``)."""

    def __init__(self, dim: int, metric: str = "l2", tie: str | None = None):
        self.dim = dim
        self.detached = DetachedIndexOracle(dim, metric, tie=tie)
        self.label_to_rowid: list[int] = []
        self.rowid_to_label: dict[int, int] = {}

    def append(self, vectors, row_ids):
        labels = self.detached.add_batch(vectors)
        for lab, rid in zip(labels, row_ids):
            while len(self.label_to_rowid) <= lab:
                self.label_to_rowid.append(-1)
            self.label_to_rowid[int(lab)] = int(rid)
            self.rowid_to_label[int(rid)] = int(lab)
        return labels

    def delete(self, row_ids):
        labs = []
        for rid in row_ids:
            lab = self.rowid_to_label.pop(int(rid), None)
            if lab is not None:
                labs.append(lab)
                self.label_to_rowid[lab] = -1
        self.detached.delete_batch(labs)

    def search(self, q, k: int):
        q = np.asarray(q, dtype=np.float32)
        if q.shape[0] != self.dim:
            return []
        labs, dists = self.detached.search(q, k)
        out = []
        for lab, d in zip(labs, dists):
            if 0 <= lab < len(self.label_to_rowid):
                out.append((self.label_to_rowid[int(lab)], float(d)))
        return out
