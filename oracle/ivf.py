"""CPU ORACLE for the IVF_FLAT / IVF_PQ search — test infrastructure only.

Only ``tests/`` (and ``bench.py``'s recall check) may use this module, and only
as the *checker*; the product path is the HIP library
(``duckdb-lancedb_amd/csrc/ivf_index.cpp`` + ``ivf_kernels.hip``).

What it restates (reference paths relative to ``/root/reference``):

* ``rust_lib/src/lance_manager.rs:411-418`` — ``vector_search(q).limit(k)
  .nprobes(n).refine_factor(r)`` on a table with an IVF_PQ index
  (``:483-515``): probe the ``n`` partitions nearest to the query, rank the
  rows of those partitions by their PQ (ADC) distance, re-rank the best
  ``k * r`` exactly and return the top ``k``; rows not covered by the index
  yet are searched exactly (LanceDB scans unindexed fragments flat) and merged.
* the published algorithms of the third-party ``lance-index 0.22.0`` (IVF
  partition search, residual product quantisation with 8-bit codes and an
  asymmetric-distance lookup table); the crate source is not in the container,
  so parity with LanceDB itself is UNPINNED for IVF (no reference test builds
  or searches an IVF index) and this oracle pins the HIP path to
  the build's own canonical numerics, given the same trained model:

  coarse    exact distances (f64 accumulate, f32 result) to the centroids —
            dot for a dot index, L2 otherwise (cosine: L2 between the
            normalised query and the centroids) — top-nprobe by (dist, id)
  IVF_FLAT  exact distance of every live row of the probed lists
  IVF_PQ    ADC = (d0 + tau) + sum_j LUT[j][code_j] in f32, j ascending, d0 =
            the coarse distance; L2/cosine: LUT = -2 P[q] and the row term
            tau = sum_j T[l][j][code_j] (f32, j ascending, from 0; the HIP
            path computes it once per row at index time); dot: LUT = -P[q],
            tau = 0.  P[j][c] = sum_t q_t y_t, T[l][j][c] = sum_t y_t (y_t +
            2 c_t), each an f32 sum in t order of f32 products (no fused
            multiply-add);
            top-(k*r) by (ADC, label ascending), exact re-rank, top-k by
            (dist, label under the tie rule: flat_knn.tie_desc)
  cosine    q^ = q / f32(sqrt(sum q^2)) (an f32 division) for the coarse
            search and P; the final distances are exact cosine distances.
  u8 LUT    the fast scan (``pq_scan`` = "fast", the default): per query
            L = sP P[q] (sP = -2, dot: -1), lo_j = min_c L[j][c], D = max_j
            (max_c L[j][c] - lo_j) / 255 (1 when 0), u[j][c] = min(255,
            rint((L[j][c] - lo_j) * f32(1 / D))), L0 = sum_j lo_j (j
            ascending); ADC = ((d0 + tau) + L0) + D * S with S = sum_j
            u[j][code_j] (an exact integer); every step one f32 rounding.
  fp8       ``pq_query`` = "fp8": P is built from q' = e4m3(q / s) * s, s =
            absmax(q) / 448 per query (OCP e4m3fn, round to nearest even, 3
            mantissa bits, subnormal step 2^-9); coarse search and re-rank
            keep the f32 query.

The model (centroids, codebook) and the layout (list and codes of every row)
come from the library (``lance_hip_ivf_export``): training is checked
separately (assignments near-nearest, recall).
"""
from __future__ import annotations

import numpy as np

from . import flat_knn

F32 = np.float32


def normalize_queries(Q):
    """q^ = q / f32(sqrt(f64 sum q^2)) per row (zero rows unchanged)."""
    Q = np.asarray(Q, F32)
    nrm = np.sqrt(np.einsum("ij,ij->i", Q.astype(np.float64), Q.astype(np.float64))).astype(F32)
    out = Q.copy()
    nz = nrm > 0
    out[nz] = (Q[nz] / nrm[nz, None]).astype(F32)
    return out


def coarse_probes(C, Q, metric, nprobe):
    """Top-``nprobe`` partitions per query: (ids [nq, nprobe], dists f32)."""
    metric = flat_knn.normalize_metric(metric)
    cm = "dot" if metric == "dot" else "l2"
    Qc = normalize_queries(Q) if metric == "cosine" else np.asarray(Q, F32)
    nl = C.shape[0]
    nprobe = min(nprobe, nl)
    ids = np.zeros((Qc.shape[0], nprobe), np.int64)
    ds = np.zeros((Qc.shape[0], nprobe), F32)
    lab = np.arange(nl, dtype=np.int64)
    for i, q in enumerate(Qc):
        d = flat_knn.exact_distances(C, q, cm)
        o = flat_knn._order(d, lab, "label_asc")[:nprobe]  # probes: lower partition id at a tie
        ids[i], ds[i] = o, d[o]
    return ids, ds


def _topk_exact(X, labels, slots, q, k, metric, tie=None):
    if slots.size == 0:
        return np.zeros(0, np.int64), np.zeros(0, F32)
    d = flat_knn.exact_distances(X[slots], q, metric)
    o = flat_knn._order(d, labels[slots], tie)[:k]
    return slots[o], d[o]


def ivf_flat_search(X, labels, live, lists, C, Q, k, nprobe, metric="l2", tie=None):
    """IVF_FLAT: exact top-k over the live rows of the probed lists plus the
    live rows not indexed yet (``lists == -1``).  X / labels / live / lists
    are per slot (ascending labels).  Returns (labels [nq,k] -1 padded,
    dists [nq,k] NaN padded, counts)."""
    X = np.asarray(X, F32)
    labels = np.asarray(labels, np.int64)
    live = np.asarray(live, bool)
    lists = np.asarray(lists, np.int64)
    probes, _ = coarse_probes(C, Q, metric, nprobe)
    nq = len(Q)
    out_l = np.full((nq, k), -1, np.int64)
    out_d = np.full((nq, k), np.nan, F32)
    cnt = np.zeros(nq, np.int32)
    tail = live & (lists < 0)
    for i, q in enumerate(np.asarray(Q, F32)):
        sel = live & np.isin(lists, probes[i])
        slots = np.nonzero(sel | tail)[0]
        s, d = _topk_exact(X, labels, slots, q, k, metric, tie)
        n = len(s)
        out_l[i, :n], out_d[i, :n], cnt[i] = labels[s], d, n
    return out_l, out_d, cnt


def e4m3_round(v):
    """OCP e4m3fn round-to-nearest-even of f32 values with |v| <= 448 (the
    HIP path's e4m3_round, ivf_kernels.hip)."""
    v = np.asarray(v, F32)
    a = np.abs(v)
    _, e = np.frexp(a)
    E = np.maximum(e - 1, -6)
    ulp = np.ldexp(np.ones_like(a), E - 3).astype(F32)
    r = np.minimum((np.rint((a / ulp).astype(F32)) * ulp).astype(F32), F32(448.0))
    r = np.where(a > 0, r, F32(0.0)).astype(F32)
    return np.copysign(r, v).astype(F32)


def fp8_queries(Qp):
    """q' = e4m3(q / s) * s per row, s = f32(absmax / 448); zero rows stay 0."""
    Qp = np.asarray(Qp, F32)
    out = np.zeros_like(Qp)
    for i, x in enumerate(Qp):
        mx = F32(np.max(np.abs(x))) if x.size else F32(0.0)
        sc = F32(mx / F32(448.0))
        if sc > 0:
            out[i] = (e4m3_round((x / sc).astype(F32)) * sc).astype(F32)
    return out


def pq_lut_u8(P_i, sP):
    """8-bit LUT of one query: (u [m, 256] uint8, D, L0) per the module docstring."""
    L = (F32(sP) * np.asarray(P_i, F32)).astype(F32)
    lo = L.min(axis=1).astype(F32)
    sp = (L.max(axis=1) - lo).astype(F32)
    mxs = max(F32(0.0), F32(sp.max()))
    D = F32(mxs / F32(255.0)) if mxs > 0 else F32(1.0)
    inv = F32(F32(1.0) / D)
    u = np.minimum(np.rint(((L - lo[:, None]).astype(F32) * inv).astype(F32)), F32(255.0)).astype(np.uint8)
    L0 = F32(0.0)
    for v in lo:
        L0 = F32(L0 + v)
    return u, D, L0


def pq_tables(C, codebook, Qp, metric):
    """P [nq, m, 256] and T [nlist, m, 256] (None for dot) per the canonical
    f32 sequential definitions."""
    cb = np.asarray(codebook, F32)
    m, K, dsub = cb.shape
    Qp = np.asarray(Qp, F32).reshape(len(Qp), m, dsub)
    P = np.zeros((len(Qp), m, K), F32)
    for t in range(dsub):
        P = (P + (Qp[:, :, t][:, :, None] * cb[None, :, :, t]).astype(F32)).astype(F32)
    T = None
    if flat_knn.normalize_metric(metric) != "dot":
        Cr = np.asarray(C, F32).reshape(len(C), m, dsub)
        T = np.zeros((len(C), m, K), F32)
        for t in range(dsub):
            y = cb[None, :, :, t]
            twoc = (F32(2.0) * Cr[:, :, t])[:, :, None]
            T = (T + (y * (y + twoc).astype(F32)).astype(F32)).astype(F32)
    return P, T


def ivf_pq_search(X, labels, live, lists, codes, C, codebook, Q, k, nprobe, refine_factor=1, metric="l2",
                  lut="f32", query_fp8=False, tie=None):
    """IVF_PQ search (see the module docstring).  ``codes`` [slots, m] uint8.
    lut: "f32" (the query-major scan, pq_scan = exact_lut) or "u8" (the fast
    scan); query_fp8: ADC tables from fp8 queries (pq_query = fp8)."""
    metric = flat_knn.normalize_metric(metric)
    X = np.asarray(X, F32)
    labels = np.asarray(labels, np.int64)
    live = np.asarray(live, bool)
    lists = np.asarray(lists, np.int64)
    codes = np.asarray(codes, np.uint8)
    Q = np.asarray(Q, F32)
    probes, pd = coarse_probes(C, Q, metric, nprobe)
    Qp = normalize_queries(Q) if metric == "cosine" else Q
    if query_fp8:
        Qp = fp8_queries(Qp)
    P, T = pq_tables(C, codebook, Qp, metric)
    m = codes.shape[1]
    kp = k * max(1, refine_factor)
    nq = len(Q)
    out_l = np.full((nq, k), -1, np.int64)
    out_d = np.full((nq, k), np.nan, F32)
    cnt = np.zeros(nq, np.int32)
    tail = np.nonzero(live & (lists < 0))[0]
    luts = [pq_lut_u8(P[i], -2.0 if T is not None else -1.0) for i in range(nq)] if lut == "u8" else None
    for i in range(nq):
        cand_adc, cand_slot = [], []
        for p, l in enumerate(probes[i]):
            rows = np.nonzero(live & (lists == l))[0]
            if rows.size == 0:
                continue
            acc = np.full(rows.size, pd[i, p], F32)
            if T is not None:
                tau = np.zeros(rows.size, F32)
                for j in range(m):
                    tau = (tau + T[l][j, codes[rows, j]]).astype(F32)
                acc = (acc + tau).astype(F32)
            if lut == "u8":
                u, D, L0 = luts[i]
                S = np.zeros(rows.size, np.int64)
                for j in range(m):
                    S += u[j, codes[rows, j]]
                acc = (acc + L0).astype(F32)
                acc = (acc + (D * S.astype(F32)).astype(F32)).astype(F32)
            else:
                lt = (F32(-2.0) * P[i]).astype(F32) if T is not None else (-P[i]).astype(F32)
                for j in range(m):
                    acc = (acc + lt[j, codes[rows, j]]).astype(F32)
            cand_adc.append(acc)
            cand_slot.append(rows)
        sel = np.zeros(0, np.int64)
        if cand_adc:
            a = np.concatenate(cand_adc)
            s = np.concatenate(cand_slot)
            o = flat_knn._order(a, labels[s], "label_asc")[:kp]  # ADC candidates: (ADC, label ascending)
            sel = s[o]
        ts, _ = _topk_exact(X, labels, tail, Q[i], k, metric, tie)
        allc = np.concatenate([sel, ts])
        s, d = _topk_exact(X, labels, allc, Q[i], k, metric, tie)
        n = len(s)
        out_l[i, :n], out_d[i, :n], cnt[i] = labels[s], d, n
    return out_l, out_d, cnt
