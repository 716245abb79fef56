"""CPU checks of the IVF oracle (oracle/ivf.py) — the checker the GPU IVF
tests compare against: with every list probed IVF_FLAT is the exact flat
search, and IVF_PQ with a re-rank window covering every row is too; the ADC
tables follow their f32 definitions."""
import numpy as np
import pytest

from oracle import flat_knn, ivf


def _model(rng, n, d, nlist, m):
    X = rng.standard_normal((n, d)).astype(np.float32)
    C = X[rng.choice(n, nlist, replace=False)].copy()
    lists = np.argmin(((X[:, None, :] - C[None]) ** 2).sum(-1), 1)
    cb = rng.standard_normal((m, 256, d // m)).astype(np.float32) * 0.3
    R = X - C[lists]
    codes = np.stack([np.argmin(((R[:, j * (d // m):(j + 1) * (d // m)][:, None, :] - cb[j][None]) ** 2).sum(-1), 1)
                      for j in range(m)], 1).astype(np.uint8)
    return X, C, lists, cb, codes


def test_flat_all_probes_equals_flat_search():
    rng = np.random.default_rng(0)
    X, C, lists, _, _ = _model(rng, 600, 16, 12, 4)
    Q = rng.standard_normal((9, 16)).astype(np.float32)
    n = len(X)
    live = np.ones(n, bool)
    live[::5] = False
    lab = np.arange(n)
    for metric in ("l2", "dot", "cosine"):
        gl, gd, gc = ivf.ivf_flat_search(X, lab, live, lists, C, Q, 7, 12, metric)
        el, ed, ec = flat_knn.flat_search_batch(X, lab, live, Q, 7, metric)
        np.testing.assert_array_equal(gl, el)
        np.testing.assert_array_equal(gc, ec)


def test_pq_full_window_is_exact_and_tail_merges():
    rng = np.random.default_rng(1)
    X, C, lists, cb, codes = _model(rng, 500, 16, 8, 4)
    Q = rng.standard_normal((6, 16)).astype(np.float32)
    lab = np.arange(len(X))
    live = np.ones(len(X), bool)
    lists = lists.copy()
    lists[450:] = -1  # the unindexed tail
    gl, gd, gc = ivf.ivf_pq_search(X, lab, live, lists, codes, C, cb, Q, 5, 8, refine_factor=100)
    el, ed, ec = flat_knn.flat_search_batch(X, lab, live, Q, 5)
    np.testing.assert_array_equal(gl, el)
    np.testing.assert_array_equal(gd, ed)


def test_pq_tables_definition():
    rng = np.random.default_rng(2)
    _, C, _, cb, _ = _model(rng, 100, 8, 3, 2)
    q = rng.standard_normal((1, 8)).astype(np.float32)
    P, T = ivf.pq_tables(C, cb, q, "l2")
    j, c, l = 1, 17, 2
    acc = np.float32(0)
    for t in range(4):
        acc = np.float32(acc + np.float32(q[0, j * 4 + t] * cb[j, c, t]))
    assert P[0, j, c] == acc
    acc = np.float32(0)
    for t in range(4):
        y = cb[j, c, t]
        acc = np.float32(acc + np.float32(y * np.float32(y + np.float32(2) * C[l, j * 4 + t])))
    assert T[l, j, c] == acc
    # L2 ADC approximates |q - c - y|^2 (T - 2P adds |q - c|^2 back through d0)
    y = cb[:, 0, :].reshape(-1)
    exact = ((q[0] - C[l] - y) ** 2).sum()
    d0 = ((q[0] - C[l]) ** 2).sum()
    adc = d0 + sum((T[l, jj, 0] - 2 * P[0, jj, 0]) for jj in range(2))
    assert abs(adc - exact) < 1e-3 * max(1.0, exact)


def test_c_ivf_port_matches_numpy_oracle():
    """oracle/flat_knn.c's IVF port (the IVF benches' cpu_baseline) restates
    oracle/ivf.py exactly in its f64 mode: same labels, same distances."""
    from oracle import c_oracle

    rng = np.random.default_rng(3)
    n, d, nlist, m = 900, 32, 10, 8
    X, C, lists, cb, codes = _model(rng, n, d, nlist, m)
    Q = rng.standard_normal((7, d)).astype(np.float32)
    lab = np.arange(n, dtype=np.int64) * 3 + 5  # ascending, not dense
    live = np.ones(n, bool)
    live[::7] = False
    lists = lists.copy()
    lists[850:] = -1  # unindexed tail
    lay = c_oracle.IvfLayout(lists, live, nlist)
    for metric in ("l2", "dot"):
        for nprobe, k in [(3, 5), (10, 12), (1, 4)]:
            el, ed, ec = ivf.ivf_flat_search(X, lab, live, lists, C, Q, k, nprobe, metric)
            gl, gd, gc = c_oracle.ivf_search_batch(X, lab, lay, C, Q, k, nprobe, metric)
            np.testing.assert_array_equal(gc, ec)
            np.testing.assert_array_equal(gl, el)
            np.testing.assert_array_equal(gd, ed)
            for rf in (1, 3):
                for lut, fp8 in (("f32", False), ("u8", False), ("u8", True), ("f32", True)):
                    el, ed, ec = ivf.ivf_pq_search(X, lab, live, lists, codes, C, cb, Q, k, nprobe, rf, metric,
                                                   lut=lut, query_fp8=fp8)
                    _, T = ivf.pq_tables(C, cb, Q[:1], metric)
                    gl, gd, gc = c_oracle.ivf_search_batch(X, lab, lay, C, Q, k, nprobe, metric, codes=codes,
                                                           codebook=cb, T=T, refine_factor=rf, lut=lut,
                                                           query_fp8=fp8)
                    np.testing.assert_array_equal(gc, ec)
                    np.testing.assert_array_equal(gl, el)
                    np.testing.assert_array_equal(gd, ed)


def test_e4m3_round_matches_torch_float8():
    """The fp8 query restatement (OCP e4m3fn, round to nearest even) equals
    torch's float8_e4m3fn cast on 1M values spanning subnormals to 448."""
    import torch

    rng = np.random.default_rng(0)
    v = (rng.standard_normal(1_000_000) * np.exp(rng.uniform(-12, 6, 1_000_000))).astype(np.float32)
    v = np.clip(v, -448, 448)
    want = torch.from_numpy(v).to(torch.float8_e4m3fn).float().numpy()
    np.testing.assert_array_equal(ivf.e4m3_round(v), want)


def test_u8_lut_bounds_the_f32_lut():
    """Each 8-bit entry reconstructs its f32 LUT entry within D / 2 (+ f32
    rounding), so the quantised ADC is within m * D / 2 of the f32 ADC."""
    rng = np.random.default_rng(4)
    P = rng.standard_normal((16, 256)).astype(np.float32) * 3
    u, D, L0 = ivf.pq_lut_u8(P, -2.0)
    L = (np.float32(-2.0) * P).astype(np.float32)
    lo = L.min(axis=1)
    rec = lo[:, None] + D * u.astype(np.float32)
    assert np.all(np.abs(rec - L) <= D * 0.5 * (1 + 1e-5) + 1e-5)
    assert u.max() <= 255 and abs(L0 - lo.astype(np.float64).sum()) < 1e-3


@pytest.mark.parametrize("tie", ["label_desc", "label_asc"])
def test_c_ivf_port_matches_numpy_oracle_with_ties(tie):
    """Duplicate rows (exact-distance ties at the k-th place, in the probed lists
    and in the unindexed tail): the C port and oracle/ivf.py pick the same tied
    rows under either tie rule (final order: distance, then label by the rule;
    probes and ADC candidates: lower id first)."""
    from oracle import c_oracle

    rng = np.random.default_rng(33)
    n, d, nlist, m = 900, 32, 10, 8
    X, C, lists, cb, codes = _model(rng, n, d, nlist, m)
    X = X.copy()
    for src in (3, 100, 500):
        X[rng.choice(n, 12, replace=False)] = X[src]
    Q = np.stack([X[3], X[100], X[500], X[3] + 0.01]).astype(np.float32)
    lab = np.arange(n, dtype=np.int64)
    live = np.ones(n, bool)
    lists = lists.copy()
    lists[850:] = -1
    lay = c_oracle.IvfLayout(lists, live, nlist)
    for nprobe, k in [(nlist, 8), (3, 6)]:
        el, ed, ec = ivf.ivf_flat_search(X, lab, live, lists, C, Q, k, nprobe, "l2", tie=tie)
        gl, gd, gc = c_oracle.ivf_search_batch(X, lab, lay, C, Q, k, nprobe, "l2", tie=tie)
        np.testing.assert_array_equal(gl, el)
        np.testing.assert_array_equal(gd, ed)
        _, T = ivf.pq_tables(C, cb, Q[:1], "l2")
        el, ed, ec = ivf.ivf_pq_search(X, lab, live, lists, codes, C, cb, Q, k, nprobe, 50, "l2", lut="u8", tie=tie)
        gl, gd, gc = c_oracle.ivf_search_batch(X, lab, lay, C, Q, k, nprobe, "l2", codes=codes, codebook=cb, T=T,
                                               refine_factor=50, lut="u8", tie=tie)
        np.testing.assert_array_equal(gl, el)
    # with every list probed the flat IVF result is the exact flat result under the same rule
    fl, fd, fc = flat_knn.flat_search_batch(X, lab, live, Q, 8, "l2", tie=tie)
    el, ed, ec = ivf.ivf_flat_search(X, lab, live, lists, C, Q, 8, nlist, "l2", tie=tie)
    np.testing.assert_array_equal(el, fl)
