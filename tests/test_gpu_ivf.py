"""GPU parity of the IVF_FLAT / IVF_PQ path (lance_detached_create_index +
nprobes / refine_factor search, rust_lib/src/lance_manager.rs:483-515 and
:411-418) against oracle/ivf.py, given the model and row layout the library
exports.  Bar: labels bit-exact, distances within 1e-4 relative (observed:
identical).  Parity with LanceDB itself is unpinned for IVF (no reference test
builds an IVF index)."""
import numpy as np
import pytest

from oracle import flat_knn, ivf

pytestmark = pytest.mark.gpu

RTOL = 1e-4
ATOL = 1e-5


def assert_same(gl, gd, gc, el, ed, ec):
    np.testing.assert_array_equal(gc, ec)
    for i in range(el.shape[0]):
        n = int(gc[i])
        np.testing.assert_array_equal(gl[i, :n], el[i, :n], err_msg=f"query {i}")
        np.testing.assert_allclose(gd[i, :n], ed[i, :n], rtol=RTOL, atol=ATOL, err_msg=f"query {i}")


@pytest.fixture
def mk(hip):
    made = []

    def make(dim, metric="l2", index_type="ivf_pq", path=""):
        h = hip.LanceCreateDetached(path, dim, metric, "ivf")
        hip.LanceHipSetOption(h, "index_type", index_type)
        made.append(h)
        return h

    yield make
    for h in made:
        hip.LanceFreeDetached(h)


def clustered(rng, n, d, centers=48, spread=0.35):
    C = rng.standard_normal((centers, d)).astype(np.float32)
    lab = rng.integers(0, centers, n)
    return (C[lab] + spread * rng.standard_normal((n, d))).astype(np.float32)


def oracle_search(hip, h, X_by_label, Q, k, nprobe, rf, metric, lut="u8", query_fp8=False, tie=None):
    """lut: "u8" for the default fast scan (pq_scan = fast), "f32" for
    pq_scan = exact_lut; query_fp8 mirrors pq_query = fp8; tie: the handle's
    tie rule (None: the default, label_desc)."""
    ex = hip.LanceHipIvfExport(h)
    X = X_by_label[ex["labels"]]
    if ex["type"] == "ivf_flat":
        return ivf.ivf_flat_search(X, ex["labels"], ex["live"], ex["lists"], ex["centroids"], Q, k, nprobe, metric,
                                   tie=tie)
    return ivf.ivf_pq_search(X, ex["labels"], ex["live"], ex["lists"], ex["codes"], ex["centroids"], ex["codebook"],
                             Q, k, nprobe, rf, metric, lut=lut, query_fp8=query_fp8, tie=tie)


@pytest.mark.parametrize("index_type", ["ivf_flat", "ivf_pq"])
@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
def test_ivf_parity(hip, mk, index_type, metric):
    rng = np.random.default_rng(11)
    n, d, nlist, m = 12_000, 64, 48, 8
    X = clustered(rng, n, d)
    Q = (X[rng.choice(n, 70, replace=False)] + 0.2 * rng.standard_normal((70, d))).astype(np.float32)
    h = mk(d, metric, index_type)
    hip.LanceDetachedAddBatch(h, X[:10_000], 10_000, d)
    hip.LanceDetachedDeleteBatch(h, rng.choice(10_000, 300, replace=False))
    hip.LanceDetachedCreateIndex(h, nlist, m)
    info = hip.LanceHipIvfInfo(h)
    assert info["type"] == index_type and info["nlist"] == nlist and info["n_indexed"] == 10_000
    # rows added after the build are searched exactly (the unindexed tail)
    hip.LanceDetachedAddBatch(h, X[10_000:], n - 10_000, d)
    hip.LanceDetachedDeleteBatch(h, rng.choice(n, 200, replace=False))
    modes = [("fast", "f32")]
    if index_type == "ivf_pq":  # both PQ scans, f32 and fp8 (e4m3) ADC queries
        modes = [("fast", "f32"), ("fast", "fp8"), ("exact_lut", "f32"), ("exact_lut", "fp8")]
    for scan, qm in modes:
        if index_type == "ivf_pq":
            hip.LanceHipSetOption(h, "pq_scan", scan)
            hip.LanceHipSetOption(h, "pq_query", qm)
        for nprobe, rf, k in [(6, 2, 10), (1, 1, 5), (20, 3, 40)]:
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, k, nprobes=nprobe, refine_factor=rf)
            el, ed, ec = oracle_search(hip, h, X, Q, k, nprobe, rf, metric, "u8" if scan == "fast" else "f32",
                                       qm == "fp8")
            assert_same(gl, gd, gc, el, ed, ec)


@pytest.mark.parametrize("metric", ["l2", "dot"])
def test_ivf_flat_all_probes_is_exact(hip, mk, metric):
    # nprobe = nlist probes every list: IVF_FLAT must equal the exact flat search
    rng = np.random.default_rng(5)
    n, d, nlist = 9_000, 48, 30
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((40, d)).astype(np.float32)
    h = mk(d, metric, "ivf_flat")
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedCreateIndex(h, nlist, 0)
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10, nprobes=nlist)
    el, ed, ec = flat_knn.flat_search_batch(X, np.arange(n), np.ones(n, bool), Q, 10, metric)
    assert_same(gl, gd, gc, el, ed, ec)


def test_ivf_pq_recall_and_defaults(hip, mk):
    rng = np.random.default_rng(3)
    n, d = 30_000, 96
    X = clustered(rng, n, d, centers=64)
    Q = (X[rng.choice(n, 100, replace=False)] + 0.1 * rng.standard_normal((100, d))).astype(np.float32)
    h = mk(d)
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedCreateIndex(h, 0, 0)  # LanceDB defaults: sqrt(n) partitions, dim/16 sub-vectors
    info = hip.LanceHipIvfInfo(h)
    assert info["nlist"] == int(np.sqrt(n)) and info["m"] == d // 16 and info["dsub"] == 16
    el, _, _ = flat_knn.flat_search_batch(X, np.arange(n), np.ones(n, bool), Q, 10)
    # PQ with 16-dim sub-vectors ranks coarsely (sklearn-trained IVF_PQ on this
    # data: recall 0.79 at refine 10, 1.0 at refine 100): a wider re-rank
    # window must recover the exact neighbours
    gl, _, _ = hip.LanceDetachedSearchBatch(h, Q, 10, nprobes=40, refine_factor=10)
    assert flat_knn.recall_at_k(gl, el, 10) >= 0.7
    gl, _, _ = hip.LanceDetachedSearchBatch(h, Q, 10, nprobes=40, refine_factor=80)
    assert flat_knn.recall_at_k(gl, el, 10) >= 0.97
    # rows are placed by exact-f32 scores: every row sits in its nearest
    # partition up to f32 rounding
    ex = hip.LanceHipIvfExport(h)
    C = ex["centroids"]
    d2 = ((X[:2000, None, :].astype(np.float64) - C[None, :, :]) ** 2).sum(-1)
    best = d2.min(1)
    got = d2[np.arange(2000), ex["lists"][:2000]]
    assert np.all(got <= best * (1 + 1e-4) + 1e-3)


def test_compact_optimizes_tail_and_keeps_parity(hip, mk):
    rng = np.random.default_rng(8)
    n, d = 8_000, 32
    X = clustered(rng, n, d, centers=20)
    Q = rng.standard_normal((30, d)).astype(np.float32)
    h = mk(d, "l2", "ivf_pq")
    hip.LanceDetachedAddBatch(h, X[:6000], 6000, d)
    hip.LanceDetachedCreateIndex(h, 16, 4)
    hip.LanceDetachedAddBatch(h, X[6000:], 2000, d)
    hip.LanceDetachedDeleteBatch(h, np.arange(0, 8000, 7))
    hip.LanceDetachedCompact(h)
    info = hip.LanceHipIvfInfo(h)
    assert info["n_indexed"] == info["n_slots"] == hip.LanceDetachedCount(h)
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10, nprobes=4, refine_factor=2)
    el, ed, ec = oracle_search(hip, h, X, Q, 10, 4, 2, "l2")
    assert_same(gl, gd, gc, el, ed, ec)
    assert not np.isin(gl, np.arange(0, 8000, 7)).any()


def test_set_model_reproduces_results(hip, mk):
    # multi-GPU path: rank 0 trains, other ranks install the same model
    rng = np.random.default_rng(21)
    n, d = 5_000, 64
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((25, d)).astype(np.float32)
    a = mk(d, "l2", "ivf_pq")
    hip.LanceDetachedAddBatch(a, X, n, d)
    hip.LanceDetachedCreateIndex(a, 20, 16)
    ex = hip.LanceHipIvfExport(a)
    b = mk(d, "l2")
    hip.LanceDetachedAddBatch(b, X, n, d)
    hip.LanceHipIvfSetModel(b, "ivf_pq", ex["centroids"], ex["codebook"])
    exb = hip.LanceHipIvfExport(b)
    np.testing.assert_array_equal(ex["lists"], exb["lists"])
    np.testing.assert_array_equal(ex["codes"], exb["codes"])
    ra = hip.LanceDetachedSearchBatch(a, Q, 10, nprobes=5, refine_factor=3)
    rb = hip.LanceDetachedSearchBatch(b, Q, 10, nprobes=5, refine_factor=3)
    for x, y in zip(ra, rb):
        np.testing.assert_array_equal(x, y)


def test_index_persists_across_reopen(hip, mk, tmp_path):
    rng = np.random.default_rng(4)
    n, d = 4_000, 32
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((10, d)).astype(np.float32)
    h = hip.LanceCreateDetached(str(tmp_path), d, "l2", "t")
    hip.LanceDetachedAddBatch(h, X[:3000], 3000, d)
    hip.LanceDetachedCreateIndex(h, 12, 8)
    hip.LanceDetachedAddBatch(h, X[3000:], 1000, d)
    r0 = hip.LanceDetachedSearchBatch(h, Q, 7, nprobes=3, refine_factor=2)
    i0 = hip.LanceHipIvfInfo(h)
    hip.LanceFreeDetached(h)
    h2 = hip.LanceOpenDetached(str(tmp_path), "t", "l2")
    try:
        assert hip.LanceHipIvfInfo(h2) == i0
        r1 = hip.LanceDetachedSearchBatch(h2, Q, 7, nprobes=3, refine_factor=2)
        for x, y in zip(r0, r1):
            np.testing.assert_array_equal(x, y)
    finally:
        hip.LanceFreeDetached(h2)


def test_ivf_errors(hip, mk):
    h = mk(24)
    with pytest.raises(hip.IOException, match="empty table"):
        hip.LanceDetachedCreateIndex(h, 4, 4)
    X = np.random.default_rng(0).standard_normal((300, 24)).astype(np.float32)
    hip.LanceDetachedAddBatch(h, X, 300, 24)
    with pytest.raises(hip.IOException, match="centroids"):
        hip.LanceDetachedCreateIndex(h, 400, 4)
    with pytest.raises(hip.IOException, match="divide"):
        hip.LanceDetachedCreateIndex(h, 4, 5)
    assert hip.LanceHipIvfInfo(h)["type"] is None
    # a failed build leaves the flat path serving exact results
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, X[:3], 5)
    assert list(gl[:, 0]) == [0, 1, 2]


@pytest.mark.parametrize("storage", ["f32", "bf16"])
@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
def test_ivf_flat_bound_scan_matches_exact_scan(hip, mk, storage, metric):
    """The MFMA bound scan (ivf_flat_scan = bound, the default with bf16 scan
    rows) returns the exact list scan's results: same labels and distances as
    the oracle, for f32 rows (bf16 scan copy) and a bf16 store."""
    rng = np.random.default_rng(21)
    n, d, nlist = 20_000, 128, 40
    X = clustered(rng, n, d, centers=60)
    if storage == "bf16":
        import torch

        X = torch.from_numpy(X).to(torch.bfloat16).float().numpy()
    Q = (X[rng.choice(n, 90, replace=False)] + 0.3 * rng.standard_normal((90, d))).astype(np.float32)
    h = mk(d, metric, "ivf_flat")
    hip.LanceHipSetOption(h, "storage", storage)
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedDeleteBatch(h, rng.choice(n, 500, replace=False))
    hip.LanceDetachedCreateIndex(h, nlist, 0)
    for nprobe, k in [(8, 10), (3, 1), (40, 15)]:
        hip.LanceHipSetOption(h, "ivf_flat_scan", "bound")
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, k, nprobes=nprobe)
        el, ed, ec = oracle_search(hip, h, X, Q, k, nprobe, 1, metric)
        assert_same(gl, gd, gc, el, ed, ec)
        hip.LanceHipSetOption(h, "ivf_flat_scan", "exact")
        xl, xd, xc = hip.LanceDetachedSearchBatch(h, Q, k, nprobes=nprobe)
        assert_same(xl, xd, xc, el, ed, ec)


@pytest.mark.parametrize("tie", ["label_desc", "label_asc"])
@pytest.mark.parametrize("index_type,scan", [("ivf_flat", "bound"), ("ivf_flat", "exact"), ("ivf_pq", "fast")])
def test_ivf_tie_rule(hip, mk, index_type, scan, tie):
    """Exact-distance ties at the k-th place through the IVF paths (IVF_FLAT
    bound scan + certified re-rank / its exact list scan, IVF_PQ's exact
    re-rank) and the exact scan of the unindexed tail, under both tie rules:
    the rule picks which tied rows come out, as the oracle's does."""
    rng = np.random.default_rng(66)
    n, d, nlist = 6_000, 64, 12
    X = clustered(rng, n, d, centers=12)
    for j, src in enumerate((100, 2000, 4000)):
        X[rng.choice(n, 6 + 4 * j, replace=False)] = X[src]
    Q = np.stack([X[100], X[2000], X[4000], X[100] + 0.01, X[7]]).astype(np.float32)
    h = mk(d, "l2", index_type)
    hip.LanceHipSetOption(h, "tie", tie)
    hip.LanceHipSetOption(h, "ivf_flat_scan", scan) if index_type == "ivf_flat" else None
    hip.LanceDetachedAddBatch(h, X[:5000], 5000, d)
    hip.LanceDetachedCreateIndex(h, nlist, 8 if index_type == "ivf_pq" else 0)
    hip.LanceDetachedAddBatch(h, X[5000:], n - 5000, d)  # the unindexed tail holds some copies too
    rf = 20 if index_type == "ivf_pq" else 1
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 8, nprobes=4, refine_factor=rf)
    el, ed, ec = oracle_search(hip, h, X, Q, 8, 4, rf, "l2", tie=tie)
    assert_same(gl, gd, gc, el, ed, ec)


def test_ivf_flat_bound_scan_ties_fall_back_exactly(hip, mk):
    """Hundreds of identical rows in one list tie every bound at the k-th
    distance: the certificate fails and the pass reruns on the exact scan,
    which orders the ties by label."""
    rng = np.random.default_rng(8)
    n, d, nlist = 6_000, 64, 12
    X = clustered(rng, n, d, centers=12)
    X[100:900] = X[100]  # 800 copies
    Q = np.stack([X[100] + 0.01, X[5], X[2000]]).astype(np.float32)
    h = mk(d, "l2", "ivf_flat")
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedCreateIndex(h, nlist, 0)
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10, nprobes=4)
    el, ed, ec = oracle_search(hip, h, X, Q, 10, 4, 1, "l2")
    assert_same(gl, gd, gc, el, ed, ec)


def test_ivf_flat_bound_scan_zero_cosine_rows_and_query(hip, mk):
    """Cosine with zero rows and a zero query: the rows' / query's bounds are
    NaN (cosine undefined).  The bound scan must not certify a result that left
    such a live row out; it reruns on the exact scan and returns what the exact
    scan returns (NaN-distance rows after every other row)."""
    rng = np.random.default_rng(17)
    n, d, nlist = 8_000, 128, 16
    X = clustered(rng, n, d, centers=16)
    X[10:14] = 0.0  # zero rows
    Q = np.concatenate([X[rng.choice(n, 6, replace=False)] + 0.2, np.zeros((1, d), np.float32)]).astype(np.float32)
    h = mk(d, "cosine", "ivf_flat")
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedCreateIndex(h, nlist, 0)
    for nprobe, k in [(16, 10), (4, 15), (1, 15)]:  # k <= 15: the bound scan applies
        hip.LanceHipSetOption(h, "ivf_flat_scan", "bound")
        bl, bd, bc = hip.LanceDetachedSearchBatch(h, Q, k, nprobes=nprobe)
        hip.LanceHipSetOption(h, "ivf_flat_scan", "exact")
        xl, xd, xc = hip.LanceDetachedSearchBatch(h, Q, k, nprobes=nprobe)
        assert bc[-1] == min(k, n)  # the zero query: every probed row, NaN distances, label order
        np.testing.assert_array_equal(bc, xc)
        np.testing.assert_array_equal(bl, xl)
        np.testing.assert_allclose(bd, xd, rtol=1e-6, equal_nan=True)


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
def test_fused_coarse_search_equals_flat(hip, mk, metric):
    """The fused coarse search (coarse_kernels.hip: f32 MFMA bounds, per-query
    select + exact refine) returns exactly the probes of the flat path over the
    centroid store (ivf_coarse = flat), so every search result is identical; a
    NaN query sends its batch to the flat path (the fallback counter moves)."""
    rng = np.random.default_rng(91)
    n, d, nlist = 20_000, 96, 300
    X = clustered(rng, n, d, centers=64)
    Q = (X[rng.choice(n, 120, replace=False)] + 0.3 * rng.standard_normal((120, d))).astype(np.float32)
    h = mk(d, metric, "ivf_flat")
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedCreateIndex(h, nlist, 0)
    for nprobe in (1, 37, 300):
        hip.LanceHipSetOption(h, "ivf_coarse", "fused")
        a = hip.LanceDetachedSearchBatch(h, Q, 10, nprobes=nprobe)
        hip.LanceHipSetOption(h, "ivf_coarse", "flat")
        b = hip.LanceDetachedSearchBatch(h, Q, 10, nprobes=nprobe)
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
        el, ed, ec = oracle_search(hip, h, X, Q, 10, nprobe, 1, metric)
        assert_same(*a, el, ed, ec)
    hip.LanceHipSetOption(h, "ivf_coarse", "fused")
    Qn = Q.copy()
    Qn[3] = np.nan
    a = hip.LanceDetachedSearchBatch(h, Qn, 10, nprobes=16)
    hip.LanceHipSetOption(h, "ivf_coarse", "flat")
    b = hip.LanceDetachedSearchBatch(h, Qn, 10, nprobes=16)
    np.testing.assert_array_equal(a[0], b[0])


@pytest.mark.parametrize("itype", ["ivf_pq", "ivf_flat"])
def test_fused_coarse_flag_reruns_the_pass(hip, mk, itype):
    """The fused coarse search's flags are read only after the whole pass has
    run (round 6: no host wait between the coarse search and the list scans).
    A flagged query (NaN) leaves no probes, so the pass runs harmlessly and is
    then rerun on the flat coarse path: every query's result equals the flat
    path's, the good queries' and the NaN query's alike, batch after batch."""
    rng = np.random.default_rng(93)
    n, d, nlist = 12_000, 64, 128
    X = clustered(rng, n, d, centers=32)
    Q = (X[rng.choice(n, 40, replace=False)] + 0.3 * rng.standard_normal((40, d))).astype(np.float32)
    h = mk(d, "l2", itype)
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedCreateIndex(h, nlist, 16 if itype == "ivf_pq" else 0)
    for bad in (None, 5, None, 0):
        Qb = Q.copy()
        if bad is not None:
            Qb[bad] = np.nan
        for nprobe in (8, 128):
            hip.LanceHipSetOption(h, "ivf_coarse", "fused")
            a = hip.LanceDetachedSearchBatch(h, Qb, 10, nprobes=nprobe, refine_factor=2)
            hip.LanceHipSetOption(h, "ivf_coarse", "flat")
            b = hip.LanceDetachedSearchBatch(h, Qb, 10, nprobes=nprobe, refine_factor=2)
            np.testing.assert_array_equal(a[2], b[2])
            np.testing.assert_array_equal(a[0], b[0])
            np.testing.assert_allclose(a[1], b[1], rtol=0, atol=0, equal_nan=True)


@pytest.mark.parametrize("seed", ["1", "0"])
def test_pq_run_merge_bound_paths_equal(hip, mk, seed):
    """The run merge with the scan's final bound (pq_merge_bound = 1, the
    default: direct sort of up to 2048 keys at or below the bound, a radix
    select of the K-th distance word past that, the streaming top-K past 8192)
    returns the same lists as the streaming merge over the whole run
    (pq_merge_bound = 0), and the oracle's.  Without the seed (pq_seed = 0) a
    query whose items never cut its buffer keeps an unbounded thrq, so every
    probed row reaches the merge: nprobe 4 / 16 / 40 / 128 over ~310-row lists
    span the three regimes."""
    rng = np.random.default_rng(95)
    n, d, nlist = 40_000, 64, 128
    X = clustered(rng, n, d, centers=32)
    Q = (X[rng.choice(n, 48, replace=False)] + 0.3 * rng.standard_normal((48, d))).astype(np.float32)
    h = mk(d, "l2", "ivf_pq")
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedCreateIndex(h, nlist, 16)
    hip.LanceHipSetOption(h, "pq_seed", seed)
    for nprobe, rf in [(4, 2), (16, 10), (40, 10), (128, 51)]:
        res = {}
        for mb in ("1", "0"):
            hip.LanceHipSetOption(h, "pq_merge_bound", mb)
            res[mb] = hip.LanceDetachedSearchBatch(h, Q, 10, nprobes=nprobe, refine_factor=rf)
        for x, y in zip(res["1"], res["0"]):
            np.testing.assert_array_equal(x, y, err_msg=f"nprobe {nprobe}")
        el, ed, ec = oracle_search(hip, h, X, Q, 10, nprobe, rf, "l2")
        assert_same(*res["1"], el, ed, ec)
    hip.LanceHipSetOption(h, "pq_merge_bound", "1")


@pytest.mark.parametrize("itype", ["ivf_pq", "ivf_flat"])
def test_ivf_async_two_in_flight(hip, mk, itype):
    """lance_hip_search_batch_device_async on an IVF handle (round 6): the whole
    search is enqueued on the handle's stream, two searches in flight sharing
    the IVF workspace in stream order, the fused coarse flags read at the wait.
    Batches: plain, one with a NaN query (its flag reruns that search on the
    flat coarse path while the next search is already queued behind it), a
    different batch size (drains first: the workspace may grow), and a
    different nprobes.  Every batch equals the synchronous search."""
    import torch
    from lance_hip.sharded import AsyncPipeline, hip_device_search

    rng = np.random.default_rng(97)
    n, d, nlist, k = 20_000, 64, 96, 10
    X = clustered(rng, n, d, centers=32)
    h = mk(d, "l2", itype)
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedCreateIndex(h, nlist, 16 if itype == "ivf_pq" else 0)
    L = hip.lib()

    def batch(nq, nan_at=None):
        Q = (X[rng.choice(n, nq, replace=False)] + 0.3 * rng.standard_normal((nq, d))).astype(np.float32)
        if nan_at is not None:
            Q[nan_at] = np.nan
        return torch.from_numpy(Q).cuda()

    for nprobe in (8, 20):
        pipe = AsyncPipeline(L, h, d, nprobes=nprobe, refine_factor=3)
        sync = hip_device_search(L, h, d, nprobes=nprobe, refine_factor=3)
        Qs = [batch(64), batch(64, nan_at=7), batch(64), batch(40), batch(64, nan_at=0), batch(64)]
        outs = []
        for q in Qs:  # batch i enqueued, then batch i - 1 completed (its outputs copied out at once)
            r = pipe.step(q, k)
            if r is not None:
                outs.append(tuple(x.cpu().numpy() for x in r))
        outs.append(tuple(x.cpu().numpy() for x in pipe.drain()))
        assert len(outs) == len(Qs)
        for i, q in enumerate(Qs):
            e = tuple(x.cpu().numpy() for x in sync(q, k))
            g = outs[i]
            np.testing.assert_array_equal(g[2], e[2], err_msg=f"batch {i}")
            np.testing.assert_array_equal(g[0], e[0], err_msg=f"batch {i}")
            np.testing.assert_allclose(g[1], e[1], rtol=0, atol=0, equal_nan=True, err_msg=f"batch {i}")


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
def test_pq_lut_fused_equals_split(hip, mk, metric):
    """The fast scan's per-query tables in one launch (pq_lut = fused, the
    default: fp8 rounding + ADC table + 8-bit LUT with P in LDS) give the same
    searches as the three launches (pq_lut = split), f32 and fp8 queries, and
    the oracle's (whose LUT restates pq_lut_u8 bit for bit)."""
    rng = np.random.default_rng(99)
    n, d, nlist = 15_000, 96, 64
    X = clustered(rng, n, d, centers=24)
    Q = (X[rng.choice(n, 50, replace=False)] + 0.3 * rng.standard_normal((50, d))).astype(np.float32)
    h = mk(d, metric, "ivf_pq")
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedCreateIndex(h, nlist, 12)
    for qm in ("f32", "fp8"):
        hip.LanceHipSetOption(h, "pq_query", qm)
        res = {}
        for mode in ("fused", "split"):
            hip.LanceHipSetOption(h, "pq_lut", mode)
            res[mode] = hip.LanceDetachedSearchBatch(h, Q, 10, nprobes=12, refine_factor=4)
        for x, y in zip(res["fused"], res["split"]):
            np.testing.assert_array_equal(x, y)
        el, ed, ec = oracle_search(hip, h, X, Q, 10, 12, 4, metric, "u8", qm == "fp8")
        assert_same(*res["fused"], el, ed, ec)
    hip.LanceHipSetOption(h, "pq_lut", "fused")
