"""GPU parity of filtered (prefilter) search: multi-column LANCE indexes
through the Arrow C Data Interface (lance_create_detached_from_arrow /
lance_detached_add_batch_arrow, rust_lib/src/lance_manager.rs:62-126,
:251-301) and the predicate the optimizer pushes down
(src/lance_optimizer.cpp:204-344, passed at src/lance_index.cpp:452-453).
Checker: the exact oracle restricted to the rows oracle/predicate.py selects.
Bar: labels bit-exact, distances within 1e-4 relative."""
import numpy as np
import pyarrow as pa
import pytest

from oracle import c_oracle, flat_knn, ivf
from oracle import predicate as P
from tests.golden_runner import check_filter_result, load_sql_goldens

pytestmark = pytest.mark.gpu

RTOL = 1e-4
ATOL = 1e-5


def assert_same(gl, gd, gc, el, ed, ec):
    np.testing.assert_array_equal(gc, ec)
    for i in range(el.shape[0]):
        n = int(gc[i])
        np.testing.assert_array_equal(gl[i, :n], el[i, :n], err_msg=f"query {i}")
        np.testing.assert_allclose(gd[i, :n], ed[i, :n], rtol=RTOL, atol=ATOL, err_msg=f"query {i}")


@pytest.mark.parametrize("tie", ["label_desc", "label_asc"])
def test_filter_goldens_through_index_mirror(hip, tmp_path, monkeypatch, tie):
    # lance_optimizer_filter.test:9-99 — CREATE INDEX docs_idx ON docs USING LANCE (embedding, lang, score);
    # the tie rule through LANCE_HIP_TIE, read when the handle is created (label_desc: :36-44 verbatim)
    monkeypatch.setenv("LANCE_HIP_TIE", tie)
    case = next(c for c in load_sql_goldens() if c["name"] == "filter_pushdown")
    ix = hip.LanceIndex("docs_idx", 3, {}, lance_path=str(tmp_path),
                        extra_columns=[("lang", pa.string()), ("score", pa.int32())])
    ix.Append(np.array(case["rows"], np.float32), list(range(5)), {"lang": case["lang"], "score": case["score"]})
    assert hip.LanceDetachedHasExtraColumns(ix.rust_handle_)
    q = np.array([1, 0, 0], np.float32)
    for query in case["queries"]:
        res = ix.Search(q, 3, query["k"], predicate=query["where"] or "")
        check_filter_result(query, [case["ids"][r] for r, _ in res], tie)


def _meta(rng, n):
    langs = ["en", "fr", "es", "de", "it's"]
    cols = {
        "lang": [None if rng.random() < 0.05 else langs[i] for i in rng.integers(0, 5, n)],
        "score": rng.integers(0, 1000, n).tolist(),
        "price": [None if rng.random() < 0.1 else float(x) for x in rng.random(n) * 100],
        "flag": rng.random(n).astype(bool).tolist(),
    }
    types = [("lang", pa.string()), ("score", pa.int64()), ("price", pa.float64()), ("flag", pa.bool_())]
    return cols, types


def _make(hip, X, cols, types, metric, path="", chunk=None):
    batch = hip.arrow_rows(X, [(nm, cols[nm], t) for nm, t in types])
    with hip.ArrowC(batch) as sch:
        h = hip.LanceCreateDetachedFromArrow(path, sch.schema_ptr, metric, "filt")
    n = len(X)
    step = chunk or n
    for lo in range(0, n, step):
        with hip.ArrowC(batch.slice(lo, min(step, n - lo))) as a:
            labs = hip.LanceDetachedAddBatchArrow(h, a.schema_ptr, a.array_ptr)
            assert a.array.release is None  # taken over by the callee (lance_manager.rs:257)
        assert labs.tolist() == list(range(lo, min(n, lo + step)))
    return h


PREDS = ["lang = 'en'", "score > 500 AND lang IN ('fr', 'es')", "NOT (lang = 'en')", "price IS NULL",
         "(score < 100) OR (price >= 90.5)", "lang = 'it''s' AND flag", "score BETWEEN 10 AND 20",
         "label % 2 = 0"]


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
@pytest.mark.parametrize("n", [3000, 120_000])
def test_filtered_flat_search(hip, metric, n):
    rng = np.random.default_rng(n + len(metric))
    d = 64
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((40, d)).astype(np.float32)
    cols, types = _meta(rng, n)
    h = _make(hip, X, cols, types, metric, chunk=50_000)
    try:
        dead = rng.choice(n, n // 20, replace=False)
        hip.LanceDetachedDeleteBatch(h, dead)
        live = np.ones(n, bool)
        live[dead] = False
        labels = np.arange(n)
        for pred in PREDS[:-1]:
            m = np.array(P.mask(pred, cols, labels, live))
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10, predicate=pred)
            el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, metric, live=m, acc64=True, nthreads=16)
            assert_same(gl, gd, gc, el, ed, ec)
        with pytest.raises(hip.IOException):
            hip.LanceDetachedSearchBatch(h, Q, 10, predicate=PREDS[-1])  # no arithmetic in the language
        # unfiltered search is unchanged after filtered ones
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, metric, live=live, acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)


def test_selective_and_empty_filters(hip):
    # a handful of matches in a large store (sample pass finds too few rows ->
    # certificate fails -> exact fallback restricted to the matches), and none
    rng = np.random.default_rng(5)
    n, d = 100_000, 32
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((8, d)).astype(np.float32)
    cols, types = _meta(rng, n)
    h = _make(hip, X, cols, types, "l2")
    try:
        labels = np.arange(n)
        live = np.ones(n, bool)
        for pred, k in [("label < 7", 10), ("label >= 99990 OR label = 5", 4), ("score = 17 AND lang = 'de'", 20)]:
            m = np.array(P.mask(pred, cols, labels, live))
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, k, predicate=pred)
            el, ed, ec = c_oracle.flat_search_batch(X, Q, k, "l2", live=m, acc64=True, nthreads=16)
            assert_same(gl, gd, gc, el, ed, ec)
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 5, predicate="score > 5000")
        assert (gc == 0).all() and (gl == -1).all()
        lab, dist = hip.LanceDetachedSearch(h, Q[0], d, 5, predicate="score > 5000")
        assert lab.size == 0
    finally:
        hip.LanceFreeDetached(h)


@pytest.mark.parametrize("index_type", ["ivf_flat", "ivf_pq"])
def test_filtered_ivf_search(hip, index_type):
    rng = np.random.default_rng(21)
    n, d, nlist = 20_000, 32, 40
    C = rng.standard_normal((30, d)).astype(np.float32)
    X = (C[rng.integers(0, 30, n)] + 0.4 * rng.standard_normal((n, d))).astype(np.float32)
    Q = (X[rng.choice(n, 30, replace=False)] + 0.1 * rng.standard_normal((30, d))).astype(np.float32)
    cols, types = _meta(rng, n)
    h = _make(hip, X[:18_000], {k: v[:18_000] for k, v in cols.items()}, types, "l2")
    try:
        hip.LanceHipSetOption(h, "index_type", index_type)
        hip.LanceDetachedCreateIndex(h, nlist, 8)
        # rows after the build: the unindexed tail is filtered too
        batch = hip.arrow_rows(X[18_000:], [(nm, cols[nm][18_000:], t) for nm, t in types])
        with hip.ArrowC(batch) as a:
            hip.LanceDetachedAddBatchArrow(h, a.schema_ptr, a.array_ptr)
        ex = hip.LanceHipIvfExport(h)
        labels = np.arange(n)
        for pred in ["lang = 'en'", "score < 300 OR price IS NULL"]:
            m = np.array(P.mask(pred, cols, labels, ex["live"]))
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10, nprobes=6, refine_factor=3, predicate=pred)
            if index_type == "ivf_flat":
                el, ed, ec = ivf.ivf_flat_search(X, ex["labels"], m, ex["lists"], ex["centroids"], Q, 10, 6, "l2")
            else:
                el, ed, ec = ivf.ivf_pq_search(X, ex["labels"], m, ex["lists"], ex["codes"], ex["centroids"],
                                               ex["codebook"], Q, 10, 6, 3, "l2", lut="u8")
            assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)


def test_metadata_persists_compacts_and_merges(hip, tmp_path):
    rng = np.random.default_rng(8)
    n, d = 5000, 16
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((6, d)).astype(np.float32)
    cols, types = _meta(rng, n)
    h = _make(hip, X, cols, types, "l2", path=str(tmp_path), chunk=1200)
    dead = rng.choice(n, 700, replace=False)
    hip.LanceDetachedDeleteBatch(h, dead)
    live = np.ones(n, bool)
    live[dead] = False
    labels = np.arange(n)
    pred = "lang IN ('en', 'fr') AND price > 20"
    m = np.array(P.mask(pred, cols, labels, live))
    el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, "l2", live=m, acc64=True)
    assert_same(*hip.LanceDetachedSearchBatch(h, Q, 10, predicate=pred), el, ed, ec)
    hip.LanceDetachedCompact(h)  # metadata follows the surviving rows
    assert_same(*hip.LanceDetachedSearchBatch(h, Q, 10, predicate=pred), el, ed, ec)
    hip.LanceFreeDetached(h)
    # reopen from the table log: rows, deletes and metadata
    h2 = hip.LanceOpenDetached(str(tmp_path), "filt", "l2")
    try:
        assert hip.LanceDetachedHasExtraColumns(h2)
        assert_same(*hip.LanceDetachedSearchBatch(h2, Q, 10, predicate=pred), el, ed, ec)
        # merge: the extra columns travel with the merged rows (new labels n..)
        X2 = rng.standard_normal((300, d)).astype(np.float32)
        cols2, _ = _meta(rng, 300)
        h3 = _make(hip, X2, cols2, types, "l2")
        try:
            old, new = hip.LanceDetachedMerge(h2, h3, np.arange(300))
            assert new.tolist() == list(range(n, n + 300))
        finally:
            hip.LanceFreeDetached(h3)
        allX = np.concatenate([X, X2])
        allc = {k: cols[k] + cols2[k] for k in cols}
        live2 = np.concatenate([live, np.ones(300, bool)])
        m2 = np.array(P.mask(pred, allc, np.arange(n + 300), live2))
        el2, ed2, ec2 = c_oracle.flat_search_batch(allX, Q, 10, "l2", live=m2, acc64=True)
        assert_same(*hip.LanceDetachedSearchBatch(h2, Q, 10, predicate=pred), el2, ed2, ec2)
    finally:
        hip.LanceFreeDetached(h2)


def test_vector_only_table_label_predicate(hip, tmp_path):
    rng = np.random.default_rng(4)
    X = rng.standard_normal((2000, 8)).astype(np.float32)
    Q = rng.standard_normal((3, 8)).astype(np.float32)
    h = hip.LanceCreateDetached(str(tmp_path), 8, "l2", "v")
    try:
        hip.LanceDetachedAddBatch(h, X, 2000, 8)
        assert not hip.LanceDetachedHasExtraColumns(h)
        live = np.arange(2000) % 3 == 0
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 7, predicate="label IN (0, 3, 6, 9) OR label >= 1500")
        m = np.array(P.mask("label IN (0, 3, 6, 9) OR label >= 1500", {}, np.arange(2000), np.ones(2000, bool)))
        el, ed, ec = flat_knn.flat_search_batch(X, np.arange(2000), m, Q, 7)
        assert_same(gl, gd, gc, el, ed, ec)
        with pytest.raises(hip.IOException, match="no column"):
            hip.LanceDetachedSearchBatch(h, Q, 7, predicate="lang = 'en'")
        del live
    finally:
        hip.LanceFreeDetached(h)


def test_scalar_index_filtered_search(hip, tmp_path):
    # lance_index.cpp:481-486 CreateScalarIndex: same results through the index,
    # for rows indexed and rows appended after it, and after a reopen
    rng = np.random.default_rng(31)
    n, d = 40_000, 32
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((12, d)).astype(np.float32)
    cols, types = _meta(rng, n)
    h = _make(hip, X[:30_000], {k: v[:30_000] for k, v in cols.items()}, types, "l2", path=str(tmp_path))
    hip.LanceDetachedCreateScalarIndex(h, "lang", "BITMAP")
    hip.LanceDetachedCreateScalarIndex(h, "score", "btree")
    hip.LanceDetachedCreateScalarIndex(h, "price", None)
    hip.LanceDetachedCreateScalarIndex(h, "label", "BTREE")  # implicitly ordered: no-op
    with pytest.raises(hip.IOException):
        hip.LanceDetachedCreateScalarIndex(h, "nosuch", "BTREE")
    with pytest.raises(hip.IOException):
        hip.LanceDetachedCreateScalarIndex(h, "lang", "FTS")
    batch = hip.arrow_rows(X[30_000:], [(nm, cols[nm][30_000:], t) for nm, t in types])
    with hip.ArrowC(batch) as a:
        hip.LanceDetachedAddBatchArrow(h, a.schema_ptr, a.array_ptr)
    dead = rng.choice(n, 2000, replace=False)
    hip.LanceDetachedDeleteBatch(h, dead)
    live = np.ones(n, bool)
    live[dead] = False
    labels = np.arange(n)
    preds = ["lang = 'fr'", "score >= 990 OR lang = 'it''s'", "price < 3.5 AND NOT (lang IN ('en', 'de'))",
             "score BETWEEN 100 AND 105", "lang != 'en'"]
    exp = {}
    for pred in preds:
        m = np.array(P.mask(pred, cols, labels, live))
        exp[pred] = c_oracle.flat_search_batch(X, Q, 10, "l2", live=m, acc64=True)
        assert_same(*hip.LanceDetachedSearchBatch(h, Q, 10, predicate=pred), *exp[pred])
    hip.LanceDetachedCompact(h)  # indexes follow the compaction
    for pred in preds:
        assert_same(*hip.LanceDetachedSearchBatch(h, Q, 10, predicate=pred), *exp[pred])
    hip.LanceFreeDetached(h)
    h2 = hip.LanceOpenDetached(str(tmp_path), "filt", "l2")
    try:
        for pred in preds:
            assert_same(*hip.LanceDetachedSearchBatch(h2, Q, 10, predicate=pred), *exp[pred])
    finally:
        hip.LanceFreeDetached(h2)
