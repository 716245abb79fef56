"""CPU: the oracle pinned against the reference's own golden answers, and the
two oracle restatements (numpy / C) cross-checked.  No GPU needed."""
import numpy as np
import pytest

from oracle import c_oracle, flat_knn
from tests.golden_runner import (check_filter_result, eval_predicate, load_seeded, load_sql_goldens, run_index_case,
                                 seeded_inputs)


class _OracleIx:
    """LanceIndex surface over the oracle (lance_index.cpp semantics)."""

    def __init__(self, dim):
        self.o = flat_knn.LanceIndexOracle(dim)

    def Append(self, rows, row_ids):
        self.o.append(rows, row_ids)

    def Delete(self, row_ids):
        self.o.delete(row_ids)

    def Search(self, q, dim, k):
        if dim != self.o.dim:
            return []
        return self.o.search(q, k)

    def CreateHnswIndex(self, m, ef):
        pass


def _restart(ix):
    ix.o.detached = ix.o.detached.reopen()
    return ix


INDEX_CASES = [c for c in load_sql_goldens() if "steps" in c and not c["name"].startswith("rust_")]


@pytest.mark.parametrize("case", INDEX_CASES, ids=[c["name"] for c in INDEX_CASES])
def test_oracle_sql_goldens(case):
    run_index_case(case, _OracleIx, _restart)


@pytest.mark.parametrize("tie", ["label_desc", "label_asc"])
def test_oracle_filter_goldens(tie):
    # label_desc (the default): every answer of lance_optimizer_filter.test verbatim, :36-44's tie included
    case = next(c for c in load_sql_goldens() if c["name"] == "filter_pushdown")
    X = np.array(case["rows"], np.float32)
    for q in case["queries"]:
        keep = np.array([eval_predicate(q["where"], l, s) for l, s in zip(case["lang"], case["score"])])
        labs, d = flat_knn.flat_search(X, np.arange(len(X)), keep, np.array([1, 0, 0], np.float32), q["k"], tie=tie)
        ids = [case["ids"][i] for i in labs]
        check_filter_result(q, ids, tie)
        if tie == "label_desc":
            assert ids == q["expect_ids"]
        keep8 = keep.astype(np.uint8)
        lc, _, _ = c_oracle.flat_search_batch(X, np.array([[1, 0, 0]], np.float32), q["k"], "l2", live=keep8,
                                              acc64=True, nthreads=1, tie=tie)
        assert list(lc[0, :len(labs)]) == list(labs)


def test_oracle_rust_label_semantics():
    cases = {c["name"]: c for c in load_sql_goldens()}
    # lance_manager.rs:779-804
    o = flat_knn.DetachedIndexOracle(3)
    labs = [int(o.add_batch(np.array([r], np.float32))[0]) for r in cases["rust_next_label_unique_after_deletes"]
            ["steps"][0]["rows"]]
    assert labs == [0, 1, 2, 3, 4]
    o.delete_batch([1, 2])
    o = o.reopen()
    assert int(o.add_batch(np.array([[99, 0, 0]], np.float32))[0]) >= 5
    # lance_manager.rs:806-818
    o = flat_knn.DetachedIndexOracle(2).reopen()
    assert int(o.add_batch(np.array([[1, 2]], np.float32))[0]) == 0
    # lance_manager.rs:843-867
    a, b = flat_knn.DetachedIndexOracle(2), flat_knn.DetachedIndexOracle(2)
    a.add_batch(np.array([[1, 0], [2, 0]], np.float32))
    b.add_batch(np.array([[10, 0]], np.float32))
    assert a.reopen().count() == 2 and b.reopen().count() == 1


def test_oracle_dimension_error():
    o = flat_knn.DetachedIndexOracle(3)
    o.add_batch(np.eye(3, dtype=np.float32))
    with pytest.raises(ValueError):
        o.search(np.zeros(2, np.float32), 1)


def test_squared_l2_not_sqrt():
    # lance_basic.test:33-42 pins 2.0 for [1,0,0] vs [0,1,0]
    d = flat_knn.exact_distances(np.array([[0, 1, 0]], np.float32), np.array([1, 0, 0], np.float32))
    assert d[0] == np.float32(2.0)


def test_metric_names():
    assert flat_knn.normalize_metric("ip") == "dot"
    assert flat_knn.normalize_metric("dot") == "dot"
    assert flat_knn.normalize_metric("cosine") == "cosine"
    assert flat_knn.normalize_metric("l2") == "l2"
    assert flat_knn.normalize_metric("whatever") == "l2"


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
def test_small_fixture_python_vs_c(metric):
    z = np.load("tests/golden/knn_small.npz")
    X, Q, live = z["X"], z["Q"], z["live"]
    l, d, c = flat_knn.flat_search_batch(X, np.arange(len(X)), live, Q, 5, metric)
    np.testing.assert_array_equal(l, z[f"{metric}_labels"])
    np.testing.assert_array_equal(d, z[f"{metric}_dists"])
    lc, dc, cc = c_oracle.flat_search_batch(X, Q, 5, metric, live=live, acc64=True, nthreads=4)
    np.testing.assert_array_equal(lc, l)
    np.testing.assert_allclose(dc, d, rtol=1e-6, atol=1e-6)


def test_ties_break_by_label():
    z = np.load("tests/golden/knn_ties.npz")
    l, d, c = flat_knn.flat_search_batch(z["X"], np.arange(40), np.ones(40, bool), z["Q"], 12)
    np.testing.assert_array_equal(l, z["labels"])
    # 10 identical rows at distance 0: the default tie rule, labels descending
    assert list(l[0, :10]) == list(range(9, -1, -1))
    lc, dc, _ = c_oracle.flat_search_batch(z["X"], z["Q"], 12, "l2", acc64=True, nthreads=3)
    np.testing.assert_array_equal(lc, l)
    # 20 rows tie at the second query's k-th distance: the tie rule picks which come out
    assert list(l[1]) == list(range(19, 7, -1))
    la, _, _ = flat_knn.flat_search_batch(z["X"], np.arange(40), np.ones(40, bool), z["Q"], 12, tie="label_asc")
    np.testing.assert_array_equal(la, z["labels_asc"])
    assert list(la[0, :10]) == list(range(10)) and list(la[1]) == list(range(12))
    lca, _, _ = c_oracle.flat_search_batch(z["X"], z["Q"], 12, "l2", acc64=True, nthreads=3, tie="label_asc")
    np.testing.assert_array_equal(lca, la)


@pytest.mark.parametrize("spec", [s for s in load_seeded() if s["n"] <= 10000], ids=lambda s: s["name"])
def test_seeded_fixture_pinned(spec):
    X, Q, exp = seeded_inputs(spec)
    l, d, c = c_oracle.flat_search_batch(X, Q, spec["k"], spec["metric"], acc64=True, nthreads=8)
    np.testing.assert_array_equal(l, exp["labels"])
    np.testing.assert_allclose(d, exp["dists"], rtol=1e-6)


def test_c_oracle_f32_mode_close_to_f64():
    X, Q, exp = seeded_inputs(next(s for s in load_seeded() if s["name"] == "c1_10k_d128"))
    l, d, c = c_oracle.flat_search_batch(X, Q, 10, "l2", acc64=False, nthreads=8)
    assert flat_knn.recall_at_k(l, exp["labels"], 10) >= 0.99
    np.testing.assert_allclose(d, exp["dists"], rtol=1e-4)


def test_k_larger_than_live_and_empty():
    X = np.eye(3, dtype=np.float32)
    live = np.array([1, 0, 1], bool)
    l, d = flat_knn.flat_search(X, np.arange(3), live, np.array([1, 0, 0], np.float32), 10)
    assert list(l) == [0, 2]
    l, d = flat_knn.flat_search(X, np.arange(3), np.zeros(3, bool), np.array([1, 0, 0], np.float32), 10)
    assert l.size == 0
