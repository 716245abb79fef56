"""GPU parity: the HIP path through the C-ABI vs the oracle and the reference's
goldens.  Bar (BASELINE.json north_star): returned labels bit-exact, distances
within 1e-4 relative (f32); the canonical order is (distance, label under the
tie rule: label descending by default, option / LANCE_HIP_TIE label_asc)."""
import os

import numpy as np
import pytest

from oracle import c_oracle, flat_knn
from tests.golden_runner import load_seeded, load_sql_goldens, run_index_case, seeded_inputs

pytestmark = pytest.mark.gpu

RTOL = 1e-4
ATOL = 1e-5


def assert_same(gl, gd, gc, el, ed, ec=None):
    gl, gd = np.asarray(gl), np.asarray(gd)
    el, ed = np.asarray(el), np.asarray(ed)
    if ec is not None:
        np.testing.assert_array_equal(gc, ec)
    for i in range(el.shape[0]):
        n = int(gc[i]) if gc is not None else el.shape[1]
        np.testing.assert_array_equal(gl[i, :n], el[i, :n], err_msg=f"query {i}")
        np.testing.assert_allclose(gd[i, :n], ed[i, :n], rtol=RTOL, atol=ATOL, err_msg=f"query {i}")


@pytest.fixture
def mk(hip, tmp_path):
    made = []

    def make(dim, metric="l2", path=None, table="vectors"):
        h = hip.LanceCreateDetached(str(path if path is not None else tmp_path), dim, metric, table)
        made.append(h)
        return h

    yield make
    for h in made:
        hip.LanceFreeDetached(h)


# ---------------------------------------------------------------------------
# the reference's own goldens through the LanceIndex mirror
# ---------------------------------------------------------------------------
INDEX_CASES = [c for c in load_sql_goldens() if "steps" in c and not c["name"].startswith("rust_")]


@pytest.mark.parametrize("case", INDEX_CASES, ids=[c["name"] for c in INDEX_CASES])
def test_sql_goldens(hip, tmp_path, case):
    def make(dim):
        return hip.LanceIndex(case["name"], dim, {}, lance_path=str(tmp_path / "db.lance" / case["name"]))

    def restart(ix):
        meta = ix.Serialize()
        ix.CommitDrop()
        return hip.LanceIndex.LoadFromStorage(ix.name, meta)

    run_index_case(case, make, restart)


def test_filter_golden_unfiltered_query(hip, tmp_path):
    # lance_optimizer_filter.test:47-54 (no WHERE): top-2 of [1,0,0] -> ids 1,2
    case = next(c for c in load_sql_goldens() if c["name"] == "filter_pushdown")
    ix = hip.LanceIndex("docs_idx", 3, {}, lance_path=str(tmp_path))
    ix.Append(np.array(case["rows"], np.float32), list(range(5)))
    res = ix.Search(np.array([1, 0, 0], np.float32), 3, 2)
    assert [case["ids"][r] for r, _ in res] == [1, 2]
    # a vector-only index has no `lang` column (multi-column tables: test_gpu_filter.py)
    with pytest.raises(hip.IOException, match="no column"):
        ix.Search(np.array([1, 0, 0], np.float32), 3, 2, predicate="lang = 'en'")


def test_rust_label_semantics(hip, tmp_path):
    p = str(tmp_path / "t.lance")
    h = hip.LanceCreateDetached(p, 3, "l2", "vectors")
    labs = [hip.LanceDetachedAdd(h, np.array([i, 0, 0], np.float32), 3) for i in range(5)]
    assert labs == [0, 1, 2, 3, 4]                                     # lance_manager.rs:786-790
    hip.LanceDetachedDelete(h, 1)
    hip.LanceDetachedDelete(h, 2)
    hip.LanceFreeDetached(h)
    h = hip.LanceOpenDetached(p, "vectors", "l2")
    assert hip.LanceDetachedAdd(h, np.array([99, 0, 0], np.float32), 3) >= 5   # :796-803
    hip.LanceFreeDetached(h)
    # empty reopen -> label 0 (:806-818)
    p2 = str(tmp_path / "e.lance")
    hip.LanceFreeDetached(hip.LanceCreateDetached(p2, 2, "l2", "vectors"))
    h = hip.LanceOpenDetached(p2, "vectors", "l2")
    assert hip.LanceDetachedAdd(h, np.array([1, 2], np.float32), 2) == 0
    hip.LanceFreeDetached(h)
    # two tables in one dataset stay independent (:843-867)
    p3 = str(tmp_path / "tbl.lance")
    a = hip.LanceCreateDetached(p3, 2, "l2", "idx_a")
    b = hip.LanceCreateDetached(p3, 2, "l2", "idx_b")
    hip.LanceDetachedAdd(a, np.array([1, 0], np.float32), 2)
    hip.LanceDetachedAdd(a, np.array([2, 0], np.float32), 2)
    hip.LanceDetachedAdd(b, np.array([10, 0], np.float32), 2)
    assert hip.LanceDetachedCount(a) == 2 and hip.LanceDetachedCount(b) == 1
    hip.LanceFreeDetached(a)
    hip.LanceFreeDetached(b)
    a = hip.LanceOpenDetached(p3, "idx_a", "l2")
    b = hip.LanceOpenDetached(p3, "idx_b", "l2")
    assert hip.LanceDetachedCount(a) == 2 and hip.LanceDetachedCount(b) == 1
    hip.LanceFreeDetached(a)
    hip.LanceFreeDetached(b)


def test_reopen_reuses_max_label_like_reference(hip, tmp_path):
    # lance_manager.rs:157-158 next_label = MAX(live label)+1: deleting the max
    # label then reopening re-issues it; the store must stay consistent.
    p = str(tmp_path)
    h = hip.LanceCreateDetached(p, 2, "l2", "vectors")
    hip.LanceDetachedAddBatch(h, np.array([[0, 0], [1, 0], [2, 0]], np.float32), 3, 2)
    hip.LanceDetachedDelete(h, 2)
    hip.LanceFreeDetached(h)
    h = hip.LanceOpenDetached(p, "vectors", "l2")
    assert hip.LanceDetachedAdd(h, np.array([5, 0], np.float32), 2) == 2
    l, d = hip.LanceDetachedSearch(h, np.array([5, 0], np.float32), 2, 3)
    assert list(l) == [2, 1, 0] and d[0] == 0.0
    hip.LanceFreeDetached(h)
    h = hip.LanceOpenDetached(p, "vectors", "l2")
    l, d = hip.LanceDetachedSearch(h, np.array([5, 0], np.float32), 2, 3)
    assert list(l) == [2, 1, 0]
    np.testing.assert_array_equal(hip.LanceDetachedGetVector(h, 2, 2), [5, 0])
    hip.LanceFreeDetached(h)


# ---------------------------------------------------------------------------
# C-ABI behaviour
# ---------------------------------------------------------------------------
def test_dimension_mismatch_is_error_at_ffi_and_empty_at_index(hip, mk):
    h = mk(3)
    hip.LanceDetachedAddBatch(h, np.eye(3, dtype=np.float32), 3, 3)
    with pytest.raises(hip.IOException, match="expected query dimension 3, got 2"):
        hip.LanceDetachedSearch(h, np.zeros(2, np.float32), 2, 1)


def test_k_and_empty_edge_cases(hip, mk):
    h = mk(4)
    l, d = hip.LanceDetachedSearch(h, np.zeros(4, np.float32), 4, 5)   # empty table
    assert l.size == 0
    hip.LanceDetachedAddBatch(h, np.eye(4, dtype=np.float32), 4, 4)
    l, d = hip.LanceDetachedSearch(h, np.zeros(4, np.float32), 4, 0)
    assert l.size == 0
    l, d = hip.LanceDetachedSearch(h, np.array([1, 0, 0, 0], np.float32), 4, 10)  # k > n
    assert list(l) == [0, 3, 2, 1]  # labels 1..3 tie at d = 2: the default tie rule, label descending
    np.testing.assert_allclose(d, [0, 2, 2, 2])
    hip.LanceDetachedDeleteBatch(h, [0, 1, 2, 3])
    assert hip.LanceDetachedCount(h) == 0
    l, d = hip.LanceDetachedSearch(h, np.array([1, 0, 0, 0], np.float32), 4, 10)
    assert l.size == 0


def test_get_vector_and_all_vectors(hip, mk):
    h = mk(5)
    X = np.random.default_rng(3).standard_normal((10, 5)).astype(np.float32)
    hip.LanceDetachedAddBatch(h, X, 10, 5)
    hip.LanceDetachedDeleteBatch(h, [3, 7])
    np.testing.assert_array_equal(hip.LanceDetachedGetVector(h, 4, 5), X[4])
    with pytest.raises(hip.IOException, match="not found"):
        hip.LanceDetachedGetVector(h, 3, 5)
    with pytest.raises(hip.IOException, match="too small"):
        hip.LanceDetachedGetVector(h, 4, 2)
    labs, vecs = hip.LanceDetachedGetAllVectors(h)
    keep = [i for i in range(10) if i not in (3, 7)]
    assert list(labs) == keep
    np.testing.assert_array_equal(vecs, X[keep])


def test_merge_assigns_fresh_labels(hip, mk, tmp_path):
    a = mk(3, path=tmp_path / "a")
    b = mk(3, path=tmp_path / "b")
    hip.LanceDetachedAddBatch(a, np.eye(3, dtype=np.float32), 3, 3)
    hip.LanceDetachedAddBatch(b, 2 * np.eye(3, dtype=np.float32), 3, 3)
    old, new = hip.LanceDetachedMerge(a, b, [0, 2])
    assert list(old) == [0, 2] and list(new) == [3, 4]
    np.testing.assert_array_equal(hip.LanceDetachedGetVector(a, 4, 3), [0, 0, 2])


def test_compact_keeps_labels(hip, mk):
    h = mk(8)
    X = np.random.default_rng(5).standard_normal((300, 8)).astype(np.float32)
    hip.LanceDetachedAddBatch(h, X, 300, 8)
    dead = list(range(0, 300, 3))
    hip.LanceDetachedDeleteBatch(h, dead)
    Q = np.random.default_rng(6).standard_normal((4, 8)).astype(np.float32)
    before = hip.LanceDetachedSearchBatch(h, Q, 7)
    hip.LanceDetachedCompact(h)
    after = hip.LanceDetachedSearchBatch(h, Q, 7)
    for x, y in zip(before, after):
        np.testing.assert_array_equal(x, y)
    live = np.ones(300, bool)
    live[dead] = False
    el, ed, ec = flat_knn.flat_search_batch(X, np.arange(300), live, Q, 7)
    assert_same(*after, el, ed, ec)


# ---------------------------------------------------------------------------
# numerics vs the oracle
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
def test_small_fixture(hip, mk, metric):
    z = np.load("tests/golden/knn_small.npz")
    X, Q, live = z["X"], z["Q"], z["live"]
    h = mk(16, metric)
    hip.LanceDetachedAddBatch(h, X, len(X), 16)
    hip.LanceDetachedDeleteBatch(h, np.nonzero(~live)[0])
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 5)
    assert_same(gl, gd, gc, z[f"{metric}_labels"], z[f"{metric}_dists"])
    # single-query entry point returns the same
    for i in range(len(Q)):
        l, d = hip.LanceDetachedSearch(h, Q[i], 16, 5)
        np.testing.assert_array_equal(l, gl[i])


@pytest.mark.parametrize("tie", [None, "label_desc", "label_asc"])
def test_ties_by_label(hip, mk, tie):
    z = np.load("tests/golden/knn_ties.npz")
    h = mk(4)
    if tie:
        hip.LanceHipSetOption(h, "tie", tie)
    hip.LanceDetachedAddBatch(h, z["X"], 40, 4)
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, z["Q"], 12)
    sfx = "_asc" if tie == "label_asc" else ""
    assert_same(gl, gd, gc, z["labels" + sfx], z["dists" + sfx], z["counts" + sfx])
    for i in range(len(z["Q"])):  # the one-query entry point (small exact kernel) agrees
        l, d = hip.LanceDetachedSearch(h, z["Q"][i], 4, 12)
        np.testing.assert_array_equal(l, gl[i])


def test_tie_option_rejects_unknown(hip, mk):
    h = mk(4)
    with pytest.raises(hip.IOException, match="tie must be"):
        hip.LanceHipSetOption(h, "tie", "random")


@pytest.mark.parametrize("tie", ["label_desc", "label_asc"])
@pytest.mark.parametrize("path", ["small_exact", "dense", "threshold"])
def test_tie_rule_on_every_path(hip, mk, tie, path):
    """Tie groups straddling the k-th place on each search path (one-launch small
    exact search, the dense path of small stores, the threshold path with its
    reruns / batched and per-query exact fallbacks), under both tie rules, vs
    the oracle: the rule decides WHICH tied rows come out, not only their order."""
    rng = np.random.default_rng(606)
    d, k = 128, 10
    n = {"small_exact": 3000, "dense": 40_000, "threshold": 120_000}[path]
    X = rng.standard_normal((n, d)).astype(np.float32)
    base = rng.standard_normal((6, d)).astype(np.float32)
    for j in range(6):  # group j: 4 + 3 j copies scattered over the store
        X[rng.choice(n, 4 + 3 * j, replace=False)] = base[j]
    Q = np.concatenate([base, base + np.float32(0.001), rng.standard_normal((4, d))]).astype(np.float32)
    live = np.ones(n, bool)
    live[rng.choice(n, n // 50, replace=False)] = False
    h = mk(d)
    hip.LanceHipSetOption(h, "tie", tie)
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedDeleteBatch(h, np.nonzero(~live)[0])
    el, ed, ec = c_oracle.flat_search_batch(X, Q, k, "l2", live=live, acc64=True, nthreads=16, tie=tie)
    if path == "small_exact":
        for i in range(len(Q)):
            l, dd = hip.LanceDetachedSearch(h, Q[i], d, k)
            np.testing.assert_array_equal(l, el[i, :ec[i]], err_msg=f"query {i}")
        return
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, k)
    assert_same(gl, gd, gc, el, ed, ec)
    st = hip.LanceHipLastSearchStats(h)
    assert st["dense_path"] == (path == "dense")


@pytest.mark.parametrize("spec", load_seeded(), ids=lambda s: s["name"])
def test_seeded_fixtures(hip, mk, spec):
    X, Q, exp = seeded_inputs(spec)
    h = mk(spec["d"], spec["metric"])
    for s in range(0, len(X), 2048):   # DuckDB sink chunks (lance_index.cpp:940-946)
        hip.LanceDetachedAddBatch(h, X[s:s + 2048], len(X[s:s + 2048]), spec["d"])
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, spec["k"])
    assert_same(gl, gd, gc, exp["labels"], exp["dists"], exp["counts"])
    st = hip.LanceHipLastSearchStats(h)
    assert st["fallback_queries"] == 0, st      # certificate holds on continuous data


@pytest.mark.parametrize("dim", [1, 3, 17, 100, 129, 1000])
def test_odd_dimensions(hip, mk, dim):
    rng = np.random.default_rng(dim)
    X = rng.standard_normal((3000, dim)).astype(np.float32)
    Q = rng.standard_normal((9, dim)).astype(np.float32)
    h = mk(dim)
    hip.LanceDetachedAddBatch(h, X, len(X), dim)
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
    el, ed, ec = flat_knn.flat_search_batch(X, np.arange(len(X)), np.ones(len(X), bool), Q, 10)
    assert_same(gl, gd, gc, el, ed, ec)


def test_sampled_path_with_deletes_and_many_queries(hip, mk):
    # > 65536 rows takes the sample + threshold-scan path; 600 queries = 3 query tiles
    rng = np.random.default_rng(99)
    n, d = 150_000, 96
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((600, d)).astype(np.float32)
    h = mk(d)
    hip.LanceDetachedAddBatch(h, X, n, d)
    dead = rng.choice(n, 20_000, replace=False)
    hip.LanceDetachedDeleteBatch(h, dead)
    live = np.ones(n, bool)
    live[dead] = False
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
    st = hip.LanceHipLastSearchStats(h)
    assert not st["dense_path"]
    el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, "l2", live=live, acc64=True, nthreads=16)
    assert_same(gl, gd, gc, el, ed, ec)


@pytest.mark.parametrize("tie", ["label_desc", "label_asc"])
def test_duplicates_force_exact_fallback(hip, mk, tie):
    # 100k identical rows: every lower bound ties, the certificate cannot hold,
    # the exact fallback must return the k largest (label_desc) / smallest labels
    n, d = 100_000, 32
    X = np.ones((n, d), np.float32)
    h = mk(d)
    hip.LanceHipSetOption(h, "tie", tie)
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedDeleteBatch(h, [0, 5, n - 2])
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, np.ones((2, d), np.float32), 10)
    if tie == "label_asc":
        assert list(gl[0]) == [1, 2, 3, 4, 6, 7, 8, 9, 10, 11]
    else:
        assert list(gl[0]) == [n - 1] + list(range(n - 3, n - 12, -1))
    assert np.all(gd == 0)
    st = hip.LanceHipLastSearchStats(h)
    assert st["fallback_queries"] == 2 and st["retried_queries"] == 2


@pytest.mark.parametrize("tie", ["label_desc", "label_asc"])
@pytest.mark.parametrize("metric", ["l2", "cosine"])
def test_batched_exact_fallback_many_queries(hip, mk, metric, tie):
    # 50 vectors each repeated ~1600 times among 100k rows: a query equal to
    # one of them ties at its nearest distance with ~1600 rows, so no
    # certificate can hold; the 50 queries (4 groups of the batched fallback)
    # must come back as the k smallest labels of their duplicates, as the
    # oracle orders them; one zero query on top (cosine: NaN distances, the
    # per-query fallback)
    rng = np.random.default_rng(77)
    n, d, k = 100_000, 32, 10
    base = rng.standard_normal((50, d)).astype(np.float32)
    X = base[rng.integers(0, 50, n)]
    X[rng.random(n) < 0.2] = rng.standard_normal((1, d)).astype(np.float32)  # another tie group
    Q = np.concatenate([base, np.zeros((1, d), np.float32)])
    live = np.ones(n, bool)
    live[rng.choice(n, 3000, replace=False)] = False
    h = mk(d, metric)
    hip.LanceHipSetOption(h, "tie", tie)
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedDeleteBatch(h, np.nonzero(~live)[0])
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, k)
    st = hip.LanceHipLastSearchStats(h)
    assert st["fallback_queries"] >= 50, st
    el, ed, ec = c_oracle.flat_search_batch(X, Q[:50], k, metric, live=live, acc64=True, nthreads=16, tie=tie)
    assert_same(gl[:50], gd[:50], gc[:50], el, ed, ec)
    assert gc[50] == k


@pytest.mark.parametrize("retry", ["1", "0"])
def test_overflowed_segment_takes_second_pass(hip, mk, retry):
    # the neighbours of three queries sit packed in tile 1 (rows 256..511),
    # which the sample pass skips: the loose sampled tau overflows that tile's
    # segment, the certificate fails, and the second threshold pass (tau = the
    # first pass's k-th exact distance, full-size segments) recovers them
    # without the exact fallback
    rng = np.random.default_rng(5)
    n, d, k = 120_000, 32, 10
    X = rng.standard_normal((n, d)).astype(np.float32)
    q0 = rng.standard_normal(d).astype(np.float32)
    dirs = rng.standard_normal((256, d))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    X[256:512] = q0 + np.sqrt(rng.uniform(0, 40, 256))[:, None] * dirs
    Q = np.concatenate([q0 + 0.01 * rng.standard_normal((3, d)), rng.standard_normal((5, d))]).astype(np.float32)
    h = mk(d)
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceHipSetOption(h, "sample_div", "100000")
    hip.LanceHipSetOption(h, "retry_pass", retry)
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, k)
    st = hip.LanceHipLastSearchStats(h)
    el, ed, ec = c_oracle.flat_search_batch(X, Q, k, "l2", acc64=True, nthreads=16)
    assert_same(gl, gd, gc, el, ed, ec)
    assert not st["dense_path"]
    if retry == "1":
        assert st["retried_queries"] >= 3 and st["fallback_queries"] == 0, st
    else:
        assert st["retried_queries"] == 0 and st["fallback_queries"] >= 3, st


def test_metric_quirk_ranks_by_l2(hip, mk):
    rng = np.random.default_rng(1)
    X = rng.standard_normal((500, 8)).astype(np.float32)
    Q = rng.standard_normal((3, 8)).astype(np.float32)
    h = mk(8, "dot")
    hip.LanceDetachedAddBatch(h, X, 500, 8)
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 5)
    el, ed, _ = flat_knn.flat_search_batch(X, np.arange(500), np.ones(500, bool), Q, 5, "dot")
    assert_same(gl, gd, gc, el, ed)
    hip.LanceHipSetOption(h, "metric_quirk", "1")
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 5)
    el, ed, _ = flat_knn.flat_search_batch(X, np.arange(500), np.ones(500, bool), Q, 5, "l2")
    assert_same(gl, gd, gc, el, ed)


def test_merge_topk_kernel(hip):
    rng = np.random.default_rng(4)
    nshard, nq, k = 4, 5, 7
    pl = np.full((nshard, nq, k), -1, np.int64)
    pd = np.full((nshard, nq, k), np.nan, np.float32)
    pc = rng.integers(0, k + 1, (nshard, nq)).astype(np.int32)
    for s in range(nshard):
        for q in range(nq):
            c = pc[s, q]
            d = np.sort(rng.integers(0, 20, c).astype(np.float32))
            pd[s, q, :c] = d
            pl[s, q, :c] = s * 1000 + np.arange(c)
    ol, od, oc = hip.LanceHipMergeTopk(pl, pd, pc)
    desc = flat_knn.tie_desc(None)  # the public merge: the process's LANCE_HIP_TIE (default label_desc)
    for q in range(nq):
        items = [(pd[s, q, i], -pl[s, q, i] if desc else pl[s, q, i]) for s in range(nshard) for i in range(pc[s, q])]
        items.sort()
        items = [(dd, -l if desc else l) for dd, l in items]
        items = items[:k]
        assert oc[q] == len(items)
        assert list(ol[q, :oc[q]]) == [l for _, l in items]


@pytest.mark.parametrize("nshard,nq,k", [(4, 5, 7), (8, 256, 10), (3, 33, 100), (3, 7, 1500)])
def test_merge_topk_packed_kernel(hip, nshard, nq, k):
    """lance_hip_merge_topk_packed over gathered packed rows (the exchange's
    one-launch merge): per-shard label offsets from the rows' tails, ragged
    counts (0..k, a few out of range), distance ties across shards, -1 slots;
    (3, 7, 1500) takes the global-memory variant (nshard * k > the LDS cap)."""
    import torch

    from lance_hip.sharded import hip_packed_merge, packed_outputs, packed_stride

    rng = np.random.default_rng(40 + k)
    stride = packed_stride(nq, k)
    offs = [int(s * 10**9 + rng.integers(0, 1000)) for s in range(nshard)]
    pl = np.full((nshard, nq, k), -1, np.int64)
    pd = np.full((nshard, nq, k), np.nan, np.float32)
    pc = rng.integers(0, k + 1, (nshard, nq)).astype(np.int32)
    pc[0, 0] = k + 5  # counts above k are read as k
    for s in range(nshard):
        for q in range(nq):
            c = min(pc[s, q], k)
            pd[s, q, :c] = np.sort(rng.integers(0, 3 * k, c).astype(np.float32))
            pl[s, q, :c] = rng.permutation(5 * k)[:c]
    rows = []
    for s in range(nshard):
        o = packed_outputs(nq, k, "cuda", offs[s], stride)
        o[0].copy_(torch.from_numpy(pl[s]))
        o[1].copy_(torch.from_numpy(pd[s]))
        o[2].copy_(torch.from_numpy(pc[s]))
        rows.append(o.pack)
    g = torch.stack(rows)
    ol, od, oc = (x.cpu().numpy() for x in hip_packed_merge(hip.lib())(g, nq, k))
    desc = flat_knn.tie_desc(None)
    for q in range(nq):
        items = [(pd[s, q, i], pl[s, q, i] + offs[s]) for s in range(nshard) for i in range(min(pc[s, q], k))]
        items.sort(key=lambda t: (t[0], -t[1] if desc else t[1]))
        items = items[:k]
        assert oc[q] == len(items)
        assert list(ol[q, :oc[q]]) == [l for _, l in items]
        assert list(od[q, :oc[q]]) == [d for d, _ in items]
        assert (ol[q, oc[q]:] == -1).all() and np.isnan(od[q, oc[q]:]).all()


def test_merge_topk_packed_rejects_bad_strides(hip):
    import torch

    from lance_hip.sharded import hip_packed_merge, packed_stride

    g = torch.zeros((2, packed_stride(4, 3) - 2), dtype=torch.int32, device="cuda")
    with pytest.raises(RuntimeError, match="row_stride"):
        hip_packed_merge(hip.lib())(g, 4, 3)


def test_cosine_repeated_searches_are_stable(hip, mk):
    # regression: the cosine epilogue once read accumulators before the last
    # MFMAs had landed (~1% of queries, timing dependent); 40 repeats x 40 queries
    rng = np.random.default_rng(3006)
    n, d = 3000, 64
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((40, d)).astype(np.float32)
    keep = rng.random(n) < 0.2
    h = mk(d, "cosine")
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedDeleteBatch(h, np.nonzero(~keep)[0])
    el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, "cosine", live=keep, acc64=True)
    for _ in range(40):
        assert_same(*hip.LanceDetachedSearchBatch(h, Q, 10), el, ed, ec)


@pytest.mark.parametrize("scan", ["copy", "f32", "bf16"])
@pytest.mark.parametrize("d", [32, 64])
def test_cosine_row_aux_slot_reuse(hip, mk, d, scan):
    # regression (root cause of the case above): a tile's stage 0 carries its
    # row aux into the LDS slot tile-2's epilogue reads; when a tile has fewer
    # k-stages than the ring (small d) that DMA was released by each wave's
    # own progress, not the workgroup's, and overwrote row terms slower waves
    # were still reading.  Append mode (> 65536 rows), many tiles per
    # workgroup, 80% deleted rows (alpha = +inf in the row aux), 1024 queries.
    rng = np.random.default_rng(4100 + d)
    n = 200_000
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((1024, d)).astype(np.float32)
    keep = rng.random(n) < 0.2
    h = mk(d, "cosine")
    if scan == "bf16":  # bf16 store: the scan streams the store itself
        hip.LanceHipSetOption(h, "storage", "bf16")
    elif scan == "f32":  # f32 store without its bf16 scan copy (32-deep f32 stages)
        hip.LanceHipSetOption(h, "scan_copy", "off")
    hip.LanceDetachedAddBatch(h, X, n, d)
    hip.LanceDetachedDeleteBatch(h, np.nonzero(~keep)[0])
    Xr = X
    if scan == "bf16":  # a bf16 store holds the round-to-nearest-even roundings
        u = X.view(np.uint32).astype(np.uint64)
        Xr = ((((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16) & 0xFFFFFFFF).astype(np.uint32).view(np.float32)
    el, ed, ec = c_oracle.flat_search_batch(Xr, Q, 10, "cosine", live=keep, acc64=True, nthreads=16)
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
    assert not hip.LanceHipLastSearchStats(h)["dense_path"]
    assert_same(gl, gd, gc, el, ed, ec)


# ---------------------------------------------------------------------------
# one-launch small exact search (<= 8 queries over <= 32768 slots)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
@pytest.mark.parametrize("n,dim,nq,k", [(1, 3, 1, 5), (300, 17, 2, 10), (10_000, 128, 1, 10), (10_000, 128, 8, 64),
                                        (32_768, 129, 3, 7), (5_000, 1000, 4, 16)])
def test_small_exact_path(hip, mk, metric, n, dim, nq, k):
    rng = np.random.default_rng(n + dim + nq)
    X = rng.standard_normal((n, dim)).astype(np.float32)
    Q = rng.standard_normal((nq, dim)).astype(np.float32)
    h = mk(dim, metric)
    hip.LanceDetachedAddBatch(h, X, n, dim)
    dead = rng.choice(n, n // 10, replace=False) if n > 10 else np.array([], np.int64)
    if len(dead):
        hip.LanceDetachedDeleteBatch(h, dead)
    live = np.ones(n, bool)
    live[dead] = False
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, k)
    assert hip.LanceHipLastSearchStats(h)["small_exact"]
    el, ed, ec = c_oracle.flat_search_batch(X, Q, k, metric, live=live, acc64=True, nthreads=16)
    assert_same(gl, gd, gc, el, ed, ec)
    # the bound/refine pipeline returns the same
    hip.LanceHipSetOption(h, "small_exact", "0")
    pl, pd, pc = hip.LanceDetachedSearchBatch(h, Q, k)
    assert not hip.LanceHipLastSearchStats(h)["small_exact"]
    np.testing.assert_array_equal(pc, gc)
    np.testing.assert_array_equal(pl, gl)
    np.testing.assert_array_equal(pd, gd)


def test_small_exact_limits_and_repeats(hip, mk):
    # just past the slot limit takes the pipeline; 9 queries take the pipeline;
    # repeated one-query calls reuse the completion counters
    rng = np.random.default_rng(3)
    X = rng.standard_normal((32_769, 8)).astype(np.float32)
    h = mk(8)
    hip.LanceDetachedAddBatch(h, X, len(X), 8)
    hip.LanceDetachedSearchBatch(h, X[:2], 4)
    assert not hip.LanceHipLastSearchStats(h)["small_exact"]
    h2 = mk(8)
    hip.LanceDetachedAddBatch(h2, X[:20_000], 20_000, 8)
    hip.LanceDetachedSearchBatch(h2, X[:9], 4)
    assert not hip.LanceHipLastSearchStats(h2)["small_exact"]
    el, ed, ec = c_oracle.flat_search_batch(X[:20_000], X[100:140], 4, "l2", acc64=True, nthreads=16)
    for i in range(40):
        l, d = hip.LanceDetachedSearch(h2, X[100 + i], 8, 4)
        assert hip.LanceHipLastSearchStats(h2)["small_exact"]
        np.testing.assert_array_equal(l, el[i])
