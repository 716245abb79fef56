"""GPU parity for a bf16-stored base (storage option "bf16"; SURVEY.md §8 C3:
flat inner product on a bf16 base).  The stored rows are the bf16 roundings
(round to nearest even) of the rows handed to add; results are exact with
respect to the STORED rows, so the oracle runs on the rounded base.  Bar as
for f32: labels bit-exact, distances within 1e-4 relative."""
import numpy as np
import pytest

from oracle import c_oracle, flat_knn
from tests.test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def bf16_round(x):
    """f32 -> nearest-even bf16 -> f32 (finite inputs)."""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return (r & 0xFFFFFFFF).astype(np.uint32).view(np.float32)


@pytest.fixture
def mkbf(hip, tmp_path):
    made = []

    def make(dim, metric="l2", path=None, table="vectors"):
        h = hip.LanceCreateDetached(str(path if path is not None else tmp_path), dim, metric, table)
        hip.LanceHipSetOption(h, "storage", "bf16")
        made.append(h)
        return h

    yield make
    for h in made:
        hip.LanceFreeDetached(h)


def test_bf16_round_helper():
    x = np.array([1.0, 1.00390625, 1.0078125, 1.01171875, -3.3e-3], np.float32)
    # 1 + 2^-8 is a tie between 1 and 1 + 2^-7: even mantissa (1.0) wins
    assert bf16_round(x)[1] == np.float32(1.0)
    assert bf16_round(x)[3] == np.float32(1.015625)


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
@pytest.mark.parametrize("dim", [3, 64, 100, 768])
def test_bf16_dense_path(hip, mkbf, metric, dim):
    rng = np.random.default_rng(dim)
    X = rng.standard_normal((3000, dim)).astype(np.float32)
    Q = rng.standard_normal((9, dim)).astype(np.float32)
    h = mkbf(dim, metric)
    hip.LanceDetachedAddBatch(h, X, len(X), dim)
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
    Xr = bf16_round(X)
    el, ed, ec = flat_knn.flat_search_batch(Xr, np.arange(len(X)), np.ones(len(X), bool), Q, 10, metric)
    assert_same(gl, gd, gc, el, ed, ec)


@pytest.mark.parametrize("metric", ["l2", "dot"])
def test_bf16_sampled_path_with_deletes(hip, mkbf, metric):
    rng = np.random.default_rng(7)
    n, d = 150_000, 96
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((300, d)).astype(np.float32)
    h = mkbf(d, metric)
    hip.LanceDetachedAddBatch(h, X, n, d)
    dead = rng.choice(n, 15_000, replace=False)
    hip.LanceDetachedDeleteBatch(h, dead)
    live = np.ones(n, bool)
    live[dead] = False
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
    assert not hip.LanceHipLastSearchStats(h)["dense_path"]
    el, ed, ec = c_oracle.flat_search_batch(bf16_round(X), Q, 10, metric, live=live, acc64=True, nthreads=16)
    assert_same(gl, gd, gc, el, ed, ec)


def test_bf16_inner_product_k100_normalized(hip, mkbf):
    # C3 at reduced N: L2-normalized base and queries, IP, k = 100
    rng = np.random.default_rng(3)
    n, d = 120_000, 768
    X = rng.standard_normal((n, d)).astype(np.float32)
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    Q = rng.standard_normal((64, d)).astype(np.float32)
    Q /= np.linalg.norm(Q, axis=1, keepdims=True)
    h = mkbf(d, "dot")
    hip.LanceDetachedAddBatch(h, X, n, d)
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 100)
    st = hip.LanceHipLastSearchStats(h)
    assert not st["dense_path"]
    el, ed, ec = c_oracle.flat_search_batch(bf16_round(X), Q, 100, "dot", acc64=True, nthreads=16)
    assert_same(gl, gd, gc, el, ed, ec)


def test_bf16_get_vector_compact_and_storage_rules(hip, mkbf):
    rng = np.random.default_rng(5)
    X = rng.standard_normal((5000, 40)).astype(np.float32)
    h = mkbf(40)
    hip.LanceDetachedAddBatch(h, X, len(X), 40)
    np.testing.assert_array_equal(hip.LanceDetachedGetVector(h, 17, 40), bf16_round(X[17]))
    with pytest.raises(hip.IOException, match="empty table"):
        hip.LanceHipSetOption(h, "storage", "f32")
    with pytest.raises(hip.IOException, match="storage must be"):
        hip.LanceHipSetOption(h, "storage", "fp8")
    dead = np.arange(0, 5000, 3)
    hip.LanceDetachedDeleteBatch(h, dead)
    hip.LanceDetachedCompact(h)
    live = np.ones(5000, bool)
    live[dead] = False
    Q = rng.standard_normal((5, 40)).astype(np.float32)
    gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
    el, ed, ec = flat_knn.flat_search_batch(bf16_round(X), np.arange(5000), live, Q, 10)
    assert_same(gl, gd, gc, el, ed, ec)


def test_bf16_storage_survives_reopen(hip, tmp_path):
    rng = np.random.default_rng(11)
    X = rng.standard_normal((2000, 24)).astype(np.float32)
    Q = rng.standard_normal((4, 24)).astype(np.float32)
    p = str(tmp_path / "db")
    h = hip.LanceCreateDetached(p, 24, "l2", "t")
    hip.LanceHipSetOption(h, "storage", "bf16")
    hip.LanceDetachedAddBatch(h, X, len(X), 24)
    hip.LanceDetachedDeleteBatch(h, [3, 4])
    a = hip.LanceDetachedSearchBatch(h, Q, 7)
    hip.LanceFreeDetached(h)
    h2 = hip.LanceOpenDetached(p, "t", "l2")
    try:
        b = hip.LanceDetachedSearchBatch(h2, Q, 7)
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
        np.testing.assert_array_equal(hip.LanceDetachedGetVector(h2, 9, 24), bf16_round(X[9]))
    finally:
        hip.LanceFreeDetached(h2)
