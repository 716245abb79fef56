"""GPU parity of the int8 scan copy (option "scan_i8"): the flat scans stream
int8 rows (per-row scale) and int8 queries on v_mfma_i32_32x32x32_i8 with their
own rigorous lower bound (|e_x||q| + |x~||e_q|, knn_kernels.hip
rows_to_i8_kernel); refine, the certificate and the fallback are unchanged, so
results must equal the f64 oracle exactly as with the bf16 scan: labels
bit-exact, distances within 1e-4 relative (reference semantics:
lance_manager.rs:393-451, squared L2 / 1 - x.q / cosine)."""
import numpy as np
import pytest

from oracle import c_oracle, flat_knn
from tests.test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def _mk(hip, tmp_path, d, metric):
    h = hip.LanceCreateDetached(str(tmp_path), d, metric, "t")
    hip.LanceHipSetOption(h, "scan_i8", "on")
    return h


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
def test_sampled_path_i8(hip, tmp_path, metric):
    rng = np.random.default_rng(31)
    n, d = 140_000, 120  # ld 128
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((260, d)).astype(np.float32)
    h = _mk(hip, tmp_path, d, metric)
    try:
        hip.LanceDetachedAddBatch(h, X, n, d)
        dead = rng.choice(n, 9_000, replace=False)
        hip.LanceDetachedDeleteBatch(h, dead)
        live = np.ones(n, bool)
        live[dead] = False
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        st = hip.LanceHipLastSearchStats(h)
        assert not st["dense_path"]
        assert hip.LanceHipKernelTimes(h)["scan_elem_bytes"] == 1
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, metric, live=live, acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
        assert st["fallback_queries"] <= 3, st
    finally:
        hip.LanceFreeDetached(h)


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
@pytest.mark.parametrize("k", [1, 10, 100])
def test_dense_path_i8(hip, tmp_path, metric, k):
    rng = np.random.default_rng(7 + k)
    n, d = 6000, 256
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((37, d)).astype(np.float32)
    h = _mk(hip, tmp_path, d, metric)
    try:
        hip.LanceDetachedAddBatch(h, X, n, d)
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, k)
        assert hip.LanceHipLastSearchStats(h)["dense_path"]
        el, ed, ec = c_oracle.flat_search_batch(X, Q, k, metric, acc64=True)
        assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)


def test_d768_k100_i8(hip, tmp_path):
    rng = np.random.default_rng(768)
    n, d = 100_000, 768
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((256, d)).astype(np.float32)
    h = _mk(hip, tmp_path, d, "l2")
    try:
        hip.LanceDetachedAddBatch(h, X, n, d)
        for k in (10, 100):
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, k)
            el, ed, ec = c_oracle.flat_search_batch(X, Q, k, "l2", acc64=True, nthreads=16)
            assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)


def test_i8_rebuilt_after_mutations(hip, tmp_path):
    # the int8 copy is derived from the f32 rows: appends, deletes, growth and
    # compaction must all be visible to the next search
    rng = np.random.default_rng(88)
    d = 128
    X = rng.standard_normal((150_000, d)).astype(np.float32)
    Q = rng.standard_normal((40, d)).astype(np.float32)
    h = _mk(hip, tmp_path, d, "l2")
    try:
        hip.LanceDetachedAddBatch(h, X[:80_000], 80_000, d)
        live = np.zeros(150_000, bool)
        live[:80_000] = True
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, "l2", live=live, acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
        # delete every current nearest neighbour: the tombstones must reach the int8 row terms
        nn = np.unique(el[:, :5])
        hip.LanceDetachedDeleteBatch(h, nn)
        live[nn] = False
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, "l2", live=live, acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
        hip.LanceDetachedAddBatch(h, X[80_000:], 70_000, d)  # grows the store
        live[80_000:] = True
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, "l2", live=live, acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
        hip.LanceDetachedCompact(h)
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        assert_same(gl, gd, gc, el, ed, ec)
        hip.LanceHipSetOption(h, "scan_i8", "off")  # back to the bf16 scan
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        assert_same(gl, gd, gc, el, ed, ec)
        with pytest.raises(hip.IOException, match="scan_i8 must be"):
            hip.LanceHipSetOption(h, "scan_i8", "maybe")
    finally:
        hip.LanceFreeDetached(h)


def test_i8_ties_and_duplicates(hip, tmp_path):
    # identical rows: bounds tie, the certificate decides, the fallback keeps it exact
    rng = np.random.default_rng(5)
    d = 128
    base = rng.standard_normal((1, d)).astype(np.float32)
    X = np.concatenate([np.repeat(base, 3000, 0), rng.standard_normal((90_000, d)).astype(np.float32)])
    Q = np.concatenate([base + 0.01 * rng.standard_normal((8, d)).astype(np.float32),
                        rng.standard_normal((8, d)).astype(np.float32)])
    h = _mk(hip, tmp_path, d, "l2")
    try:
        hip.LanceDetachedAddBatch(h, X, len(X), d)
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, "l2", acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)


@pytest.mark.parametrize("d", [64, 1100])
def test_i8_not_applicable_falls_back_to_bf16(hip, tmp_path, d):
    # ld not a multiple of 128, or past the exact-integer limit: the bf16 scan runs
    rng = np.random.default_rng(d)
    X = rng.standard_normal((70_000, d)).astype(np.float32)
    Q = rng.standard_normal((9, d)).astype(np.float32)
    h = _mk(hip, tmp_path, d, "cosine")
    try:
        hip.LanceDetachedAddBatch(h, X, len(X), d)
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        assert hip.LanceHipKernelTimes(h)["scan_elem_bytes"] == 2
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, "cosine", acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)


def test_i8_zero_cosine_query(hip, tmp_path):
    rng = np.random.default_rng(2)
    d = 128
    X = rng.standard_normal((70_000, d)).astype(np.float32)
    Q = rng.standard_normal((4, d)).astype(np.float32)
    Q[2] = 0.0
    h = _mk(hip, tmp_path, d, "cosine")
    try:
        hip.LanceDetachedAddBatch(h, X, len(X), d)
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 5)
        el, ed, ec = flat_knn.flat_search_batch(X, np.arange(len(X)), np.ones(len(X), bool), Q, 5, metric="cosine")
        for i in (0, 1, 3):
            assert gc[i] == ec[i]
            np.testing.assert_array_equal(gl[i], el[i])
    finally:
        hip.LanceFreeDetached(h)


def test_i8_prepare_option(hip, tmp_path):
    # "prepare" builds the int8 copy eagerly; searches after it (and after a
    # later change, which rebuilds lazily) stay exact; a no-op where int8 does not apply
    rng = np.random.default_rng(12)
    d = 256
    X = rng.standard_normal((90_000, d)).astype(np.float32)
    Q = rng.standard_normal((20, d)).astype(np.float32)
    h = _mk(hip, tmp_path, d, "dot")
    try:
        hip.LanceDetachedAddBatch(h, X[:60_000], 60_000, d)
        hip.LanceHipSetOption(h, "prepare", "1")
        live = np.zeros(90_000, bool)
        live[:60_000] = True
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 7)
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 7, "dot", live=live, acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
        hip.LanceDetachedAddBatch(h, X[60_000:], 30_000, d)
        live[:] = True
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 7)
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 7, "dot", live=live, acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)
    h2 = _mk(hip, tmp_path, 40, "l2")  # ld 64: int8 does not apply
    try:
        hip.LanceDetachedAddBatch(h2, X[:1000, :40].copy(), 1000, 40)
        hip.LanceHipSetOption(h2, "prepare", "1")
    finally:
        hip.LanceFreeDetached(h2)


def test_i8_incremental_append_and_delete(hip, tmp_path):
    # appends that fit the reserved capacity and deletes update a current int8
    # copy in place (no rebuild); results stay exact after each change
    rng = np.random.default_rng(321)
    d = 128
    X = rng.standard_normal((120_000, d)).astype(np.float32)
    X[100_000:] *= 3.0  # later rows with larger norms: the int8 maxima must grow
    Q = rng.standard_normal((24, d)).astype(np.float32) * 2.0
    h = _mk(hip, tmp_path, d, "l2")
    try:
        hip.LanceHipSetOption(h, "reserve_rows", "131072")
        live = np.zeros(len(X), bool)
        for lo, hi in ((0, 70_000), (70_000, 100_000), (100_000, 120_000)):
            hip.LanceDetachedAddBatch(h, X[lo:hi], hi - lo, d)
            live[lo:hi] = True
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
            el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, "l2", live=live, acc64=True, nthreads=16)
            assert_same(gl, gd, gc, el, ed, ec)
            dead = np.unique(el[:, :3])
            hip.LanceDetachedDeleteBatch(h, dead)
            live[dead] = False
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
            el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, "l2", live=live, acc64=True, nthreads=16)
            assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)
