"""GPU parity of the f32 store with and without its bf16 scan copy (option
"scan_copy").  The scan copy only changes what the lower-bound scan streams;
refine reads the f32 rows, so results must equal the f32 oracle either way:
labels bit-exact, distances within 1e-4 relative."""
import numpy as np
import pytest

from oracle import c_oracle, flat_knn
from tests.test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scan_copy", ["on", "off"])
@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
def test_sampled_path_both_scan_sources(hip, tmp_path, metric, scan_copy):
    rng = np.random.default_rng(21)
    n, d = 140_000, 72
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((260, d)).astype(np.float32)
    h = hip.LanceCreateDetached(str(tmp_path), d, metric, "t")
    try:
        hip.LanceHipSetOption(h, "scan_copy", scan_copy)
        hip.LanceDetachedAddBatch(h, X, n, d)
        dead = rng.choice(n, 9_000, replace=False)
        hip.LanceDetachedDeleteBatch(h, dead)
        live = np.ones(n, bool)
        live[dead] = False
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        assert not hip.LanceHipLastSearchStats(h)["dense_path"]
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, metric, live=live, acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)


def test_toggle_grow_compact(hip, tmp_path):
    # scan copy dropped and rebuilt on a populated store, kept in step through
    # growth (reserve) and compaction
    rng = np.random.default_rng(8)
    d = 48
    X = rng.standard_normal((90_000, d)).astype(np.float32)
    Q = rng.standard_normal((33, d)).astype(np.float32)
    h = hip.LanceCreateDetached(str(tmp_path), d, "l2", "t")
    try:
        hip.LanceDetachedAddBatch(h, X[:30_000], 30_000, d)
        hip.LanceHipSetOption(h, "scan_copy", "off")
        hip.LanceDetachedAddBatch(h, X[30_000:50_000], 20_000, d)
        hip.LanceHipSetOption(h, "scan_copy", "on")  # rebuilt from the f32 rows
        hip.LanceDetachedAddBatch(h, X[50_000:], 40_000, d)  # grows the store
        dead = np.arange(0, 90_000, 7)
        hip.LanceDetachedDeleteBatch(h, dead)
        live = np.ones(90_000, bool)
        live[dead] = False
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 16)
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 16, "l2", live=live, acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
        hip.LanceDetachedCompact(h)
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 16)
        assert_same(gl, gd, gc, el, ed, ec)
        np.testing.assert_array_equal(hip.LanceDetachedGetVector(h, 12, d), X[12])
        with pytest.raises(hip.IOException, match="scan_copy must be"):
            hip.LanceHipSetOption(h, "scan_copy", "maybe")
    finally:
        hip.LanceFreeDetached(h)


def test_dense_path_with_scan_copy(hip, tmp_path):
    rng = np.random.default_rng(4)
    X = rng.standard_normal((5000, 130)).astype(np.float32)
    Q = rng.standard_normal((7, 130)).astype(np.float32)
    h = hip.LanceCreateDetached(str(tmp_path), 130, "l2", "t")
    try:
        hip.LanceDetachedAddBatch(h, X, len(X), 130)
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        el, ed, ec = flat_knn.flat_search_batch(X, np.arange(len(X)), np.ones(len(X), bool), Q, 10)
        assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)
