"""GPU parity of the register-streamed append scan (rscan_kernels.hip, option
"rscan") against the exact oracle and against the LDS-staged scan_kernel, over
the ring depths it instantiates (6 / 8 / 4 windows of 128 B per row), f32 rows
and the bf16 scan copy, every metric, deleted rows and several query tiles.
Bar: labels bit-exact, distances within 1e-4 relative (exact f64 refine)."""
import numpy as np
import pytest

from oracle import c_oracle
from tests.test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


# dim -> windows per row: f32 ld*4/128, bf16 ld*2/128 (ld = dim rounded up to 64)
@pytest.mark.parametrize("dim", [128, 256, 384, 768])
@pytest.mark.parametrize("scan_copy", ["on", "off"])
@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
def test_rscan_matches_oracle(hip, tmp_path, dim, scan_copy, metric):
    rng = np.random.default_rng(dim + (7 if scan_copy == "on" else 0))
    n = 70_000 + 3 * dim  # past the dense-path limit; ragged last tile
    X = rng.standard_normal((n, dim)).astype(np.float32)
    Q = rng.standard_normal((300, dim)).astype(np.float32)  # two query tiles
    h = hip.LanceCreateDetached(str(tmp_path), dim, metric, "t")
    try:
        hip.LanceHipSetOption(h, "scan_copy", scan_copy)
        hip.LanceDetachedAddBatch(h, X, n, dim)
        dead = rng.choice(n, 5_000, replace=False)
        hip.LanceDetachedDeleteBatch(h, dead)
        live = np.ones(n, bool)
        live[dead] = False
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, metric, live=live, acc64=True, nthreads=16)
        for rs in ("1", "0"):
            hip.LanceHipSetOption(h, "rscan", rs)
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
            st = hip.LanceHipLastSearchStats(h)
            assert not st["dense_path"]
            assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)
