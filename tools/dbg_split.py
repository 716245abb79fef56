"""Development-only: the split_div parity case of tests/test_gpu_scan8.py with
per-k statistics (which library: LANCE_HIP_LIB)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-lancedb_amd")]
import torch  # noqa: F401,E402
import lance_hip as hip  # noqa: E402
from oracle import c_oracle  # noqa: E402

rng = np.random.default_rng(77)
n, d = 262_144, 768
X = rng.standard_normal((n, d), dtype=np.float32)
Q = rng.standard_normal((256, d), dtype=np.float32)
for metric in sys.argv[1:] or ["l2"]:
    h = hip.LanceCreateDetached("", d, metric, "t")
    for lo in range(0, n, 131_072):
        hip.LanceDetachedAddBatch(h, X[lo:lo + 131_072], 131_072, d)
    for k in (10, 100):
        el, ed, ec = c_oracle.flat_search_batch(X, Q, k, metric, acc64=True, nthreads=16)
        for sd in ("0", "8"):
            hip.LanceHipSetOption(h, "split_div", sd)
            for rp in ("1", "0"):
                hip.LanceHipSetOption(h, "retry_pass", rp)
                gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, k)
                st = hip.LanceHipLastSearchStats(h)
                print(f"{metric} k={k} split={sd} retry={rp} exact={bool((gl == el).all())} "
                      f"bad_q={int((gl != el).any(1).sum())} {st}", flush=True)
    hip.LanceFreeDetached(h)
