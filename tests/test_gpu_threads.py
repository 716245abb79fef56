"""GPU: concurrent callers, as DuckDB drives the library.

The reference searches without ``IndexLock`` (``lance_search.cpp:73-74``,
``lance_optimizer.cpp:77-78``) while ``Append`` / ``Delete`` take it
(``lance_index.hpp:37-40``), so under DuckDB a search can run while another
thread appends to or deletes from the same index, and several indexes are
searched at once (SURVEY.md §8b threading, §5 race detection).  The library
serialises calls on one handle internally (a per-handle mutex, one HIP stream
per handle); ctypes releases the GIL, so these Python threads are real
concurrency inside the library.

Checks (the f64 oracle is the checker): every search returns exactly the
oracle's lists for one store version between the mutations completed before the
call and those completed after it (a linearizable history); searches of two
handles in parallel equal their oracles; nothing hangs.
"""
import threading
import time

import numpy as np
import pytest

from oracle import flat_knn
from tests.test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

D, K = 128, 10


def _matches(res, exp):
    gl, gd, gc = res
    el, ed, ec = exp
    if not np.array_equal(gc, ec):
        return False
    for i in range(len(gc)):
        n = int(gc[i])
        if not np.array_equal(gl[i, :n], el[i, :n]):
            return False
        if not np.allclose(gd[i, :n], ed[i, :n], rtol=1e-4, atol=1e-5):
            return False
    return True


def test_search_concurrent_with_append_and_delete(hip):
    rng = np.random.default_rng(2024)
    n0, n_add, m = 80_000, 4096, 10
    X = rng.standard_normal((n0 + m * n_add, D), dtype=np.float32)
    QS = rng.standard_normal((6, D), dtype=np.float32)     # <= 8 queries: pinned host-buffer path
    QB = rng.standard_normal((40, D), dtype=np.float32)    # staged H2D / D2H path
    Q1 = QB[:1]                                           # one query per call (lance_search())
    h = hip.LanceCreateDetached("", D, "l2", "conc")
    try:
        hip.LanceDetachedAddBatch(h, X[:n0], n0, D)
        # the mutation sequence (version v = after v mutations): appends and deletes alternate
        muts = []
        n_rows = n0
        live = np.ones(len(X), bool)
        live[n0:] = False
        versions = [(n_rows, live.copy())]
        for i in range(m):
            if i % 2 == 0:
                muts.append(("add", n_rows, n_rows + n_add))
                live[n_rows:n_rows + n_add] = True
                n_rows += n_add
            else:
                cand = np.nonzero(live[:n_rows])[0]
                dead = np.sort(rng.choice(cand, 1500, replace=False))
                muts.append(("del", dead))
                live[dead] = False
            versions.append((n_rows, live.copy()))
        done_v = [0]
        stop = threading.Event()
        errors = []
        records = {"small": [], "big": [], "one": []}

        def mutator():
            try:
                for mt in muts:
                    time.sleep(0.02)
                    if mt[0] == "add":
                        hip.LanceDetachedAddBatch(h, X[mt[1]:mt[2]], mt[2] - mt[1], D)
                    else:
                        hip.LanceDetachedDeleteBatch(h, mt[1])
                    done_v[0] += 1
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))
            finally:
                stop.set()

        def searcher(kind):
            try:
                while not stop.is_set() or len(records[kind]) < 3:
                    lo = done_v[0]
                    if kind == "one":
                        l, dd = hip.LanceDetachedSearch(h, Q1[0], D, K)
                        res = (np.full((1, K), -1, np.int64), np.full((1, K), np.nan, np.float32),
                               np.array([len(l)], np.int32))
                        res[0][0, :len(l)] = l
                        res[1][0, :len(l)] = dd
                    else:
                        res = hip.LanceDetachedSearchBatch(h, QS if kind == "small" else QB, K)
                    records[kind].append((lo, done_v[0], tuple(np.array(a) for a in res)))
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))

        threads = [threading.Thread(target=mutator)] + [threading.Thread(target=searcher, args=(kd,))
                                                       for kd in ("small", "big", "big", "one")]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=300)
            assert not t.is_alive(), "a thread hung"
        assert not errors, errors
        assert done_v[0] == m
        # the oracle of every version, per query set
        qsets = {"small": QS, "big": QB, "one": Q1}
        exp = {kd: [flat_knn.flat_search_batch(X[:nr], np.arange(nr), lv[:nr], qs, K)
                    for nr, lv in versions] for kd, qs in qsets.items()}
        n_checked, seen = 0, set()
        for kd, recs in records.items():
            assert recs, kd
            for lo, hi, res in recs:
                # the search ran against one version in [lo, hi + 1] (a mutation may
                # have completed inside the library before its thread bumped the counter)
                ok = [v for v in range(lo, min(hi + 1, m) + 1) if _matches(res, exp[kd][v])]
                assert ok, (kd, lo, hi)
                seen.add(ok[0])
                n_checked += 1
        assert n_checked >= 12
        assert len(seen) >= 2, seen  # the searches did interleave with the mutations
        # the final state, once more, synchronously
        nr, lv = versions[-1]
        assert hip.LanceDetachedCount(h) == int(lv[:nr].sum())
        assert_same(*hip.LanceDetachedSearchBatch(h, QB, K), *exp["big"][-1])
    finally:
        hip.LanceFreeDetached(h)


def test_two_handles_searched_in_parallel(hip):
    """Two indexes searched by two threads each, at the same time (each handle
    has its own stream and workspace; no state is shared between handles)."""
    rng = np.random.default_rng(7)
    XA = rng.standard_normal((90_000, D), dtype=np.float32)
    XB = rng.standard_normal((70_000, 256), dtype=np.float32)
    QA = rng.standard_normal((64, D), dtype=np.float32)
    QB = rng.standard_normal((300, 256), dtype=np.float32)
    ha = hip.LanceCreateDetached("", D, "l2", "a")
    hb = hip.LanceCreateDetached("", 256, "cosine", "b")
    try:
        hip.LanceDetachedAddBatch(ha, XA, len(XA), D)
        hip.LanceDetachedAddBatch(hb, XB, len(XB), 256)
        hip.LanceDetachedDeleteBatch(hb, np.arange(0, 70_000, 7))
        liveb = np.ones(len(XB), bool)
        liveb[::7] = False
        ea = flat_knn.flat_search_batch(XA, np.arange(len(XA)), np.ones(len(XA), bool), QA, K)
        eb = flat_knn.flat_search_batch(XB, np.arange(len(XB)), liveb, QB, 25, metric="cosine")
        errors, results = [], {"a": [], "b": []}

        def run(which):
            try:
                for _ in range(6):
                    if which == "a":
                        results["a"].append(tuple(np.array(x) for x in hip.LanceDetachedSearchBatch(ha, QA, K)))
                    else:
                        results["b"].append(tuple(np.array(x) for x in hip.LanceDetachedSearchBatch(hb, QB, 25)))
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))

        threads = [threading.Thread(target=run, args=(w,)) for w in ("a", "b", "a", "b")]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=300)
            assert not t.is_alive(), "a thread hung"
        assert not errors, errors
        assert len(results["a"]) == 12 and len(results["b"]) == 12
        for r in results["a"]:
            assert_same(*r, *ea)
        for r in results["b"]:
            assert_same(*r, *eb)
    finally:
        hip.LanceFreeDetached(ha)
        hip.LanceFreeDetached(hb)
