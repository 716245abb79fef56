"""GPU: a multi-device handle inside one process (shards.cpp).

With ``LANCE_HIP_DEVICES=0,1,...`` (or option ``devices``) a handle row-shards
its table over one store per listed device; DuckDB's unchanged calls
(``lance_search.cpp:73-74`` -> ``lance_index.cpp:452-453`` ->
``lance_detached_search``) then search every shard and merge the per-shard
top-k lists on the first device.  The box has one GPU, so the shards share
device 0 ("0,0"): every code path of the split (routing of ingest batches,
deletes on every shard, concurrent shard searches, peer copies of the partial
lists, the device merge, persistence, IVF) runs; only the copies stay on one
device.  Checker: the f64 oracle; bar as everywhere (labels bit-exact,
distances within 1e-4 relative)."""
import os

import numpy as np
import pytest

from oracle import c_oracle, flat_knn
from tests.test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def _sharded(hip, d, metric="l2", path="", devices="0,0", table="t"):
    h = hip.LanceCreateDetached(path, d, metric, table)
    hip.LanceHipSetOption(h, "devices", devices)
    return h


# "0,0": both shards on device 0 (every box); "0,1": two distinct devices — the
# peer copies really cross xGMI and the merge reads lists of another GPU (runs
# wherever two devices are visible; skipped on a one-GPU box)
DEVLISTS = ["0,0", "0,1"]


def _need(hip, devices):
    want = max(int(x) for x in devices.split(",")) + 1
    if hip.device_count() < want:
        pytest.skip(f"needs {want} HIP devices (box has {hip.device_count()})")


@pytest.mark.parametrize("devices", DEVLISTS)
@pytest.mark.parametrize("metric", ["l2", "cosine"])
def test_two_shards_d768_match_oracle(hip, metric, devices):
    # 2 x ~75k rows x 768 in DuckDB's 2048-row chunks (every shard on the
    # threshold path: sample pass, int8 scan8 append pass, pool_refine)
    _need(hip, devices)
    rng = np.random.default_rng(71)
    n, d, k = 150_000, 768, 10
    X = rng.standard_normal((n, d), dtype=np.float32)
    Q = rng.standard_normal((256, d), dtype=np.float32)
    h = _sharded(hip, d, metric, devices=devices)
    try:
        for lo in range(0, n, 2048):
            hi = min(n, lo + 2048)
            labs = hip.LanceDetachedAddBatch(h, X[lo:hi], hi - lo, d)
            assert labs.tolist() == list(range(lo, hi))
        assert hip.LanceDetachedCount(h) == n
        dead = rng.choice(n, 5000, replace=False)
        hip.LanceDetachedDeleteBatch(h, dead)
        live = np.ones(n, bool)
        live[dead] = False
        assert hip.LanceDetachedCount(h) == int(live.sum())
        el, ed, ec = c_oracle.flat_search_batch(X, Q, k, metric, live=live, acc64=True, nthreads=16)
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, k)
        assert_same(gl, gd, gc, el, ed, ec)
        st = hip.LanceHipLastSearchStats(h)
        assert st["fallback_queries"] == 0 and not st["dense_path"], st
        assert st["append_launches"] == 2, st  # one threshold scan per shard
        # one query per call (the lance_search() pattern)
        for i in (0, 7, 255):
            l, dd = hip.LanceDetachedSearch(h, Q[i], d, k)
            np.testing.assert_array_equal(l, el[i])
            np.testing.assert_allclose(dd, ed[i], rtol=1e-4, atol=1e-5)
        # k = 100 (past one shard's k = 10 lists: the merge keeps 100 of 200)
        el2, ed2, ec2 = c_oracle.flat_search_batch(X, Q[:32], 100, metric, live=live, acc64=True, nthreads=16)
        assert_same(*hip.LanceDetachedSearchBatch(h, Q[:32], 100), el2, ed2, ec2)
        # the vectors come back from whichever shard holds them
        for lab in (0, 2048, 149_999):
            if live[lab]:
                np.testing.assert_array_equal(hip.LanceDetachedGetVector(h, lab, d), X[lab])
        with pytest.raises(hip.IOException, match="not found"):
            hip.LanceDetachedGetVector(h, int(dead[0]), d)
    finally:
        hip.LanceFreeDetached(h)


def test_device_api_and_compaction_on_two_shards(hip):
    import torch

    L = hip.lib()
    rng = np.random.default_rng(72)
    n, d, k = 140_000, 256, 10
    X = rng.standard_normal((n, d), dtype=np.float32)
    Q = rng.standard_normal((300, d), dtype=np.float32)
    h = _sharded(hip, d)
    e = hip._err()
    try:
        Xd = torch.from_numpy(X).cuda()
        for lo in range(0, n, 35_000):
            assert L.lance_hip_add_batch_device(h, Xd[lo:lo + 35_000].data_ptr(), 35_000, d, e, len(e)) == lo, e.value
        hip.LanceDetachedDeleteBatch(h, np.arange(0, n, 3))
        live = np.ones(n, bool)
        live[::3] = False
        el, ed, ec = c_oracle.flat_search_batch(X, Q, k, "l2", live=live, acc64=True, nthreads=16)
        from lance_hip.sharded import AsyncPipeline, hip_device_search

        Qd = torch.from_numpy(Q).cuda()
        got = hip_device_search(L, h, d)(Qd, k)
        assert_same(*(x.cpu().numpy() for x in got), el, ed, ec)
        pipe = AsyncPipeline(L, h, d)  # (two sharded searches in flight; merged at the wait)
        t = pipe.submit(Qd, k)
        assert_same(*(x.cpu().numpy() for x in pipe.wait(t)), el, ed, ec)
        hip.LanceDetachedCompact(h)
        assert hip.LanceDetachedCount(h) == int(live.sum())
        assert_same(*hip.LanceDetachedSearchBatch(h, Q, k), el, ed, ec)
        labs, vecs = hip.LanceDetachedGetAllVectors(h)
        np.testing.assert_array_equal(labs, np.nonzero(live)[0])
        np.testing.assert_array_equal(vecs, X[live])
        # a new batch after compaction keeps dense labels
        assert hip.LanceDetachedAddBatch(h, X[:5], 5, d).tolist() == list(range(n, n + 5))
    finally:
        hip.LanceFreeDetached(h)


def test_two_shards_persist_and_reopen_from_environment(hip, tmp_path):
    # LANCE_HIP_DEVICES is how a DuckDB process asks for it (no per-call option channel)
    rng = np.random.default_rng(73)
    n, d, k = 20_000, 64, 5
    X = rng.standard_normal((n, d), dtype=np.float32)
    Q = rng.standard_normal((16, d), dtype=np.float32)
    old = os.environ.get("LANCE_HIP_DEVICES")
    os.environ["LANCE_HIP_DEVICES"] = "0,0"
    try:
        h = hip.LanceCreateDetached(str(tmp_path), d, "dot", "v")
        for lo in range(0, n, 2048):
            hi = min(n, lo + 2048)
            hip.LanceDetachedAddBatch(h, X[lo:hi], hi - lo, d)
        hip.LanceDetachedDeleteBatch(h, [1, 5, 19_999])
        before = hip.LanceDetachedSearchBatch(h, Q, k)
        hip.LanceFreeDetached(h)
        h = hip.LanceOpenDetached(str(tmp_path), "v", "dot")
        live = np.ones(n, bool)
        live[[1, 5, 19_999]] = False
        el, ed, ec = flat_knn.flat_search_batch(X, np.arange(n), live, Q, k, metric="dot")
        after = hip.LanceDetachedSearchBatch(h, Q, k)
        assert_same(*before, el, ed, ec)
        assert_same(*after, el, ed, ec)
        # next_label = max(live label) + 1 (lance_manager.rs:157-158): 19_999 was deleted
        assert hip.LanceDetachedAdd(h, X[0], d) == 19_999
        hip.LanceFreeDetached(h)
        # the same log opens as a single-store handle too
        del os.environ["LANCE_HIP_DEVICES"]
        h = hip.LanceOpenDetached(str(tmp_path), "v", "dot")
        live = np.concatenate([live, [True]])
        X2 = np.concatenate([X, X[:1]])
        el, ed, ec = flat_knn.flat_search_batch(X2, np.arange(n + 1), live, Q, k, metric="dot")
        assert_same(*hip.LanceDetachedSearchBatch(h, Q, k), el, ed, ec)
        hip.LanceFreeDetached(h)
    finally:
        if old is None:
            os.environ.pop("LANCE_HIP_DEVICES", None)
        else:
            os.environ["LANCE_HIP_DEVICES"] = old


def test_ivf_flat_model_on_two_shards_equals_one_store(hip):
    # the same IVF_FLAT model on a single store and on two shards: the bound scan
    # is exact within the probed lists, so both must return the same lists
    rng = np.random.default_rng(74)
    n, d, k, nlist = 60_000, 128, 10, 64
    centers = rng.standard_normal((nlist, d)).astype(np.float32) * 3
    X = (centers[rng.integers(0, nlist, n)] + rng.standard_normal((n, d))).astype(np.float32)
    Q = (centers[rng.integers(0, nlist, 64)] + rng.standard_normal((64, d))).astype(np.float32)
    h1 = hip.LanceCreateDetached("", d, "l2", "one")
    h2 = _sharded(hip, d)
    try:
        for h in (h1, h2):
            hip.LanceHipSetOption(h, "index_type", "ivf_flat")
            for lo in range(0, n, 4096):
                hi = min(n, lo + 4096)
                hip.LanceDetachedAddBatch(h, X[lo:hi], hi - lo, d)
        hip.LanceDetachedCreateIndex(h1, nlist, 0)
        m = hip.LanceHipIvfExport(h1)
        hip.LanceHipIvfSetModel(h2, "ivf_flat", m["centroids"])
        info = hip.LanceHipIvfInfo(h2)
        assert info["type"] == "ivf_flat" and info["n_indexed"] == n, info
        for nprobes in (4, 16):
            g1 = hip.LanceDetachedSearchBatch(h1, Q, k, nprobes=nprobes)
            g2 = hip.LanceDetachedSearchBatch(h2, Q, k, nprobes=nprobes)
            assert_same(*g2, *g1)
        # and create_index on the multi-device handle itself trains once, installs everywhere
        hip.LanceDetachedCreateIndex(h2, nlist, 0)
        info = hip.LanceHipIvfInfo(h2)
        assert info["type"] == "ivf_flat" and info["n_indexed"] == n, info
        el, ed, ec = c_oracle.flat_search_batch(X, Q, k, "l2", acc64=True, nthreads=16)
        gl, gd, gc = hip.LanceDetachedSearchBatch(h2, Q, k, nprobes=nlist)  # every list probed: exact
        assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h1)
        hip.LanceFreeDetached(h2)


def test_devices_option_errors(hip):
    h = hip.LanceCreateDetached("", 8, "l2", "t")
    try:
        with pytest.raises(hip.IOException, match="at least two"):
            hip.LanceHipSetOption(h, "devices", "0")
        with pytest.raises(hip.IOException, match="out of range"):
            hip.LanceHipSetOption(h, "devices", "0,1000")
        hip.LanceDetachedAddBatch(h, np.ones((3, 8), np.float32), 3, 8)
        with pytest.raises(hip.IOException, match="empty table"):
            hip.LanceHipSetOption(h, "devices", "0,0")
    finally:
        hip.LanceFreeDetached(h)


@pytest.mark.parametrize("devices", DEVLISTS)
def test_async_sharded_searches_in_flight(hip, devices):
    """lance_hip_search_batch_device_async on a multi-device handle keeps two
    searches in flight (every shard's pass enqueued at the submit; certificates,
    peer copies and the merge at the wait): three batches submitted back to back
    (the third completes the first), each equal to the oracle and to the
    synchronous call; statistics count only the shards that searched."""
    import torch
    from lance_hip.sharded import AsyncPipeline

    _need(hip, devices)
    L = hip.lib()
    rng = np.random.default_rng(76)
    n, d, k = 160_000, 256, 10
    X = rng.standard_normal((n, d), dtype=np.float32)
    Qs = [rng.standard_normal((nq, d), dtype=np.float32) for nq in (256, 100, 256)]
    h = _sharded(hip, d, devices=devices)
    try:
        for lo in range(0, n, 40_000):
            hip.LanceDetachedAddBatch(h, X[lo:lo + 40_000], 40_000, d)
        exp = [c_oracle.flat_search_batch(X, q, k, "l2", acc64=True, nthreads=16) for q in Qs]
        pipe = AsyncPipeline(L, h, d)
        Qd = [torch.from_numpy(q).cuda() for q in Qs]
        t = [pipe.submit(q, k) for q in Qd[:2]]
        t.append(pipe.submit(Qd[2], k))  # (a third submit completes the oldest first)
        out = {}
        for ti in t:
            r = pipe.wait(ti)
            out[ti] = tuple(x.cpu().numpy().copy() for x in r)
        for ti, e in zip(t, exp):
            assert_same(*out[ti], *e)
        st = hip.LanceHipLastSearchStats(h)
        assert st["fallback_queries"] == 0 and st["append_launches"] == 2, st
        sync = hip.LanceDetachedSearchBatch(h, Qs[0], k)
        np.testing.assert_array_equal(sync[0], out[t[0]][0])
    finally:
        hip.LanceFreeDetached(h)


def test_options_before_devices_reach_every_shard(hip):
    """Options set on a handle before `devices` are replayed on each shard (the
    round-5 shard_init copied only the table's own settings): here the tie rule
    and the int8 scan switch."""
    rng = np.random.default_rng(77)
    n, d, k = 100_000, 32, 10
    X = np.ones((n, d), np.float32)  # every row ties: the tie rule alone orders them
    h = hip.LanceCreateDetached("", d, "l2", "t")
    try:
        hip.LanceHipSetOption(h, "tie", "label_asc")
        hip.LanceHipSetOption(h, "scan_i8", "off")
        hip.LanceHipSetOption(h, "devices", "0,0")
        for lo in range(0, n, 25_000):
            hip.LanceDetachedAddBatch(h, X[lo:lo + 25_000], 25_000, d)
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, np.ones((2, d), np.float32), k)
        assert list(gl[0]) == list(range(k))
        kt = hip.LanceHipKernelTimes(h)
        assert kt["scan_elem_bytes"] != 1  # scan_i8 off on the shards: no int8 scan
    finally:
        hip.LanceFreeDetached(h)


@pytest.mark.parametrize("index_type", ["ivf_flat", "ivf_pq"])
def test_ivf_defaults_from_the_whole_table(hip, index_type):
    """create_index on a multi-device handle resolves nlist / m from the table's
    live count (the model a single store of the same rows gets), and a table one
    store can index is indexable on two shards even when no single shard could
    train it alone (IVF_PQ needs 256 rows: 2 x 150 here)."""
    rng = np.random.default_rng(78)
    d = 64
    for n, parts in ((40_000, 0), (300, 4)):
        X = rng.standard_normal((n, d)).astype(np.float32)
        h1 = hip.LanceCreateDetached("", d, "l2", "one")
        h2 = _sharded(hip, d)
        try:
            for h in (h1, h2):
                hip.LanceHipSetOption(h, "index_type", index_type)
                for lo in range(0, n, 2048 if n > 2048 else 150):
                    hi = min(n, lo + (2048 if n > 2048 else 150))
                    hip.LanceDetachedAddBatch(h, X[lo:hi], hi - lo, d)
                hip.LanceDetachedCreateIndex(h, parts, 0)
            i1, i2 = hip.LanceHipIvfInfo(h1), hip.LanceHipIvfInfo(h2)
            assert i2["type"] == index_type and i2["n_indexed"] == n, i2
            assert (i1["nlist"], i1["m"]) == (i2["nlist"], i2["m"]), (i1, i2)
            gl, gd, gc = hip.LanceDetachedSearchBatch(h2, X[:8], 5, nprobes=i2["nlist"], refine_factor=50)
            assert list(gl[:, 0]) == list(range(8))  # each row finds itself
        finally:
            hip.LanceFreeDetached(h1)
            hip.LanceFreeDetached(h2)
