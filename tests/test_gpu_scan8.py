"""GPU parity of scan8_kernel, the int8 append pass (scan8_kernels.hip,
DESIGN.md §3): query halves resident in LDS, rows streamed into registers, the
bound screened in exact integers against per-tile / per-batch scales, then the
pool refined in bound order until certified (pool_refine_kernel).  Results must
equal the f64 oracle exactly (labels bit-exact, distances within 1e-4 relative;
reference semantics lance_manager.rs:393-451, squared L2 / 1 - x.q / cosine).

Covers every ld the kernel is instantiated for, the three metrics, the
distributions where common scales are worst (the CPU restatement
tests/test_i8_bound_cpu.py checks the same algebra in f64), in-place appends
into partly filled tiles (the tile scale grows), zero rows, deletes, every
query-batch geometry (one tile split into halves, a small batch on every
workgroup, several tiles) and the C2 configuration at full size."""
import numpy as np
import pytest

from oracle import c_oracle, flat_knn
from tests.test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def _mk(hip, tmp_path, d, metric):
    h = hip.LanceCreateDetached(str(tmp_path), d, metric, "t")
    hip.LanceHipSetOption(h, "scan_i8", "on")
    hip.LanceHipSetOption(h, "time_kernels", "1")
    return h


def _ran_scan8(hip, h):
    kt = hip.LanceHipKernelTimes(h)
    return kt["scan_elem_bytes"] == 1 and kt["scan_kernel"] == "scan8_kernel"


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
@pytest.mark.parametrize("d", [512, 600, 768, 896, 1000])  # ld 512, 640, 768, 896, 1024
def test_scan8_every_ld(hip, tmp_path, d, metric):
    rng = np.random.default_rng(d)
    n = 80_000
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((300, d)).astype(np.float32)  # a split tile + a small one
    h = _mk(hip, tmp_path, d, metric)
    try:
        hip.LanceDetachedAddBatch(h, X, n, d)
        dead = rng.choice(n, 4_000, replace=False)
        hip.LanceDetachedDeleteBatch(h, dead)
        live = np.ones(n, bool)
        live[dead] = False
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        assert _ran_scan8(hip, h)
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, metric, live=live, acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
        assert hip.LanceHipLastSearchStats(h)["fallback_queries"] <= 3
    finally:
        hip.LanceFreeDetached(h)


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
@pytest.mark.parametrize("d", [512, 600, 768, 896, 1000])
def test_scan8_small_batch_every_ld(hip, tmp_path, d, metric):
    # at most 16 queries (no halves: every workgroup its own row group, the
    # padding queries of its 128 pass nothing) for the sample and the append
    # pass; deletes, k = 1, 10 and 100 (a deeper pool per query), one query
    # (lance_search's pattern)
    rng = np.random.default_rng(1000 + d)
    n = 75_000
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((16, d)).astype(np.float32)
    h = _mk(hip, tmp_path, d, metric)
    try:
        hip.LanceDetachedAddBatch(h, X, n, d)
        dead = rng.choice(n, 3_000, replace=False)
        hip.LanceDetachedDeleteBatch(h, dead)
        live = np.ones(n, bool)
        live[dead] = False
        for nq, k in ((16, 10), (16, 100), (1, 10), (5, 1)):
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q[:nq], k)
            assert _ran_scan8(hip, h)
            el, ed, ec = c_oracle.flat_search_batch(X, Q[:nq], k, metric, live=live, acc64=True, nthreads=16)
            assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)


def _datasets(rng, n, d):
    yield "heavy", rng.standard_cauchy((n, d)).clip(-1e4, 1e4).astype(np.float32)
    spike = rng.standard_normal((n, d)).astype(np.float32) * 1e-3
    spike[np.arange(n), rng.integers(0, d, n)] = 50.0
    yield "spike", spike
    yield "near_const", (3.0 + 1e-4 * rng.standard_normal((n, d))).astype(np.float32)
    yield "tiny", (1e-15 * rng.standard_normal((n, d))).astype(np.float32)
    yield "huge", (1e15 * rng.standard_normal((n, d))).astype(np.float32)
    yield "sparse_int", rng.integers(-3, 4, (n, d)).astype(np.float32)
    mixed = rng.standard_normal((n, d)).astype(np.float32)
    mixed[rng.random(n) < 0.5] *= 100.0  # two norm scales inside every tile
    yield "mixed_norms", mixed


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
def test_scan8_adversarial_distributions(hip, tmp_path, metric):
    # the distributions tests/test_i8_bound_cpu.py pins in f64, end to end at d = 768
    rng = np.random.default_rng(99)
    n, d = 70_000, 768
    for name, X in _datasets(rng, n, d):
        Q = np.concatenate([X[:32] + np.float32(0.01) * np.abs(X[:32]).max() * rng.standard_normal((32, d)).astype(np.float32),
                            rng.standard_normal((32, d)).astype(np.float32) * np.abs(X).max()])
        h = _mk(hip, tmp_path, d, metric)
        try:
            hip.LanceDetachedAddBatch(h, X, n, d)
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
            assert _ran_scan8(hip, h), name
            el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, metric, acc64=True, nthreads=16)
            assert_same(gl, gd, gc, el, ed, ec)
        finally:
            hip.LanceFreeDetached(h)


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
def test_scan8_incremental_append_and_delete(hip, tmp_path, metric):
    # appends into a partly filled tile re-quantise it (its scale grows with
    # larger rows); rows of smaller norm keep it; zero rows (cosine: undefined,
    # exact fallback) and deletes update the copy in place
    rng = np.random.default_rng(4321)
    d = 768
    X = rng.standard_normal((110_000, d)).astype(np.float32)
    X[90_000:100_000] *= 4.0    # larger norms: tile scales grow
    X[100_000:] *= 0.25         # smaller norms: scales unchanged
    X[100_500:100_510] = 0.0    # zero rows
    Q = rng.standard_normal((40, d)).astype(np.float32)
    h = _mk(hip, tmp_path, d, metric)
    try:
        hip.LanceHipSetOption(h, "reserve_rows", "131072")
        live = np.zeros(len(X), bool)
        for lo, hi in ((0, 70_100), (70_100, 90_000), (90_000, 100_000), (100_000, 110_000)):
            hip.LanceDetachedAddBatch(h, X[lo:hi], hi - lo, d)
            live[lo:hi] = True
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
            el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, metric, live=live, acc64=True, nthreads=16)
            assert_same(gl, gd, gc, el, ed, ec)
            dead = np.unique(el[:, :3])
            hip.LanceDetachedDeleteBatch(h, dead)
            live[dead] = False
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
            el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, metric, live=live, acc64=True, nthreads=16)
            assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)


@pytest.mark.parametrize("nq", [1, 7, 128, 129, 256, 257, 700])
def test_scan8_query_batches(hip, tmp_path, nq):
    # one workgroup per half of a tile (> 128 queries in it) or all workgroups on
    # one half (<= 128), several tiles per launch
    rng = np.random.default_rng(nq)
    n, d = 90_000, 768
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((nq, d)).astype(np.float32)
    h = _mk(hip, tmp_path, d, "l2")
    try:
        hip.LanceDetachedAddBatch(h, X, n, d)
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, "l2", acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)


def test_scan8_zero_cosine_query_and_k_edges(hip, tmp_path):
    rng = np.random.default_rng(3)
    n, d = 70_000, 768
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((6, d)).astype(np.float32)
    Q[2] = 0.0
    h = _mk(hip, tmp_path, d, "cosine")
    try:
        hip.LanceDetachedAddBatch(h, X, n, d)
        for k in (1, 32):
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, k)
            el, ed, ec = flat_knn.flat_search_batch(X, np.arange(n), np.ones(n, bool), Q, k, metric="cosine")
            for i in (0, 1, 3, 4, 5):
                assert gc[i] == ec[i]
                np.testing.assert_array_equal(gl[i], el[i])
    finally:
        hip.LanceFreeDetached(h)


def test_c2_full_size(hip, tmp_path):
    # BASELINE.json configs[1] at its own size: 1M x 768 f32, k = 10, 256 queries,
    # every query against the f64 oracle
    rng = np.random.default_rng(20260)
    n, d = 1_000_000, 768
    X = rng.standard_normal((n, d), dtype=np.float32)
    Q = rng.standard_normal((256, d), dtype=np.float32)
    h = _mk(hip, tmp_path, d, "l2")
    try:
        for lo in range(0, n, 250_000):
            hip.LanceDetachedAddBatch(h, X[lo:lo + 250_000], 250_000, d)
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        assert _ran_scan8(hip, h)
        st = hip.LanceHipLastSearchStats(h)
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, "l2", acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
        assert st["fallback_queries"] == 0, st
    finally:
        hip.LanceFreeDetached(h)


@pytest.mark.parametrize("metric", ["dot", "l2"])
def test_bf16_store_k100_int8(hip, tmp_path, metric):
    # C3's shape at reduced size (configs[2]: a bf16 store, L2-normalised rows,
    # inner product, k = 100): the int8 copy is built from the bf16 rows, the
    # pools of the first pass exceed pool_refine's LDS capacity (the smallest
    # bounds are kept, the rest bounds the certificate) and every query must
    # still certify without a rerun; ids exact against the f64 oracle on the
    # stored (bf16-rounded) rows
    import torch
    rng = np.random.default_rng(100)
    n, d = 400_000, 768
    X = rng.standard_normal((n, d), dtype=np.float32)
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    Q = rng.standard_normal((96, d), dtype=np.float32)
    Q /= np.linalg.norm(Q, axis=1, keepdims=True)
    Xs = torch.from_numpy(X).to(torch.bfloat16).float().numpy()  # what a bf16 store holds
    h = hip.LanceCreateDetached(str(tmp_path), d, metric, "t")
    try:
        hip.LanceHipSetOption(h, "storage", "bf16")
        hip.LanceHipSetOption(h, "time_kernels", "1")
        for lo in range(0, n, 100_000):
            hip.LanceDetachedAddBatch(h, X[lo:lo + 100_000], 100_000, d)
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 100)
        assert _ran_scan8(hip, h)
        st = hip.LanceHipLastSearchStats(h)
        el, ed, ec = c_oracle.flat_search_batch(Xs, Q, 100, metric, acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
        assert st["fallback_queries"] == 0, st
        assert st["retried_queries"] == 0, st
    finally:
        hip.LanceFreeDetached(h)


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
def test_split_div_progressive_threshold(hip, metric):
    """Option split_div (progressive threshold, lance_hip_abi.cpp search_chunk):
    the first 1/8 of the tiles with the sample's tau, their pool refined in tau
    mode (tau' = min(tau, k-th exact distance)), the other 7/8 with tau' into a
    disjoint segment range, the final certificate against tau'.  Two scan8
    launches must run, and the results must equal the one-pass search and the
    f64 oracle for k = 10 and k = 100."""
    rng = np.random.default_rng(77)
    n, d = 262_144, 768  # 1024 tiles = 128 * split_div
    X = rng.standard_normal((n, d), dtype=np.float32)
    Q = rng.standard_normal((256, d), dtype=np.float32)
    h = hip.LanceCreateDetached("", d, metric, "t")
    try:
        hip.LanceHipSetOption(h, "time_kernels", "1")
        for lo in range(0, n, 131_072):
            hip.LanceDetachedAddBatch(h, X[lo:lo + 131_072], 131_072, d)
        for k in (10, 100):
            el, ed, ec = c_oracle.flat_search_batch(X, Q, k, metric, acc64=True, nthreads=16)
            hip.LanceHipSetOption(h, "split_div", "0")
            g1 = hip.LanceDetachedSearchBatch(h, Q, k)
            assert hip.LanceHipLastSearchStats(h)["append_launches"] == 1
            hip.LanceHipSetOption(h, "split_div", "8")
            g8 = hip.LanceDetachedSearchBatch(h, Q, k)
            st = hip.LanceHipLastSearchStats(h)
            assert _ran_scan8(hip, h)
            assert st["append_launches"] == 2, st
            assert st["fallback_queries"] == 0, st
            assert_same(*g8, el, ed, ec)
            assert_same(*g1, el, ed, ec)
            np.testing.assert_array_equal(g8[0], g1[0])
            np.testing.assert_array_equal(g8[1], g1[1])
    finally:
        hip.LanceFreeDetached(h)


def test_release_build_rejects_development_knobs(hip):
    """The wrong-result scan8 timing ablations are not in a release build:
    option scan8_variant accepts only the default geometry; pr_first is a
    per-handle value, range-checked, and leaves the results unchanged."""
    rng = np.random.default_rng(5)
    n, d = 70_000, 768
    X = rng.standard_normal((n, d), dtype=np.float32)
    Q = rng.standard_normal((64, d), dtype=np.float32)
    h = hip.LanceCreateDetached("", d, "l2", "t")
    h2 = hip.LanceCreateDetached("", d, "l2", "t2")
    try:
        for v in ("1", "6", "21", "22", "24", "28", "34", "-1"):
            with pytest.raises(hip.IOException):
                hip.LanceHipSetOption(h, "scan8_variant", v)
        hip.LanceHipSetOption(h, "scan8_variant", "0")
        for v in ("4", "2000", "-3"):
            with pytest.raises(hip.IOException):
                hip.LanceHipSetOption(h, "pr_first", v)
        hip.LanceDetachedAddBatch(h, X, n, d)
        hip.LanceDetachedAddBatch(h2, X, n, d)
        hip.LanceHipSetOption(h, "pr_first", "8")  # this handle only
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, "l2", acc64=True, nthreads=16)
        assert_same(*hip.LanceDetachedSearchBatch(h, Q, 10), el, ed, ec)
        assert_same(*hip.LanceDetachedSearchBatch(h2, Q, 10), el, ed, ec)
    finally:
        hip.LanceFreeDetached(h)
        hip.LanceFreeDetached(h2)


def test_async_submit_orders_after_torch_stream(hip):
    """AsyncPipeline.submit with torch's stream still busy: the queries are
    written there (behind a long chain of matmuls) right before the submit, and
    lance_hip_stream_after orders the search after that work on the device (no
    host wait): the results are those of the new queries, every time."""
    import torch
    from lance_hip.sharded import AsyncPipeline

    rng = np.random.default_rng(43)
    n, d, k = 100_000, 768, 10
    X = rng.standard_normal((n, d), dtype=np.float32)
    Qa = rng.standard_normal((256, d), dtype=np.float32)
    Qb = rng.standard_normal((256, d), dtype=np.float32)
    ea = c_oracle.flat_search_batch(X, Qa, k, "l2", acc64=True, nthreads=16)
    eb = c_oracle.flat_search_batch(X, Qb, k, "l2", acc64=True, nthreads=16)
    h = hip.LanceCreateDetached("", d, "l2", "t")
    try:
        hip.LanceDetachedAddBatch(h, X, n, d)
        pipe = AsyncPipeline(hip.lib(), h, d)
        Q = torch.from_numpy(Qa).cuda()
        srcs = [torch.from_numpy(Qb).cuda(), torch.from_numpy(Qa).cuda()]
        M = torch.randn((4096, 4096), device="cuda")
        torch.cuda.synchronize()
        outs = []
        for i in range(4):
            for _ in range(6):  # keep torch's stream busy for milliseconds
                M = torch.tanh(M @ M * 1e-3)
            Q.copy_(srcs[i % 2])  # the batch's queries, written on torch's stream
            assert not torch.cuda.current_stream().query()
            t = pipe.submit(Q, k)
            o = pipe.wait(t)
            outs.append(tuple(x.cpu().numpy() for x in o))
        for i, r in enumerate(outs):
            assert_same(*r, *(eb if i % 2 == 0 else ea))
    finally:
        hip.LanceFreeDetached(h)


def test_async_pipeline_matches_sync(hip):
    """lance_hip_search_batch_device_async / lance_hip_search_wait: two batches
    in flight per handle (the second pass enqueued while the first is on the
    device, each with its own query / status buffers), a third submit completes
    the oldest, a mutation completes every pending search before it changes the
    store; every batch's results equal the synchronous search and the oracle."""
    import torch
    from lance_hip.sharded import AsyncPipeline, hip_device_search

    rng = np.random.default_rng(42)
    n, d, k = 120_000, 768, 10
    X = rng.standard_normal((n, d), dtype=np.float32)
    Qs = [rng.standard_normal((nq, d), dtype=np.float32) for nq in (256, 300, 17, 256)]
    h = hip.LanceCreateDetached("", d, "l2", "t")
    try:
        hip.LanceDetachedAddBatch(h, X[:100_000], 100_000, d)
        L = hip.lib()
        pipe = AsyncPipeline(L, h, d)
        sync = hip_device_search(L, h, d)
        Qd = [torch.from_numpy(q).cuda() for q in Qs]
        exp = [c_oracle.flat_search_batch(X[:100_000], q, k, "l2", acc64=True, nthreads=16) for q in Qs]
        t = [pipe.submit(Qd[i], k) for i in range(3)]  # the third submit completes the first
        assert t[0] < t[1] < t[2]
        outs = {}
        o = pipe.wait(t[1])  # completes batches 0 (already finished inside the third submit) and 1
        assert set(pipe.completed) == {t[0], t[1]} and o is pipe.completed[t[1]]
        outs[0] = tuple(x.cpu().numpy() for x in pipe.completed[t[0]])
        outs[1] = tuple(x.cpu().numpy() for x in o)
        outs[2] = tuple(x.cpu().numpy() for x in pipe.wait(t[2]))
        for i in (0, 1, 2):
            assert_same(*outs[i], *exp[i])
        # a pending search, then an append: the append first completes it
        t3 = pipe.submit(Qd[3], k)
        o3 = pipe.pending[-1][1]
        hip.LanceDetachedAddBatch(h, X[100_000:], n - 100_000, d)
        pipe.wait(t3)
        assert_same(*(x.cpu().numpy() for x in o3), *exp[3])
        # after the append: pipelined steps over the whole store, a different batch
        # each step (outputs copied out before the next-but-one submit reuses them)
        e0 = c_oracle.flat_search_batch(X, Qs[0], k, "l2", acc64=True, nthreads=16)
        Qr = Qd[0].flip(0).contiguous()
        er = tuple(a[::-1] for a in e0)
        steps = [Qd[0], Qr, Qd[0], Qr, Qd[0]]
        got = []
        for Qi in steps:
            r = pipe.step(Qi, k)
            if r is not None:
                got.append(tuple(x.cpu().numpy() for x in r))
        got.append(tuple(x.cpu().numpy() for x in pipe.drain()))
        assert len(got) == len(steps)
        for i, r in enumerate(got):
            assert_same(*r, *(e0 if i % 2 == 0 else er))
        assert_same(*(x.cpu().numpy() for x in sync(Qd[0], k)), *e0)
        st = hip.LanceHipLastSearchStats(h)
        assert st["fallback_queries"] == 0 and st["append_launches"] == 1, st
    finally:
        hip.LanceFreeDetached(h)


def test_async_rerun_and_fallback_with_next_pass_in_flight(hip):
    """pass A's completion (reruns of uncertified queries and the
    exact fallback, lance_hip_abi.cpp finish_chunk) runs while pass B is still
    queued behind it on the handle's stream and shares the workspace (segment
    pools, rerun / fallback buffers).  Cosine store; A holds three queries whose
    neighbours sit packed in a tile the sample pass skips (their first pass
    overflows a segment: rerun), one query equal to 200 duplicate rows and one
    zero query (NaN distances: the exact fallback); B and C are plain batches,
    C enqueued into A's pass buffers while B is pending.  Every batch equals the
    f64 oracle, A's statistics equal those of the same batch run synchronously
    (reruns and a fallback), and pass B really was in flight during A's wait."""
    import torch
    from lance_hip.sharded import AsyncPipeline

    rng = np.random.default_rng(505)
    n, d, k = 120_000, 128, 10
    X = rng.standard_normal((n, d), dtype=np.float32)
    q0 = rng.standard_normal(d).astype(np.float32)
    dirs = rng.standard_normal((256, d))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    X[256:512] = q0 + np.sqrt(rng.uniform(0, 60, 256))[:, None] * dirs
    q1 = rng.standard_normal(d).astype(np.float32)
    X[1000:1200] = q1
    ZERO = 4
    QA = np.concatenate([q0 + 0.01 * rng.standard_normal((3, d)), q1[None, :], np.zeros((1, d)),
                         rng.standard_normal((60, d))]).astype(np.float32)
    QB = rng.standard_normal((256, d), dtype=np.float32)
    QC = rng.standard_normal((40, d), dtype=np.float32)
    keep = np.arange(len(QA)) != ZERO
    h = hip.LanceCreateDetached("", d, "cosine", "t")
    try:
        hip.LanceDetachedAddBatch(h, X, n, d)
        hip.LanceHipSetOption(h, "sample_div", "100000")  # the sample skips tile 1
        exp = [c_oracle.flat_search_batch(X, q, k, "cosine", acc64=True, nthreads=16) for q in (QA[keep], QB, QC)]
        sync = hip.LanceDetachedSearchBatch(h, QA, k)
        stS = hip.LanceHipLastSearchStats(h)
        assert stS["retried_queries"] >= 1 and stS["fallback_queries"] >= 1, stS
        assert_same(*hip.LanceDetachedSearchBatch(h, QB, k), *exp[1])  # (workspace sized for B: no drain at its submit)
        pipe = AsyncPipeline(hip.lib(), h, d)
        tA = pipe.submit(torch.from_numpy(QA).cuda(), k)
        tB = pipe.submit(torch.from_numpy(QB).cuda(), k)  # B queued behind A
        oA = tuple(x.cpu().numpy() for x in pipe.wait(tA))  # A's reruns + fallback, B still in flight
        stA = hip.LanceHipLastSearchStats(h)
        tC = pipe.submit(torch.from_numpy(QC).cuda(), k)  # C takes A's pass buffers while B is pending
        oB = tuple(x.cpu().numpy() for x in pipe.wait(tB))
        oC = tuple(x.cpu().numpy() for x in pipe.wait(tC))
        stC = hip.LanceHipLastSearchStats(h)
        assert stA == stS, (stA, stS)
        assert stC["fallback_queries"] == 0, stC
        for got in (sync, oA):
            assert_same(got[0][keep], got[1][keep], got[2][keep], *exp[0])
            assert got[2][ZERO] == k
            # 200 duplicates at distance 0: the default tie rule (label descending) keeps the last ten
            assert list(got[0][3]) == list(range(1199, 1189, -1)) and (np.abs(got[1][3]) < 1e-6).all()
        assert_same(*oB, *exp[1])
        assert_same(*oC, *exp[2])
    finally:
        hip.LanceFreeDetached(h)


@pytest.mark.parametrize("couple", ["1", "8", "64"])
def test_scan8_pair_coupling_is_exact(hip, tmp_path, couple):
    # option s8_couple (speed only): the workgroups of a pair wait for each
    # other's progress; results must not change.  300k rows x 256 queries: 256
    # workgroups in pairs (b, b ^ 8), two append launches (split_div) and the
    # tilemin sample pass, each with its own coupling epoch
    rng = np.random.default_rng(7070)
    n, d = 300_000, 768
    X = rng.standard_normal((n, d), dtype=np.float32)
    Q = rng.standard_normal((256, d), dtype=np.float32)
    h = _mk(hip, tmp_path, d, "l2")
    try:
        hip.LanceDetachedAddBatch(h, X, n, d)
        hip.LanceHipSetOption(h, "s8_couple", couple)
        hip.LanceHipSetOption(h, "split_div", "4")
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, 10)
        assert _ran_scan8(hip, h)
        el, ed, ec = c_oracle.flat_search_batch(X, Q, 10, "l2", acc64=True, nthreads=16)
        assert_same(gl, gd, gc, el, ed, ec)
        for _ in range(3):  # repeated launches: fresh epochs over the same progress words
            gl2, _, _ = hip.LanceDetachedSearchBatch(h, Q, 10)
            np.testing.assert_array_equal(gl2, gl)
    finally:
        hip.LanceFreeDetached(h)
