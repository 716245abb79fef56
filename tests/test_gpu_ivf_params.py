"""GPU parity of IVF_FLAT / IVF_PQ at the BASELINE.json C4 / C5 parameters
(nlist = 4096, nprobe = 64, IVF_PQ m = 96 nbits = 8, d = 768, k = 10, a batch
of 256 queries) on a reduced per-GPU shard of 1M clustered rows (the configs'
100M rows over 8 GPUs are 12.5M per GPU; the list count, probe count, code
width and dimension — what the kernels are specialised on — are the configs').

Reference: rust_lib/src/lance_manager.rs:411-419 (vector_search .nprobes
.refine_factor) and :483-515 (IVF_PQ build).  Checker: oracle/flat_knn.c's IVF
port (f64-accumulated exact distances; f32 ADC sums in the canonical order of
oracle/ivf.py, no fused multiply-add: the C file is built as ISO C11) over the
model and row layout the library exports — labels bit-exact, distances within
1e-4 relative.  Parity with LanceDB itself is unpinned for IVF (no reference
test builds an IVF index); recall is measured against the exact
flat search instead.
"""
import numpy as np
import pytest

from oracle import c_oracle, flat_knn, ivf

pytestmark = pytest.mark.gpu

N, D, NLIST, NPROBE, M, K, B = 1_000_000, 768, 4096, 64, 96, 10, 256
NCENT, SIGMA = 1024, 1.0  # bench.py's clustered synthetic data (C4 / C5)


def clustered(n, nq, seed=1234):
    rng = np.random.default_rng(seed)
    C = rng.standard_normal((NCENT, D), dtype=np.float32)
    X = rng.standard_normal((n, D), dtype=np.float32)
    X *= SIGMA
    X += C[rng.integers(0, NCENT, n)]
    Q = rng.standard_normal((nq, D), dtype=np.float32)
    Q *= SIGMA
    Q += C[rng.integers(0, NCENT, nq)]
    return X, Q


@pytest.fixture(scope="module")
def data():
    return clustered(N, B)


@pytest.fixture(scope="module")
def exact(data):
    X, Q = data
    el, ed, _ = c_oracle.flat_search_batch(X, Q, K, "l2", acc64=True, nthreads=16)
    return el, ed


def build(hip, X, index_type):
    h = hip.LanceCreateDetached("", D, "l2", "c45")
    # IVF_FLAT keeps the default bf16 scan copy (its bound scan streams it, as
    # bench.py --config c4 runs); IVF_PQ scans codes only
    if index_type == "ivf_pq":
        hip.LanceHipSetOption(h, "scan_copy", "off")
    hip.LanceHipSetOption(h, "reserve_rows", str(len(X)))
    hip.LanceHipSetOption(h, "index_type", index_type)
    for lo in range(0, len(X), 1 << 18):
        hi = min(len(X), lo + (1 << 18))
        hip.LanceDetachedAddBatch(h, X[lo:hi], hi - lo, D)
    hip.LanceDetachedCreateIndex(h, NLIST, M if index_type == "ivf_pq" else 0)
    info = hip.LanceHipIvfInfo(h)
    assert info["type"] == index_type and info["nlist"] == NLIST and info["n_indexed"] == len(X)
    if index_type == "ivf_pq":
        assert info["m"] == M and info["dsub"] == D // M
    return h


def port_search(hip, h, X, Q, nprobe, refine, lut="u8", query_fp8=False):
    ex = hip.LanceHipIvfExport(h)
    Xs = X[ex["labels"]]
    lay = c_oracle.IvfLayout(ex["lists"], ex["live"], NLIST)
    kw = {}
    if ex["type"] == "ivf_pq":
        _, T = ivf.pq_tables(ex["centroids"], ex["codebook"], Q[:1], "l2")
        kw = dict(codes=ex["codes"], codebook=ex["codebook"], T=T, refine_factor=refine, lut=lut, query_fp8=query_fp8)
    return c_oracle.ivf_search_batch(Xs, ex["labels"], lay, ex["centroids"], Q, K, nprobe, "l2", acc64=True,
                                     nthreads=16, **kw)


def check(gl, gd, gc, el, ed, ec):
    np.testing.assert_array_equal(gc, ec)
    for i in range(len(ec)):
        n = int(gc[i])
        np.testing.assert_array_equal(gl[i, :n], el[i, :n], err_msg=f"query {i}")
        np.testing.assert_allclose(gd[i, :n], ed[i, :n], rtol=1e-4, atol=1e-5, err_msg=f"query {i}")


def test_c4_ivf_flat_nlist4096_nprobe64(hip, data, exact):
    """The shipped default IVF_FLAT path at C4's parameters — the bf16 MFMA bound
    scan of every probed list (flat_list_lb_kernel) + certified exact re-rank,
    what bench.py --config c4 times — then the exact f64 list scan
    (ivf_flat_scan=exact) on the same index; both against the C port."""
    X, Q = data
    h = build(hip, X, "ivf_flat")
    try:
        ref = port_search(hip, h, X, Q, NPROBE, 1)
        hip.LanceHipSetOption(h, "time_kernels", "1")
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, K, nprobes=NPROBE, refine_factor=1)
        kt = hip.LanceHipKernelTimes(h)
        hip.LanceHipSetOption(h, "time_kernels", "0")
        check(gl, gd, gc, *ref)
        # IVF_FLAT distances are exact: recall is the probe coverage alone
        rec = flat_knn.recall_at_k(gl, exact[0], K)
        print(f"C4 params, bound scan: recall@10 = {rec:.4f} (nprobe {NPROBE})")
        assert rec >= 0.99
        hip.LanceHipSetOption(h, "ivf_flat_scan", "exact")
        hip.LanceHipSetOption(h, "time_kernels", "1")
        gl2, gd2, gc2 = hip.LanceDetachedSearchBatch(h, Q, K, nprobes=NPROBE, refine_factor=1)
        kt2 = hip.LanceHipKernelTimes(h)
        hip.LanceHipSetOption(h, "time_kernels", "0")
        check(gl2, gd2, gc2, *ref)
        np.testing.assert_array_equal(gl2, gl)
        # the default run was ONE certified bound-scan launch over bf16 rows (2 B per
        # element: half the exact scan's f32 bytes for the same probed lists; an
        # uncertified batch would have added an exact launch)
        assert kt["ivf_scan_launches"] == 1 and kt2["ivf_scan_launches"] == 1, (kt, kt2)
        assert kt2["ivf_scan_bytes"] == 2 * kt["ivf_scan_bytes"], (kt, kt2)
    finally:
        hip.LanceFreeDetached(h)


def test_c5_ivf_pq_m96_refine_sweep(hip, data, exact):
    """The default fast scan (8-bit LUT, list-major) over a refine sweep, the
    fp8-query variant the C5 config names, and the f32-LUT query-major scan,
    each against the C port in the same mode."""
    X, Q = data
    h = build(hip, X, "ivf_pq")
    try:
        recalls = {}
        for rf in (1, 10, 50):
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, K, nprobes=NPROBE, refine_factor=rf)
            check(gl, gd, gc, *port_search(hip, h, X, Q, NPROBE, rf))
            recalls[rf] = flat_knn.recall_at_k(gl, exact[0], K)
        print("C5 params, fast scan: recall@10 by refine_factor", recalls)
        # a wider exact re-rank window can only help (the ADC candidates of
        # refine r are a prefix of those of r' > r)
        assert recalls[1] <= recalls[10] + 1e-9 <= recalls[50] + 2e-9
        # f32-LUT scan measured on MI355X: 0.294 / 0.818 / 0.996 (profiles/r02_c_ivf_params.log)
        assert recalls[10] >= 0.75
        assert recalls[50] >= 0.98
        # the per-query bound seeded from the nearest probed list (option pq_seed,
        # default on) only skips work: the same lists without it
        g_seed = hip.LanceDetachedSearchBatch(h, Q, K, nprobes=NPROBE, refine_factor=10)
        hip.LanceHipSetOption(h, "pq_seed", "0")
        g_noseed = hip.LanceDetachedSearchBatch(h, Q, K, nprobes=NPROBE, refine_factor=10)
        hip.LanceHipSetOption(h, "pq_seed", "1")
        for a, b in zip(g_seed, g_noseed):
            np.testing.assert_array_equal(a, b)
        # a NaN query (no probed list: the seed skips it) and a zero query in the
        # batch: seeded == unseeded, and the other queries keep their lists
        Qx = Q.copy()
        Qx[3] = np.nan
        Qx[5] = 0.0
        gx = hip.LanceDetachedSearchBatch(h, Qx, K, nprobes=NPROBE, refine_factor=10)
        hip.LanceHipSetOption(h, "pq_seed", "0")
        gx0 = hip.LanceDetachedSearchBatch(h, Qx, K, nprobes=NPROBE, refine_factor=10)
        hip.LanceHipSetOption(h, "pq_seed", "1")
        for a, b in zip(gx, gx0):
            np.testing.assert_array_equal(a, b)
        keep = np.setdiff1d(np.arange(len(Q)), [3, 5])
        for a, b in zip(gx, g_seed):
            np.testing.assert_array_equal(a[keep], b[keep])
        hip.LanceHipSetOption(h, "pq_query", "fp8")
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, K, nprobes=NPROBE, refine_factor=10)
        check(gl, gd, gc, *port_search(hip, h, X, Q, NPROBE, 10, query_fp8=True))
        r8 = flat_knn.recall_at_k(gl, exact[0], K)
        print(f"C5 params, fast scan, fp8 queries: recall@10 = {r8:.4f} (refine 10)")
        assert r8 >= recalls[10] - 0.05
        hip.LanceHipSetOption(h, "pq_query", "f32")
        hip.LanceHipSetOption(h, "pq_scan", "exact_lut")
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, K, nprobes=NPROBE, refine_factor=10)
        check(gl, gd, gc, *port_search(hip, h, X, Q, NPROBE, 10, lut="f32"))
        r32 = flat_knn.recall_at_k(gl, exact[0], K)
        print(f"C5 params, f32-LUT scan: recall@10 = {r32:.4f} (refine 10)")
        assert r32 >= 0.75
    finally:
        hip.LanceFreeDetached(h)
