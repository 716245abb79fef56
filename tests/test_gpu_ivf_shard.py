"""GPU parity of IVF_FLAT and IVF_PQ at the C4 / C5 per-GPU shard size itself:
12.5M clustered rows x 768 (BASELINE.json configs[3] / [4]: 100M rows over 8
GPUs), nlist = 4096, nprobe = 64, IVF_PQ m = 96, k = 10, a batch of 256
queries — the shapes bench.py --config c4 / c5 time (clustered rows drawn
like bench.py's: 1024 centres, sigma 1), with every list holding ~3k rows (tests/test_gpu_ivf_params.py runs the same parameters on 1M rows).

Reference: rust_lib/src/lance_manager.rs:411-419 (search with nprobes /
refine_factor) and :483-515 (IVF_PQ build).  Checker: oracle/flat_knn.c's IVF
port over the model and row layout the library exports (labels bit-exact,
distances within 1e-4 relative); parity with LanceDB itself is unpinned for
IVF (no reference test builds an IVF index)."""
import numpy as np
import pytest

from oracle import c_oracle, ivf

pytestmark = pytest.mark.gpu

N, D, NLIST, NPROBE, M, K, B = 12_500_000, 768, 4096, 64, 96, 10, 256
NCENT, SIGMA = 1024, 1.0


def check(gl, gd, gc, el, ed, ec):
    np.testing.assert_array_equal(gc, ec)
    for i in range(len(ec)):
        n = int(gc[i])
        np.testing.assert_array_equal(gl[i, :n], el[i, :n], err_msg=f"query {i}")
        np.testing.assert_allclose(gd[i, :n], ed[i, :n], rtol=1e-4, atol=1e-5, err_msg=f"query {i}")


def test_c4_c5_at_shard_size(hip):
    import torch

    L = hip.lib()
    g = torch.Generator(device="cuda")
    g.manual_seed(12_500_003)
    C = torch.randn((NCENT, D), generator=g, device="cuda", dtype=torch.float32)
    Xh = np.empty((N, D), np.float32)
    h = hip.LanceCreateDetached("", D, "l2", "shard")
    e = hip._err()
    try:
        hip.LanceHipSetOption(h, "reserve_rows", str(N))
        for lo in range(0, N, 1 << 20):
            hi = min(N, lo + (1 << 20))
            ids = torch.randint(0, NCENT, (hi - lo,), generator=g, device="cuda")
            X = torch.randn((hi - lo, D), generator=g, device="cuda", dtype=torch.float32).mul_(SIGMA).add_(C[ids])
            torch.cuda.synchronize()
            assert L.lance_hip_add_batch_device(h, X.data_ptr(), hi - lo, D, e, len(e)) >= 0, e.value
            Xh[lo:hi] = X.cpu().numpy()
            del X, ids
        qids = torch.randint(0, NCENT, (B,), generator=g, device="cuda")
        Q = (C[qids] + SIGMA * torch.randn((B, D), generator=g, device="cuda", dtype=torch.float32)).cpu().numpy()

        def port(nprobe, refine, query_fp8=False):
            ex = hip.LanceHipIvfExport(h)
            # slots are the rows in insertion order (added once, never deleted): the
            # label-ordered host copy is the slot-ordered one
            np.testing.assert_array_equal(ex["labels"], np.arange(N))
            lay = c_oracle.IvfLayout(ex["lists"], ex["live"], NLIST)
            kw = {}
            if ex["type"] == "ivf_pq":
                _, T = ivf.pq_tables(ex["centroids"], ex["codebook"], Q[:1], "l2")
                kw = dict(codes=ex["codes"], codebook=ex["codebook"], T=T, refine_factor=refine, lut="u8",
                          query_fp8=query_fp8)
            return c_oracle.ivf_search_batch(Xh, ex["labels"], lay, ex["centroids"], Q, K, nprobe, "l2", acc64=True,
                                             nthreads=16, **kw)

        # C4: IVF_FLAT, the default certified bound scan
        hip.LanceHipSetOption(h, "index_type", "ivf_flat")
        hip.LanceDetachedCreateIndex(h, NLIST, 0)
        info = hip.LanceHipIvfInfo(h)
        assert info["type"] == "ivf_flat" and info["nlist"] == NLIST and info["n_indexed"] == N, info
        hip.LanceHipSetOption(h, "time_kernels", "1")
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, K, nprobes=NPROBE, refine_factor=1)
        kt = hip.LanceHipKernelTimes(h)
        hip.LanceHipSetOption(h, "time_kernels", "0")
        assert kt["ivf_scan_launches"] == 1, kt  # one certified bound-scan launch, no exact rerun
        check(gl, gd, gc, *port(NPROBE, 1))
        # C5: IVF_PQ m = 96 over the same rows (replace = true), fp8 queries as configs[4] names
        hip.LanceHipSetOption(h, "index_type", "ivf_pq")
        hip.LanceDetachedCreateIndex(h, NLIST, M)
        info = hip.LanceHipIvfInfo(h)
        assert info["type"] == "ivf_pq" and info["m"] == M and info["n_indexed"] == N, info
        for rf in (1, 10):
            gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, K, nprobes=NPROBE, refine_factor=rf)
            check(gl, gd, gc, *port(NPROBE, rf))
        hip.LanceHipSetOption(h, "pq_query", "fp8")
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q, K, nprobes=NPROBE, refine_factor=10)
        check(gl, gd, gc, *port(NPROBE, 10, query_fp8=True))
    finally:
        hip.LanceFreeDetached(h)
        del Xh
