"""The north_star size on the GPU: flat squared L2 over 10M x 768 f32 rows,
256 queries, k = 10 (BASELINE.json north_star; bench.py --config nstar).
Every query's search runs the default large-store path (sample pass, int8
scan8 append pass, pool_refine) and must come out certified (no rerun, no
exact fallback); the ids of a 64-query subset are checked against the f64 C
oracle (labels bit-exact, distances within 1e-4 relative), and recall@10 is
1.0 on them.  Reference semantics: rust_lib/src/lance_manager.rs:393-451."""
import numpy as np
import pytest

from oracle import c_oracle, flat_knn
from tests.test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

N, D, K, B, NCHECK = 10_000_000, 768, 10, 256, 64


def test_north_star_10m_exact(hip):
    import torch

    L = hip.lib()
    h = hip.LanceCreateDetached("", D, "l2", "nstar")
    Xh = np.empty((N, D), np.float32)
    try:
        hip.LanceHipSetOption(h, "reserve_rows", str(N))
        g = torch.Generator(device="cuda")
        g.manual_seed(10_000_019)
        e = hip._err()
        for lo in range(0, N, 1 << 20):
            hi = min(N, lo + (1 << 20))
            X = torch.randn((hi - lo, D), generator=g, device="cuda", dtype=torch.float32)
            torch.cuda.synchronize()
            assert L.lance_hip_add_batch_device(h, X.data_ptr(), hi - lo, D, e, len(e)) >= 0, e.value
            Xh[lo:hi] = X.cpu().numpy()
            del X
        Q = torch.randn((B, D), generator=g, device="cuda", dtype=torch.float32)
        hip.LanceHipSetOption(h, "time_kernels", "1")
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Q.cpu().numpy(), K)
        st = hip.LanceHipLastSearchStats(h)
        kt = hip.LanceHipKernelTimes(h)
        assert kt["scan_kernel"] == "scan8_kernel" and kt["scan_elem_bytes"] == 1, kt
        assert not st["dense_path"] and st["fallback_queries"] == 0 and st["retried_queries"] == 0, st
        assert (gc == K).all()
        el, ed, ec = c_oracle.flat_search_batch(Xh, Q[:NCHECK].cpu().numpy(), K, "l2", acc64=True, nthreads=16)
        assert_same(gl[:NCHECK], gd[:NCHECK], gc[:NCHECK], el, ed, ec)
        assert flat_knn.recall_at_k(gl[:NCHECK], el, K) == 1.0
        # every distance row ascending, every label in range
        assert (np.diff(gd, axis=1) >= 0).all() and gl.min() >= 0 and gl.max() < N
    finally:
        hip.LanceFreeDetached(h)
        del Xh


def test_c3_full_size_bf16_dot_k100(hip):
    """BASELINE.json configs[2] at its own size: a bf16 store of 10M x 768
    L2-normalised rows, inner product, k = 100, 256 normalised queries.  The
    pools reach ~32k bounds per query, far past pool_refine's LDS capacity (the
    smallest are kept, the rest bound the certificate); every query must certify
    without a rerun or the exact fallback, and the ids of a 64-query subset equal
    the f64 C oracle over the stored (bf16-rounded) rows."""
    import torch

    L = hip.lib()
    h = hip.LanceCreateDetached("", D, "dot", "c3")
    Xh = np.empty((N, D), np.float32)
    try:
        hip.LanceHipSetOption(h, "storage", "bf16")
        hip.LanceHipSetOption(h, "reserve_rows", str(N))
        g = torch.Generator(device="cuda")
        g.manual_seed(30_000_001)
        e = hip._err()
        for lo in range(0, N, 1 << 20):
            hi = min(N, lo + (1 << 20))
            X = torch.randn((hi - lo, D), generator=g, device="cuda", dtype=torch.float32)
            X /= X.norm(dim=1, keepdim=True)
            torch.cuda.synchronize()
            assert L.lance_hip_add_batch_device(h, X.data_ptr(), hi - lo, D, e, len(e)) >= 0, e.value
            Xh[lo:hi] = X.to(torch.bfloat16).float().cpu().numpy()  # what the bf16 store holds (RNE)
            del X
        Q = torch.randn((B, D), generator=g, device="cuda", dtype=torch.float32)
        Q /= Q.norm(dim=1, keepdim=True)
        Qh = Q.cpu().numpy()
        hip.LanceHipSetOption(h, "time_kernels", "1")
        gl, gd, gc = hip.LanceDetachedSearchBatch(h, Qh, 100)
        st = hip.LanceHipLastSearchStats(h)
        kt = hip.LanceHipKernelTimes(h)
        assert kt["scan_kernel"] == "scan8_kernel" and kt["scan_elem_bytes"] == 1, kt
        assert not st["dense_path"] and st["fallback_queries"] == 0 and st["retried_queries"] == 0, st
        assert st["max_pool"] > 16384, st  # the pools overflow pool_refine's LDS capacity (PR_CAP) at this size
        assert (gc == 100).all()
        el, ed, ec = c_oracle.flat_search_batch(Xh, Qh[:NCHECK], 100, "dot", acc64=True, nthreads=16)
        assert_same(gl[:NCHECK], gd[:NCHECK], gc[:NCHECK], el, ed, ec)
        assert flat_knn.recall_at_k(gl[:NCHECK], el, 100) == 1.0
        assert (np.diff(gd, axis=1) >= 0).all() and gl.min() >= 0 and gl.max() < N
    finally:
        hip.LanceFreeDetached(h)
        del Xh
