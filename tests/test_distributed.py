"""Multi-rank sharded search, world_size 2-3 over gloo.

CPU tests: the exchange/merge logic of ``lance_hip.sharded`` with the oracle as
each rank's shard searcher and a reference merge; the result on every rank must
equal the unsharded oracle.  GPU test: two ranks on one device, each searching
its shard through the C-ABI, gathered over gloo, merged by the HIP merge kernel.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from lance_hip.sharded import ShardedSearch, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def ref_merge(gl, gd, gc):
    """Reference merge under the (distance, label) order, the default tie rule
    (label_desc; LANCE_HIP_TIE) (test-side)."""
    from oracle import flat_knn

    sgn = -1 if flat_knn.tie_desc(None) else 1
    world, nq, k = gl.shape
    ol = torch.full((nq, k), -1, dtype=torch.int64)
    od = torch.full((nq, k), float("nan"), dtype=torch.float32)
    oc = torch.zeros(nq, dtype=torch.int32)
    for q in range(nq):
        items = []
        for s in range(world):
            for i in range(int(gc[s, q])):
                items.append((float(gd[s, q, i]), sgn * int(gl[s, q, i])))
        items.sort()
        items = [(dd, sgn * l) for dd, l in items[:k]]
        oc[q] = len(items)
        for i, (d, l) in enumerate(items):
            ol[q, i] = l
            od[q, i] = d
    return ol, od, oc


def _cpu_worker(rank, world, port, n, d, k, q, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from oracle import flat_knn

    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(7)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((q, d)).astype(np.float32)
    s0, s1 = shard_range(n, world, rank)
    Xs = X[s0:s1]

    def local_search(Qt, kk):
        l, dd, c = flat_knn.flat_search_batch(Xs, np.arange(s1 - s0), np.ones(s1 - s0, bool), Qt.numpy(), kk)
        return torch.from_numpy(l), torch.from_numpy(dd), torch.from_numpy(c)

    s = ShardedSearch(local_search, ref_merge, label_offset=s0, dist=dist, world=world)
    l, dd, c = s.search(torch.from_numpy(Q), k)
    out[rank] = (l.numpy(), dd.numpy(), c.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1000), (3, 1001)])
def test_sharded_merge_equals_unsharded_cpu(world, n):
    from oracle import flat_knn

    d, k, q = 8, 6, 5
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_cpu_worker, args=(world, _free_port(), n, d, k, q, out), nprocs=world, join=True)
    rng = np.random.default_rng(7)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((q, d)).astype(np.float32)
    el, ed, ec = flat_knn.flat_search_batch(X, np.arange(n), np.ones(n, bool), Q, k)
    for r in range(world):
        l, dd, c = out[r]
        np.testing.assert_array_equal(l, el)
        np.testing.assert_array_equal(c, ec)
        np.testing.assert_allclose(dd, ed, rtol=1e-6)


class _CpuPipe:
    """CPU stand-in for AsyncPipeline: submit computes, wait returns by ticket."""

    def __init__(self, search):
        self.search, self.done, self.t = search, {}, 0

    def submit(self, Q, k):
        self.t += 1
        self.done[self.t] = self.search(Q, k)
        return self.t

    def wait(self, t):
        return self.done.pop(t)


def _cpu_pipeline_worker(rank, world, port, n, d, k, q, nb, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from lance_hip.sharded import ShardedPipeline
    from oracle import flat_knn

    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(9)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Qs = [rng.standard_normal((q, d)).astype(np.float32) for _ in range(nb)]
    s0, s1 = shard_range(n, world, rank)
    Xs = X[s0:s1]

    def local_search(Qt, kk):
        l, dd, c = flat_knn.flat_search_batch(Xs, np.arange(s1 - s0), np.ones(s1 - s0, bool), Qt.numpy(), kk)
        return torch.from_numpy(l), torch.from_numpy(dd), torch.from_numpy(c)

    sh = ShardedSearch(local_search, ref_merge, label_offset=s0, dist=dist, world=world)
    pipe = ShardedPipeline(_CpuPipe(local_search), sh)
    res = []
    for Q in Qs:  # batch i's result arrives one step later
        r = pipe.step(torch.from_numpy(Q), k)
        if r is not None:
            res.append(tuple(x.numpy() for x in r))
    res.append(tuple(x.numpy() for x in pipe.drain()))
    assert pipe.drain() is None
    out[rank] = res
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_pipeline_two_batches_in_flight_cpu(world):
    """bench.py's N > 1 loop: batch i-1's exchange runs after batch i is
    submitted; every batch's merged lists equal the unsharded search, in order."""
    from oracle import flat_knn

    n, d, k, q, nb = 997, 8, 5, 4, 4
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_cpu_pipeline_worker, args=(world, _free_port(), n, d, k, q, nb, out), nprocs=world, join=True)
    rng = np.random.default_rng(9)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Qs = [rng.standard_normal((q, d)).astype(np.float32) for _ in range(nb)]
    for r in range(world):
        assert len(out[r]) == nb
        for Q, (l, dd, c) in zip(Qs, out[r]):
            el, ed, ec = flat_knn.flat_search_batch(X, np.arange(n), np.ones(n, bool), Q, k)
            np.testing.assert_array_equal(l, el)
            np.testing.assert_array_equal(c, ec)
            np.testing.assert_allclose(dd, ed, rtol=1e-6)


class _CpuPackedPipe(_CpuPipe):
    """CPU stand-in for ``AsyncPipeline(packed=True)``: the results land in a
    packed row (``packed_outputs``) carrying the rank's label offset."""

    def __init__(self, search, label_offset):
        super().__init__(search)
        self.off = label_offset

    def submit(self, Q, k):
        from lance_hip.sharded import packed_outputs, packed_stride

        l, dd, c = self.search(Q, k)
        o = packed_outputs(l.shape[0], k, "cpu", self.off, packed_stride(l.shape[0], k))
        for dst, src in zip(o, (l, dd, c)):
            dst.copy_(src)
        self.t += 1
        self.done[self.t] = o
        return self.t


def _cpu_packed_worker(rank, world, port, n, d, k, q, nb, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from lance_hip.sharded import ShardedPipeline, unpack_rows
    from oracle import flat_knn

    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(13)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Qs = [rng.standard_normal((q, d)).astype(np.float32) for _ in range(nb)]
    s0, s1 = shard_range(n, world, rank)
    Xs = X[s0:s1]

    def local_search(Qt, kk):
        l, dd, c = flat_knn.flat_search_batch(Xs, np.arange(s1 - s0), np.ones(s1 - s0, bool), Qt.numpy(), kk)
        return torch.from_numpy(l), torch.from_numpy(dd), torch.from_numpy(c)

    def no_generic(*_):
        raise AssertionError("the packed outputs must take the packed exchange")

    sh = ShardedSearch(local_search, no_generic, label_offset=s0, dist=dist, world=world,
                       merge_packed=lambda g, nq, kk: ref_merge(*unpack_rows(g, nq, kk)))
    pipe = ShardedPipeline(_CpuPackedPipe(local_search, s0), sh)
    res = []
    for Q in Qs:
        r = pipe.step(torch.from_numpy(Q), k)
        if r is not None:
            res.append(tuple(x.numpy() for x in r))
    res.append(tuple(x.numpy() for x in pipe.drain()))
    out[rank] = res
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,q", [(2, 4), (3, 5)])
def test_sharded_pipeline_packed_exchange_cpu(world, q):
    """The packed exchange (one gathered row per rank, label offsets carried in
    the rows' tails, odd nq padded): merged lists equal the unsharded search."""
    from oracle import flat_knn

    n, d, k, nb = 1003, 8, 6, 3
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_cpu_packed_worker, args=(world, _free_port(), n, d, k, q, nb, out), nprocs=world, join=True)
    rng = np.random.default_rng(13)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Qs = [rng.standard_normal((q, d)).astype(np.float32) for _ in range(nb)]
    for r in range(world):
        assert len(out[r]) == nb
        for Q, (l, dd, c) in zip(Qs, out[r]):
            el, ed, ec = flat_knn.flat_search_batch(X, np.arange(n), np.ones(n, bool), Q, k)
            np.testing.assert_array_equal(l, el)
            np.testing.assert_array_equal(c, ec)
            np.testing.assert_allclose(dd, ed, rtol=1e-6)


def test_packed_stride_matches_the_library():
    import lance_hip
    from lance_hip.sharded import packed_stride

    L = lance_hip.lib()
    for nq, k in ((1, 1), (5, 6), (256, 10), (255, 100), (4096, 1000)):
        s = packed_stride(nq, k)
        assert s % 2 == 0 and s >= 3 * nq * k + nq + 2
        assert L.lance_hip_merge_packed_stride(nq, k) == s
    assert L.lance_hip_merge_packed_stride(0, 10) == -1
    # argument checks come before any device call (no GPU needed)
    import ctypes

    e = ctypes.create_string_buffer(2048)
    assert L.lance_hip_merge_topk_packed(2, 4, 3, None, packed_stride(4, 3), None, None, None, e, 2048) == -1
    assert "null buffer" in e.value.decode()
    buf = ctypes.create_string_buffer(1024)
    addr = (ctypes.addressof(buf) + 7) // 8 * 8
    assert L.lance_hip_merge_topk_packed(2, 4, 3, addr, packed_stride(4, 3) - 2, addr, addr, addr, e, 2048) == -1
    assert "row_stride" in e.value.decode()
    assert L.lance_hip_merge_topk_packed(0, 4, 3, None, 0, None, None, None, e, 2048) == 0


def test_shard_range_partitions_exactly():
    for n in (0, 1, 7, 1000, 1_000_000):
        for world in (1, 2, 3, 8):
            rs = [shard_range(n, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a0, a1), (b0, b1) in zip(rs, rs[1:]):
                assert a1 == b0
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1


def _gpu_worker(rank, world, port, n, d, k, q, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import lance_hip
    from lance_hip.sharded import hip_device_merge, hip_device_search

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    L = lance_hip.lib()
    rng = np.random.default_rng(11)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((q, d)).astype(np.float32)
    s0, s1 = shard_range(n, world, rank)
    h = lance_hip.LanceCreateDetached("", d, "l2", f"shard{rank}")
    lance_hip.LanceDetachedAddBatch(h, X[s0:s1], s1 - s0, d)
    dev_search = hip_device_search(L, h, d)
    dev_merge = hip_device_merge(L)

    def local_search(Qt, kk):  # GPU search, results moved to the CPU for gloo
        l, dd, c = dev_search(Qt.cuda(), kk)
        return l.cpu(), dd.cpu(), c.cpu()

    def merge(gl, gd, gc):  # HIP merge kernel on the device
        l, dd, c = dev_merge(gl.cuda(), gd.cuda(), gc.cuda())
        return l.cpu(), dd.cpu(), c.cpu()

    s = ShardedSearch(local_search, merge, label_offset=s0, dist=dist, world=world)
    l, dd, c = s.search(torch.from_numpy(Q), k)
    out[rank] = (l.numpy(), dd.numpy(), c.numpy())
    lance_hip.LanceFreeDetached(h)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_hip_search_two_ranks_one_gpu():
    from oracle import flat_knn

    world, n, d, k, q = 2, 90_000, 64, 10, 40   # 45k rows per shard: dense path on each
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gpu_worker, args=(world, _free_port(), n, d, k, q, out), nprocs=world, join=True)
    rng = np.random.default_rng(11)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Q = rng.standard_normal((q, d)).astype(np.float32)
    el, ed, ec = flat_knn.flat_search_batch(X, np.arange(n), np.ones(n, bool), Q, k)
    for r in range(world):
        l, dd, c = out[r]
        np.testing.assert_array_equal(l, el)
        np.testing.assert_allclose(dd, ed, rtol=1e-4, atol=1e-5)


def _gpu_scan8_worker(rank, world, port, n, d, k, q, out, pipelined=False):
    # the bench's flat multi-GPU flow on the DEFAULT large-store path: each shard
    # > 65536 rows at d = 768 takes the threshold pipeline (sample pass, int8
    # scan8_kernel append pass, pool_refine), per-shard lists gathered and merged
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import lance_hip
    from lance_hip.sharded import hip_device_merge, hip_device_search

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    L = lance_hip.lib()
    rng = np.random.default_rng(21)
    X = rng.standard_normal((n, d), dtype=np.float32)
    Q = rng.standard_normal((q, d), dtype=np.float32)
    s0, s1 = shard_range(n, world, rank)
    h = lance_hip.LanceCreateDetached("", d, "l2", f"s8shard{rank}")
    for lo in range(s0, s1, 1 << 16):
        hi = min(s1, lo + (1 << 16))
        lance_hip.LanceDetachedAddBatch(h, X[lo:hi], hi - lo, d)
    del X
    lance_hip.LanceHipSetOption(h, "time_kernels", "1")
    dev_search = hip_device_search(L, h, d)
    dev_merge = hip_device_merge(L)

    def local_search(Qt, kk):
        l, dd, c = dev_search(Qt.cuda(), kk)
        return l.cpu(), dd.cpu(), c.cpu()

    def merge(gl, gd, gc):
        l, dd, c = dev_merge(gl.cuda(), gd.cuda(), gc.cuda())
        return l.cpu(), dd.cpu(), c.cpu()

    packed = pipelined == "packed"
    from lance_hip.sharded import hip_packed_merge

    dev_pmerge = hip_packed_merge(L)

    def merge_packed(g, nq, kk):  # the packed exchange's one-launch merge on the device
        return tuple(x.cpu() for x in dev_pmerge(g.cuda(), nq, kk))

    s = ShardedSearch(local_search, merge, label_offset=s0, dist=dist, world=world,
                      merge_packed=merge_packed if packed else None)
    if pipelined:
        # bench.py's N > 1 loop: two batches in flight on the handle (the async
        # C-ABI), batch i-1 exchanged while batch i is on the device
        from lance_hip.sharded import AsyncPipeline, ShardedPipeline

        lance_hip.LanceHipSetOption(h, "time_kernels", "0")  # (timing forces the synchronous path)
        ap = AsyncPipeline(L, h, d, packed=packed, label_offset=s0)

        class _Pipe:
            held = []  # the device queries stay alive until their batch completes (AsyncPipeline holds them too)

            def submit(self, Qt, kk):
                Qd = Qt.cuda()
                self.held = (self.held + [Qd])[-3:]
                return ap.submit(Qd, kk)

            def wait(self, t):
                from lance_hip.sharded import Outputs

                o = ap.wait(t)
                r = Outputs(x.cpu() for x in o)
                if packed:  # (gloo gathers host tensors: the packed row moves as one)
                    assert o.pack is not None
                    r.pack = o.pack.cpu()
                return r

        pipe = ShardedPipeline(_Pipe(), s)
        Qs = [torch.from_numpy(Q), torch.from_numpy(Q[::-1].copy()), torch.from_numpy(Q)]
        res = [pipe.step(Qt, k) for Qt in Qs] + [pipe.drain()]
        assert res[0] is None
        st = lance_hip.LanceHipLastSearchStats(h)
        out[rank] = [tuple(x.numpy() for x in r) for r in res[1:]] + [st]
    else:
        l, dd, c = s.search(torch.from_numpy(Q), k)
        st = lance_hip.LanceHipLastSearchStats(h)
        kt = lance_hip.LanceHipKernelTimes(h)
        out[rank] = (l.numpy(), dd.numpy(), c.numpy(), st, kt["scan_kernel"], kt["scan_launches"])
    lance_hip.LanceFreeDetached(h)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_scan8_two_ranks_one_gpu():
    """2 ranks x 80k rows x 768, 256 queries: every rank's shard search is the
    int8 threshold path (scan8_kernel + pool_refine, certified, no fallback);
    the merged top-10 equals the unsharded exact search (f64 C oracle)."""
    from oracle import c_oracle

    world, n, d, k, q = 2, 160_000, 768, 10, 256
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gpu_scan8_worker, args=(world, _free_port(), n, d, k, q, out), nprocs=world, join=True)
    rng = np.random.default_rng(21)
    X = rng.standard_normal((n, d), dtype=np.float32)
    Q = rng.standard_normal((q, d), dtype=np.float32)
    el, ed, _ = c_oracle.flat_search_batch(X, Q, k, "l2", acc64=True, nthreads=16)
    for r in range(world):
        l, dd, c, st, kern, launches = out[r]
        assert kern == "scan8_kernel" and launches == 1, (kern, launches)
        assert not st["dense_path"] and st["append_launches"] == 1 and st["fallback_queries"] == 0, st
        assert (c == k).all()
        np.testing.assert_array_equal(l, el)
        np.testing.assert_allclose(dd, ed, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["generic", "packed"])
def test_sharded_scan8_pipelined_two_ranks_one_gpu(exchange):
    """The same shards through bench.py's pipelined N > 1 loop (async C-ABI,
    two batches in flight, exchange one batch behind): three batches, each
    merged result equal to the unsharded exact search, in submission order.
    packed: the search writes into the rank's packed row (label offset in its
    tail), gathered as one and merged by lance_hip_merge_topk_packed."""
    from oracle import c_oracle

    world, n, d, k, q = 2, 160_000, 768, 10, 256
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gpu_scan8_worker, args=(world, _free_port(), n, d, k, q, out, exchange), nprocs=world, join=True)
    rng = np.random.default_rng(21)
    X = rng.standard_normal((n, d), dtype=np.float32)
    Q = rng.standard_normal((q, d), dtype=np.float32)
    el, ed, _ = c_oracle.flat_search_batch(X, Q, k, "l2", acc64=True, nthreads=16)
    for r in range(world):
        *res, st = out[r]
        assert len(res) == 3 and st["fallback_queries"] == 0, st
        for i, (l, dd, c) in enumerate(res):
            el_i, ed_i = (el[::-1], ed[::-1]) if i == 1 else (el, ed)
            assert (c == k).all()
            np.testing.assert_array_equal(l, el_i)
            np.testing.assert_allclose(dd, ed_i, rtol=1e-4, atol=1e-5)


def _gpu_ivf_worker(rank, world, port, n, d, k, q, nlist, nprobe, out):
    # the bench's IVF multi-GPU flow (bench.py main_ivf): rank 0 trains, the model
    # is broadcast, every other rank installs it and indexes its own shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import lance_hip
    from lance_hip.sharded import hip_device_merge, hip_device_search

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    L = lance_hip.lib()
    rng = np.random.default_rng(12)
    C = rng.standard_normal((24, d)).astype(np.float32)
    X = (C[rng.integers(0, 24, n)] + 0.5 * rng.standard_normal((n, d))).astype(np.float32)
    Q = (X[rng.choice(n, q, replace=False)] + 0.1 * rng.standard_normal((q, d))).astype(np.float32)
    s0, s1 = shard_range(n, world, rank)
    h = lance_hip.LanceCreateDetached("", d, "l2", f"ivfshard{rank}")
    lance_hip.LanceHipSetOption(h, "index_type", "ivf_flat")
    lance_hip.LanceDetachedAddBatch(h, X[s0:s1], s1 - s0, d)
    Cm = torch.zeros((nlist, d), dtype=torch.float32)
    if rank == 0:
        lance_hip.LanceDetachedCreateIndex(h, nlist, 0)
        Cm.copy_(torch.from_numpy(lance_hip.LanceHipIvfExport(h)["centroids"]))
    dist.broadcast(Cm, 0)
    if rank != 0:
        lance_hip.LanceHipIvfSetModel(h, "ivf_flat", Cm.numpy())
    ex = lance_hip.LanceHipIvfExport(h)
    dev_search = hip_device_search(L, h, d, nprobes=nprobe)
    dev_merge = hip_device_merge(L)

    def local_search(Qt, kk):
        l, dd, c = dev_search(Qt.cuda(), kk)
        return l.cpu(), dd.cpu(), c.cpu()

    def merge(gl, gd, gc):
        l, dd, c = dev_merge(gl.cuda(), gd.cuda(), gc.cuda())
        return l.cpu(), dd.cpu(), c.cpu()

    s = ShardedSearch(local_search, merge, label_offset=s0, dist=dist, world=world)
    l, dd, c = s.search(torch.from_numpy(Q), k)
    out[rank] = (l.numpy(), dd.numpy(), c.numpy(), ex["lists"].copy(), Cm.numpy().copy())
    lance_hip.LanceFreeDetached(h)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_ivf_flat_two_ranks_one_gpu():
    # sharded IVF_FLAT over one broadcast model == unsharded IVF_FLAT with that
    # model and the same row placement (PQ is not: each shard re-ranks its own
    # k*refine_factor candidates, a superset of the unsharded re-rank window)
    from oracle import ivf

    world, n, d, k, q, nlist, nprobe = 2, 30_000, 32, 10, 24, 32, 5
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gpu_ivf_worker, args=(world, _free_port(), n, d, k, q, nlist, nprobe, out), nprocs=world, join=True)
    rng = np.random.default_rng(12)
    C = rng.standard_normal((24, d)).astype(np.float32)
    X = (C[rng.integers(0, 24, n)] + 0.5 * rng.standard_normal((n, d))).astype(np.float32)
    Q = (X[rng.choice(n, q, replace=False)] + 0.1 * rng.standard_normal((q, d))).astype(np.float32)
    lists = np.concatenate([out[r][3] for r in range(world)])
    el, ed, ec = ivf.ivf_flat_search(X, np.arange(n), np.ones(n, bool), lists, out[0][4], Q, k, nprobe, "l2")
    for r in range(world):
        l, dd, c = out[r][:3]
        np.testing.assert_array_equal(c, ec)
        np.testing.assert_array_equal(l, el)
        np.testing.assert_allclose(dd, ed, rtol=1e-4, atol=1e-5)
