"""Row-sharded search over several GPUs.

The base of one LANCE index is split into contiguous row ranges, one per rank
(one process per GPU).  Because the reference's labels are dense consecutive
integers (``rust_lib/src/lance_manager.rs:232-233``), shard ``r`` holding
global rows ``[s0, s1)`` stores them under local labels ``[0, s1-s0)`` and the
global label is ``s0 + local`` — no id translation table.  Every rank searches
its shard for the same query batch; the per-shard top-k lists are exchanged by
ONE all-gather (RCCL over xGMI on GPUs, gloo in CPU tests; labels, distances
and counts packed into one int32 buffer) and merged on the
device by ``lance_hip_merge_topk_device`` under the (distance, label) order.

Packed exchange (``AsyncPipeline(packed=True)`` + ``hip_packed_merge``): the
search writes its outputs straight into the rank's packed row, whose last two
words hold the rank's label offset, and the merge kernel reads the gathered
rows in place and shifts the labels itself — the exchange is then two
launches (the all-gather and ``lance_hip_merge_topk_packed``) where the
generic path needs eight (label shift, pack, three unpack copies, ...), and
every launch waits for a CU the next batch's scan is holding.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced row range of ``rank`` (sizes differ by at most 1)."""
    return rank * n_total // world, (rank + 1) * n_total // world


class Outputs(tuple):
    """``(labels, dists, counts)``; ``pack`` is the packed int32 row the three
    are views of (``None`` when they are separate tensors)."""
    pack = None


def packed_stride(nq: int, k: int) -> int:
    """int32 words per packed row (= ``lance_hip_merge_packed_stride``): the
    lists (3 * nq * k + nq words) rounded up to even, then the label offset."""
    body = 3 * nq * k + nq
    return (body + 1) // 2 * 2 + 2


def unpack_rows(g, nq: int, k: int):
    """Gathered packed rows ``g[world, stride]`` -> ``(labels[world,nq,k] with
    each row's label offset applied, dists, counts)``: the layout the packed
    merge kernel reads, restated with torch views (CPU tests' stand-in)."""
    import torch

    nqk = nq * k
    off = g[:, -2:].contiguous().view(torch.int64)  # [world, 1]
    gl = g[:, :2 * nqk].contiguous().view(torch.int64).view(-1, nq, k)
    gl = torch.where(gl >= 0, gl + off.view(-1, 1, 1), gl)
    gd = g[:, 2 * nqk:3 * nqk].contiguous().view(torch.float32).view(-1, nq, k)
    gc = g[:, 3 * nqk:3 * nqk + nq].contiguous()
    return gl, gd, gc


def packed_outputs(nq: int, k: int, device, label_offset: int, stride: int):
    """Output tensors as views of one packed row of ``stride`` int32 words
    (``lance_hip_merge_packed_stride``): labels int64[nq,k], dists f32[nq,k],
    counts i32[nq], the label offset (int64) in the last two words."""
    import torch

    buf = torch.empty((stride,), dtype=torch.int32, device=device)
    nqk = nq * k
    o = Outputs((buf[:2 * nqk].view(torch.int64).view(nq, k), buf[2 * nqk:3 * nqk].view(torch.float32).view(nq, k),
                 buf[3 * nqk:3 * nqk + nq]))
    buf[stride - 2:].view(torch.int64).fill_(int(label_offset))
    o.pack = buf
    return o


class ShardedSearch:
    """One rank's view of a sharded index.

    ``local_search(Q, k) -> (labels[nq,k] int64, dists[nq,k] f32, counts[nq] i32)``
    searches this rank's shard (local labels).  ``merge(gl, gd, gc) -> same``
    merges ``world`` gathered lists; ``dist`` is ``torch.distributed`` (or None
    for a single shard).  Tensors may live on the GPU (RCCL) or the CPU (gloo).
    ``merge_packed(g[world, stride], nq, k) -> same`` (optional) merges gathered
    packed rows; it is used when the outputs carry their ``pack``.
    """

    def __init__(self, local_search: Callable, merge: Callable, label_offset: int, dist=None,
                 world: int = 1, force_exchange: bool = False, merge_packed: Optional[Callable] = None):
        self.local_search = local_search
        self.merge = merge
        self.label_offset = int(label_offset)
        self.dist = dist
        self.world = int(world)
        # (force_exchange: a one-rank rehearsal of the multi-rank path — the packed
        # all-gather and the device merge run even for world == 1)
        self.force_exchange = bool(force_exchange)
        self.merge_packed = merge_packed
        self._bufs = None

    def search(self, Q, k: int, **kw):
        return self.exchange(*self.local_search(Q, k, **kw))

    def _gather(self, pack):
        import torch

        key = (pack.numel(), pack.device)
        if self._bufs is None or self._bufs[0] != key:
            self._bufs = (key, torch.empty((self.world * pack.numel(),), dtype=torch.int32, device=pack.device))
        g = self._bufs[1]
        self.dist.all_gather_into_tensor(g, pack)
        return g.view(self.world, -1)

    def exchange(self, lab, dis, cnt, pack=None):
        """This shard's top-k lists (local labels) -> the merged global lists.
        ``pack``: the packed row the lists are views of (``packed_outputs``,
        label offset already in its tail) — gathered and merged as it is."""
        if self.world == 1 and not self.force_exchange:
            return lab, dis, cnt
        if pack is not None and self.merge_packed is not None:
            nq, kk = lab.shape
            return self.merge_packed(self._gather(pack), nq, kk)
        # local -> global labels (unused slots stay -1)
        import torch

        lab = torch.where(lab >= 0, lab + self.label_offset, lab)  # no host sync
        nq, kk = lab.shape
        # ONE collective per batch: labels (int64 as 2 x int32), distances (f32
        # bits) and counts packed into an int32 row per rank (collective latency,
        # not bytes, is the cost at these sizes: 3 all-gathers would pay it 3x)
        pack = torch.cat([lab.contiguous().view(torch.int32).reshape(-1),
                          dis.contiguous().view(torch.int32).reshape(-1), cnt.to(torch.int32).reshape(-1)])
        g = self._gather(pack)
        nl, nd = 2 * nq * kk, nq * kk
        gl = g[:, :nl].contiguous().view(torch.int64).view(self.world, nq, kk)
        gd = g[:, nl:nl + nd].contiguous().view(torch.float32).view(self.world, nq, kk)
        gc = g[:, nl + nd:].contiguous().view(self.world, nq).to(cnt.dtype)
        return self.merge(gl, gd, gc)


def hip_device_merge(lib, err_len: int = 2048):
    """The product merge: ``lance_hip_merge_topk_device`` on the current device."""
    import ctypes

    import torch

    def merge(gl, gd, gc):
        world, nq, k = gl.shape
        ol = torch.empty((nq, k), dtype=torch.int64, device=gl.device)
        od = torch.empty((nq, k), dtype=torch.float32, device=gl.device)
        oc = torch.empty((nq,), dtype=torch.int32, device=gl.device)
        e = ctypes.create_string_buffer(err_len)
        r = lib.lance_hip_merge_topk_device(world, nq, k, gl.data_ptr(), gd.data_ptr(), gc.data_ptr(),
                                            ol.data_ptr(), od.data_ptr(), oc.data_ptr(), e, err_len)
        if r < 0:
            raise RuntimeError(e.value.decode())
        return ol, od, oc

    return merge


def hip_packed_merge(lib, err_len: int = 2048):
    """The packed-exchange merge: ``lance_hip_merge_topk_packed`` over the
    gathered rows ``g[world, stride]`` on the current device."""
    import ctypes

    import torch

    e = ctypes.create_string_buffer(err_len)

    def merge(g, nq, k):
        world, stride = g.shape
        ol = torch.empty((nq, k), dtype=torch.int64, device=g.device)
        od = torch.empty((nq, k), dtype=torch.float32, device=g.device)
        oc = torch.empty((nq,), dtype=torch.int32, device=g.device)
        r = lib.lance_hip_merge_topk_packed(world, nq, k, g.data_ptr(), stride, ol.data_ptr(), od.data_ptr(),
                                            oc.data_ptr(), e, err_len)
        if r < 0:
            raise RuntimeError(e.value.decode())
        return ol, od, oc

    return merge


def hip_device_search(lib, handle, dim: int, nprobes: int = 20, refine_factor: int = 1, err_len: int = 2048):
    """The product shard search: ``lance_hip_search_batch_device`` (inputs in HBM)."""
    import ctypes

    import torch

    e = ctypes.create_string_buffer(err_len)
    fn = lib.lance_hip_search_batch_device
    cache = {}

    def search(Q, k, reuse_outputs: bool = False):
        """reuse_outputs: return the same output tensors on every call of this
        shape (the caller consumes them before the next call)."""
        nq = Q.shape[0]
        key = (nq, k, Q.device)
        outs = cache.get(key) if reuse_outputs else None
        if outs is None:
            outs = (torch.empty((nq, k), dtype=torch.int64, device=Q.device),
                    torch.empty((nq, k), dtype=torch.float32, device=Q.device),
                    torch.empty((nq,), dtype=torch.int32, device=Q.device))
            if reuse_outputs:
                cache[key] = outs
        ol, od, oc = outs
        # Q written on torch's stream: wait for it only when that stream still has
        # work (a query of an idle stream costs ~1 us, a synchronize ~15 us)
        cs = torch.cuda.current_stream()
        if not cs.query():
            cs.synchronize()
        r = fn(handle, Q.data_ptr(), nq, dim, k, nprobes, refine_factor, ol.data_ptr(), od.data_ptr(), oc.data_ptr(),
               e, err_len)
        if r < 0:
            raise RuntimeError(e.value.decode())
        return ol, od, oc

    return search


class AsyncPipeline:
    """Two batches in flight on one handle (lance_hip_search_batch_device_async):
    ``step(Q, k)`` enqueues a batch and completes the previous one (certificate
    check, reruns, fallbacks at its wait), so the host's per-batch work overlaps
    the device's; ``drain()`` completes the last.  Returns the outputs of the
    batch completed by the call (None on the first).

    The pipeline holds each submitted query tensor until its batch completes
    (the library reads it on its own stream, behind the previous pass, so a
    temporary must not go back to torch's allocator before the wait).  Output
    tensors are double-buffered per shape: the tensors a wait returns stay valid
    until the next-but-one ``submit`` of the same shape (clone them to keep
    them longer).

    ``packed=True``: the outputs are views of one packed row per buffer
    (``packed_outputs``, carrying ``label_offset``), for ``ShardedSearch``'s
    packed exchange."""

    def __init__(self, lib, handle, dim: int, nprobes: int = 20, refine_factor: int = 1, err_len: int = 2048,
                 packed: bool = False, label_offset: int = 0, host_sync: bool = False):
        import ctypes

        self.lib, self.h, self.dim = lib, handle, dim
        self.nprobes, self.refine = nprobes, refine_factor
        self.e = ctypes.create_string_buffer(err_len)
        self.err_len = err_len
        self.outs = {}
        self.packed, self.label_offset = bool(packed), int(label_offset)
        self.host_sync = bool(host_sync)  # (an A/B: a host wait on torch's stream instead)
        self.completed = {}
        self.pending = []  # (ticket, outputs, query tensor held until the wait)
        self.i = 0

    def _out(self, nq, k, dev, j):
        import torch

        key = (nq, k, dev, j)
        if key not in self.outs and self.packed:
            self.outs[key] = packed_outputs(nq, k, dev, self.label_offset,
                                            int(self.lib.lance_hip_merge_packed_stride(nq, k)))
        if key not in self.outs:
            self.outs[key] = (torch.empty((nq, k), dtype=torch.int64, device=dev),
                              torch.empty((nq, k), dtype=torch.float32, device=dev),
                              torch.empty((nq,), dtype=torch.int32, device=dev))
        return self.outs[key]

    def submit(self, Q, k):
        import torch

        nq = Q.shape[0]
        ol, od, oc = o = self._out(nq, k, Q.device, self.i & 1)
        self.i += 1
        # Q (and, with a packed exchange, the all-gather still reading the output
        # row this batch overwrites) on torch's stream: the handle's stream waits
        # for that stream's work so far on the device (no host wait)
        cs = torch.cuda.current_stream()
        if not cs.query():
            if self.host_sync:
                cs.synchronize()
            elif self.lib.lance_hip_stream_after(self.h, cs.cuda_stream, self.e, self.err_len) != 0:
                raise RuntimeError(self.e.value.decode())
        t = self.lib.lance_hip_search_batch_device_async(self.h, Q.data_ptr(), nq, self.dim, k, self.nprobes,
                                                         self.refine, ol.data_ptr(), od.data_ptr(), oc.data_ptr(),
                                                         self.e, self.err_len)
        if t < 0:
            raise RuntimeError(self.e.value.decode())
        self.pending.append((t, o, Q))
        return t

    def wait(self, ticket=0):
        """Completes every batch up to ``ticket`` (<= 0: all) and returns the
        outputs of batch ``ticket`` (of the last completed one for <= 0);
        ``completed`` maps the ticket of every batch this call completed to its
        outputs."""
        if self.lib.lance_hip_search_wait(self.h, ticket, self.e, self.err_len) != 0:
            raise RuntimeError(self.e.value.decode())
        done = [p for p in self.pending if ticket <= 0 or p[0] <= ticket]
        self.pending = [p for p in self.pending if not (ticket <= 0 or p[0] <= ticket)]
        self.completed = {p[0]: p[1] for p in done}
        if not done:
            return None
        return self.completed.get(ticket, done[-1][1]) if ticket > 0 else done[-1][1]

    def step(self, Q, k):
        prev = self.pending[-1][0] if self.pending else None
        self.submit(Q, k)
        return self.wait(prev) if prev is not None else None

    def drain(self):
        return self.wait(0)


class ShardedPipeline:
    """Row-sharded search with two batches in flight per rank: ``step(Q, k)``
    enqueues batch i on this rank's shard (``pipe.submit``, the handle's
    stream), then completes batch i-1 (``pipe.wait``) and runs its exchange —
    the one all-gather and the device merge — while batch i's scan is still on
    the device.  Every rank calls ``step`` in the same order, so the collectives
    of all ranks pair up batch for batch.  Returns the merged lists of the batch
    completed by the call (None on the first); ``drain()`` completes the last.

    ``pipe`` has ``submit(Q, k) -> ticket`` and ``wait(ticket) -> (labels,
    dists, counts)`` (``AsyncPipeline`` on the GPU; a CPU stand-in in tests);
    ``sharded`` is this rank's ``ShardedSearch`` (its exchange is used)."""

    def __init__(self, pipe, sharded: ShardedSearch):
        self.pipe = pipe
        self.sharded = sharded
        self.prev = None

    def step(self, Q, k: int):
        t = self.pipe.submit(Q, k)
        out = None
        if self.prev is not None:
            o = self.pipe.wait(self.prev)
            out = self.sharded.exchange(*o, pack=getattr(o, "pack", None))
        self.prev = t
        return out

    def drain(self):
        if self.prev is None:
            return None
        o = self.pipe.wait(self.prev)
        out = self.sharded.exchange(*o, pack=getattr(o, "pack", None))
        self.prev = None
        return out
