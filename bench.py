#!/usr/bin/env python3
"""Headline benchmark: BASELINE.json metric "kNN queries/sec + recall@10,
1M x 768 f32 flat; GB/s vs HBM roofline" on configs[1] (C2): flat squared-L2,
N = 1,000,000 x d = 768 f32 base, k = 10, query batch B = 256.

One step = one batch of 256 queries searched through the C-ABI
(lance_hip_search_batch_device) against the whole base, inputs resident in HBM.
With --gpus N (one process per GPU, launched by torch.distributed.run) the base
is row-sharded over the ranks; every rank searches its shard for the same
batch, the per-shard top-k lists are all-gathered over RCCL (one collective per
batch) and merged on the device (lance_hip_merge_topk_device).
  --scaling weak   (default) fixed N, global batch = B x world: per-GPU flops
                   fixed as the GPU count grows ("scaling": "weak");
  --scaling strong fixed N and fixed global batch B: each rank scans N/world
                   rows for the same B queries ("scaling": "strong").
--config nstar is the north_star target: flat L2 over 10M x 768 f32.

Prints ONE JSON line on rank 0 (driver contract).  The CPU baseline (rank 0,
N = 1 only) times oracle/flat_knn.c — the port of the reference's flat search
(rust_lib/src/lance_manager.rs:393-451 -> lance flat KNN) — on a bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "duckdb-lancedb_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

lance_hip = None  # loaded by _load_lib() in the ranks (the --gpus N parent never touches the GPU)


def _load_lib():
    global lance_hip
    if lance_hip is None:
        import lance_hip as _lh

        lance_hip = _lh
    return lance_hip

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
MFMA_BF16_PEAK_TFS = 2500.0  # dense bf16 MFMA (no sparsity), same table

# --config presets (BASELINE.json configs): c2 is the headline line the driver
# runs; c3 = "Flat inner-product bf16 on MFMA, 10Mx768, k=100" (bf16-stored base,
# L2-normalized base and queries so that IP and L2 rankings coincide).
CONFIGS = {
    # C1: the reference's own CPU-runnable case through the reference API shape
    # (lance_search(): one query per call, host buffers, lance_detached_search)
    "c1": dict(n=10_000, dim=128, k=10, batch=1, metric="l2", storage="f32", normalize=False),
    "c2": dict(n=1_000_000, dim=768, k=10, batch=256, metric="l2", storage="f32", normalize=False),
    "c3": dict(n=10_000_000, dim=768, k=100, batch=256, metric="dot", storage="bf16", normalize=True),
    # north_star target: ">= 70 % HBM roofline on flat-L2 scan at 10M x 768 f32, recall@10 >= 0.99"
    "nstar": dict(n=10_000_000, dim=768, k=10, batch=256, metric="l2", storage="f32", normalize=False),
    # IVF configs: n is ROWS PER GPU (the 8-GPU configs of BASELINE.json hold 100M rows,
    # 12.5M per GPU; --gpus N runs N such shards), clustered synthetic rows
    "c4": dict(n=12_500_000, dim=768, k=10, batch=256, metric="l2", storage="f32", normalize=False,
               index_type="ivf_flat", nlist=4096, nprobe=64, m=0, refine=1),
    "c5": dict(n=12_500_000, dim=768, k=10, batch=256, metric="l2", storage="f32", normalize=False,
               index_type="ivf_pq", nlist=4096, nprobe=64, m=96, refine=10, pq_query="fp8", pq_scan="fast"),
}
# clustered synthetic data of the IVF configs: NCENT Gaussian clusters, centers
# N(0, 1) per dim (seed CENT_SEED), rows = center + SIGMA * N(0, 1)
NCENT, SIGMA, CENT_SEED = 1024, 1.0, 777
GEN_CHUNK = 65536


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--settle-s", type=float, default=0.3,
                    help="untimed steps for about this long BEFORE the W warmup steps: the GPU clocks up over its "
                         "first ~40-60 steps under load (C2 0.34 -> 0.27 ms per step, tools/ramp_probe.py, "
                         "profiles/r06e_ramp.jsonl); 0 = none")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--dim", type=int, default=None)
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--metric", default=None)
    ap.add_argument("--storage", choices=["f32", "bf16"], default=None, help="index option storage")
    ap.add_argument("--scan-copy", choices=["on", "off"], default="on", help="index option scan_copy")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                    help="multi-GPU (flat configs): strong (default, SURVEY.md §8e) = the global batch B over N/world "
                         "rows per rank; weak = global batch B x world. With --gpus > 1 the other mode is timed too "
                         "and reported under its own key")
    ap.add_argument("--no-other-scaling", action="store_true", help="multi-GPU: skip the extra weak/strong leg")
    ap.add_argument("--sync", action="store_true",
                    help="one GPU, device API: one synchronous search call per batch instead of two batches in "
                         "flight (the synchronous figure is reported beside the pipelined one either way)")
    ap.add_argument("--no-host-batch", action="store_true",
                    help="N = 1 flat configs: skip the extra host-buffer leg (H2D + D2H timed, SURVEY.md §8d QPS)")
    ap.add_argument("--exchange-rehearsal", action="store_true",
                    help="one GPU: a one-rank RCCL process group and the multi-rank exchange "
                         "(packed all-gather + device merge) on every batch, to exercise that path without a "
                         "multi-GPU node")
    ap.add_argument("--exchange", choices=["packed", "generic"], default="packed",
                    help="N > 1 / rehearsal exchange: packed (the search writes into the rank's packed row, one "
                         "all-gather + lance_hip_merge_topk_packed) or generic (label shift, pack, all-gather, "
                         "unpack copies, lance_hip_merge_topk_device)")
    ap.add_argument("--submit-host-sync", action="store_true",
                    help="pipelined submits wait on the host for torch's stream (an A/B of the default device-side "
                         "ordering, lance_hip_stream_after)")
    ap.add_argument("--no-sync-leg", action="store_true",
                    help="IVF configs: skip the extra synchronous-call leg (kernel traces of the pipelined steps)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: ranks join a gloo group and time a CPU stand-in step "
                         "through the same barrier / max-over-ranks code (tests/test_bench_launcher_cpu.py)")
    ap.add_argument("--recall-queries", type=int, default=None, help="default: the whole batch")
    ap.add_argument("--cpu-threads", type=int, default=None, help="default: every core this job may use")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-recall", action="store_true")
    ap.add_argument("--sample-div", type=int, default=None, help="index option sample_div (default: library's)")
    ap.add_argument("--cand-extra", type=int, default=None, help="index option cand_extra (default: library's)")
    ap.add_argument("--nlist", type=int, default=None, help="IVF configs: num_partitions")
    ap.add_argument("--nprobe", type=int, default=None, help="IVF configs: nprobes")
    ap.add_argument("--m", type=int, default=None, help="IVF_PQ: num_sub_vectors")
    ap.add_argument("--refine", type=int, default=None, help="IVF configs: refine_factor")
    ap.add_argument("--pq-query", dest="pq_query", choices=["fp8", "f32"], default=None,
                    help="IVF_PQ: ADC tables from fp8 (e4m3) or f32 queries (index option pq_query)")
    ap.add_argument("--pq-scan", dest="pq_scan", choices=["fast", "exact_lut"], default=None,
                    help="IVF_PQ: list-major 8-bit-LUT scan or the f32-LUT query-major scan (option pq_scan)")
    ap.add_argument("--refine-sweep", default="1,10,50", help="IVF_PQ: refine factors of the recall sweep")
    ap.add_argument("--api", choices=["device", "host_batch", "per_call"], default="device",
                    help="flat configs, one GPU: device = lance_hip_search_device on resident queries (a step = the "
                         "batch); host_batch = lance_detached_search_batch on host buffers (H2D queries + D2H results "
                         "inside the step); per_call = one lance_detached_search per query, the DuckDB call pattern "
                         "(lance_search.cpp:73-74; a step = one query)")
    ap.add_argument("--inproc", action="store_true",
                    help="flat configs: ONE process drives --gpus N devices through one multi-device handle "
                         "(option devices / LANCE_HIP_DEVICES, shards.cpp) — the form a DuckDB process uses; "
                         "default: one process per GPU")
    ap.add_argument("--inproc-devices", default=None,
                    help="with --inproc: the device list (default 0..N-1; e.g. 0,0 rehearses two shards on one GPU)")
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE",
                    help="extra index option (lance_hip_set_option), repeatable, e.g. --opt scan_i8=off")
    a = ap.parse_args()
    for key, v in CONFIGS[a.config].items():
        if getattr(a, key, None) is None:
            setattr(a, key, v)
    for key in ("index_type", "pq_query", "pq_scan"):
        if not hasattr(a, key) or getattr(a, key) is None:
            setattr(a, key, None)
    return a


def _free_port():
    import socket

    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    return port


def launch_ranks(a):
    """`bench.py --gpus N` with no WORLD_SIZE in the environment: start N fresh
    rank processes (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set,
    RCCL backend), BEFORE this process makes any GPU call; only rank 0's JSON
    line reaches stdout.  Returns the exit status (the first failing rank's)."""
    import subprocess

    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                                      stdout=None if r == 0 else sys.stderr))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for o in live:  # a rank failed: the others would wait in a collective
                    o.terminate()
        time.sleep(0.05)
    return rc


def settle(step, sync, seconds, dist, device):
    """Untimed steps for about `seconds` before the warmup and timed steps (the
    GPU's clock / power state ramps over the first tens of ms of a load:
    profiles/r06e_ramp.jsonl).  Every rank runs the same number of steps (a
    multi-GPU step holds a collective): each times steps 4..8 (past the first
    calls' lazy allocations), the max over ranks sets the count.  Returns the
    steps run."""
    if seconds <= 0:
        return 0
    for _ in range(3):
        step()
    sync()
    t0 = time.perf_counter()
    for _ in range(5):
        step()
    sync()
    est = torch.tensor([(time.perf_counter() - t0) / 5.0], dtype=torch.float64, device=device)
    if dist:
        dist.all_reduce(est, op=dist.ReduceOp.MAX)
    n = int(min(200_000, max(0.0, seconds / max(float(est.item()), 1e-6) - 8)))
    for _ in range(n):
        step()
    sync()
    return n + 8


def timed_steps(step, steps, warmup, dist, device, sync):
    """W untimed steps, then EXACTLY K steps bracketed by a barrier + device sync
    on both sides; returns (max over ranks of the elapsed seconds, the last
    step's result, per-step host marks)."""
    for _ in range(warmup):
        step()
    sync()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    marks = []
    res = None
    for _ in range(steps):
        res = step()
        marks.append(time.perf_counter())
    sync()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=device)
    if dist:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    return float(elapsed.item()), res, np.diff(np.array([t0] + marks)) * 1e3


def main_dry_run(a):
    """--dry-run: the rank launch, process group, barrier and max-over-ranks
    timing of a real run, with a CPU stand-in step on gloo (no GPU, no library)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)
    x = torch.randn(64, 64)

    def step():
        return x @ x

    t, _, _ = timed_steps(step, a.steps, a.warmup, dist, "cpu", lambda: None)
    ranks = torch.tensor([rank], dtype=torch.int64)
    if dist:
        allr = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allr, ranks)
        seen = sorted(int(v.item()) for v in allr)
    else:
        seen = [rank]
    if rank == 0:
        print(json.dumps({"metric": "dry run (launcher check, no GPU)", "value": a.steps / t, "unit": "steps/s",
                          "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": round(1000.0 * t / a.steps, 4), "higher_is_better": True,
                          "scaling": a.scaling, "dry_run": True, "ranks_seen": seen,
                          "pids_differ": bool(dist) and world > 1}), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def gen_rows(start, stop, dim, device, seed=1234, normalize=False):
    """Rows [start, stop) of the synthetic N(0,1) base, identical whatever the
    sharding: chunk c of GEN_CHUNK rows comes from generator seed (seed, c).
    normalize: each row scaled to unit L2 norm (C3)."""
    out = torch.empty((stop - start, dim), dtype=torch.float32, device=device)
    c0, c1 = start // GEN_CHUNK, (stop - 1) // GEN_CHUNK
    g = torch.Generator(device=device)
    for c in range(c0, c1 + 1):
        g.manual_seed(seed * 1_000_003 + c)
        chunk = torch.randn((GEN_CHUNK, dim), generator=g, device=device, dtype=torch.float32)
        lo, hi = max(start, c * GEN_CHUNK), min(stop, (c + 1) * GEN_CHUNK)
        out[lo - start:hi - start] = chunk[lo - c * GEN_CHUNK:hi - c * GEN_CHUNK]
    if normalize:
        out /= torch.linalg.vector_norm(out, dim=1, keepdim=True)
    return out


def cluster_centers(dim, device):
    g = torch.Generator(device=device)
    g.manual_seed(CENT_SEED)
    return torch.randn((NCENT, dim), generator=g, device=device, dtype=torch.float32)


def gen_clustered(start, stop, dim, device, centers, seed=1234):
    """Rows [start, stop) of the clustered base (IVF configs); chunk c from
    generator seed (seed, c) whatever the sharding."""
    out = torch.empty((stop - start, dim), dtype=torch.float32, device=device)
    c0, c1 = start // GEN_CHUNK, (stop - 1) // GEN_CHUNK
    g = torch.Generator(device=device)
    for c in range(c0, c1 + 1):
        g.manual_seed(seed * 1_000_003 + c)
        ids = torch.randint(0, NCENT, (GEN_CHUNK,), generator=g, device=device)
        chunk = torch.randn((GEN_CHUNK, dim), generator=g, device=device, dtype=torch.float32)
        chunk.mul_(SIGMA).add_(centers[ids])
        lo, hi = max(start, c * GEN_CHUNK), min(stop, (c + 1) * GEN_CHUNK)
        out[lo - start:hi - start] = chunk[lo - c * GEN_CHUNK:hi - c * GEN_CHUNK]
    return out


def measured_traffic(n, dim, batch, elem_bytes, kernel=None):
    """Per-launch HBM bytes of the scan kernel from the committed rocprofv3 PMC
    passes (profiles/*_scan_traffic.json, made by tools/pmc_traffic.py from
    separate FETCH_SIZE / WRITE_SIZE runs of this bench) for the same shape."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_scan_traffic.json"))):
        try:
            with open(f) as fh:
                t = json.load(fh)
        except (OSError, ValueError):
            continue
        if (t.get("n"), t.get("dim"), t.get("batch"), t.get("scan_elem_bytes", 4)) == (n, dim, batch, elem_bytes) and \
                (kernel is None or t.get("bench_kernel") == kernel):
            best = t
    return None if best is None else int(best["traffic_bytes_per_launch"])


def ivf_traffic(config, n, dim, batch, kernel=None):
    """Per-launch HBM bytes of the IVF list scan from the committed rocprofv3
    PMC passes of the same config (profiles/*_<config>_ivf_traffic.json, made by
    tools/pmc_passes.sh + tools/pmc_traffic.py)."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{config}_ivf_traffic.json"))):
        try:
            with open(f) as fh:
                t = json.load(fh)
        except (OSError, ValueError):
            continue
        if (t.get("n"), t.get("dim"), t.get("batch")) == (n, dim, batch) and \
                (kernel is None or t.get("bench_kernel") == kernel):
            best = t
    return None if best is None else int(best["traffic_bytes_per_launch"])


def err_buf():
    return ctypes.create_string_buffer(2048)


def host_cpus():
    """The host cores this job may use (affinity mask, capped by a cgroup CPU
    quota when one is set) and what they are: recorded with every CPU baseline."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    usable = min(aff, quota) if quota else aff
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": nproc, "affinity": aff, "cgroup_quota_cpus": quota, "usable": usable, "model": model,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_threads(a):
    return a.cpu_threads or host_cpus()["usable"]


def init_dist(a, world, dev):
    """torch.distributed for N > 1 (nccl = RCCL), or the one-rank nccl group of
    --exchange-rehearsal; None otherwise."""
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)
        return dist
    if a.exchange_rehearsal:
        import socket

        import torch.distributed as dist

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(port))
        dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
        return dist
    return None


def exchange_note(a, world, pipelined):
    if not (a.exchange_rehearsal or world > 1):
        return {}
    return {"exchange": ("rehearsal: one-rank RCCL group, " if world == 1 else "")
            + ("packed: one all-gather of the rank's packed row + lance_hip_merge_topk_packed"
               if a.exchange == "packed" and pipelined else
               "generic: label shift + pack + all-gather + unpack + lance_hip_merge_topk_device") + " per batch"}


def main_ivf(a):
    """IVF configs (C4 IVF-Flat / C5 IVF-PQ of BASELINE.json): every rank holds
    a shard of a.n rows (the 8-GPU configs' 100M rows = 8 x 12.5M), rank 0
    trains the model (lance_detached_create_index), the others install it
    (lance_hip_ivf_set_model) and index their shard; one step = one batch of
    a.batch x world queries through lance_hip_search_batch_device with nprobes /
    refine_factor, per-shard top-k all-gathered and merged on the device."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = init_dist(a, world, dev)
    L = lance_hip.lib()
    N, D, K, B = a.n, a.dim, a.k, a.batch
    s0 = rank * N  # global label offset of this shard
    e = err_buf()
    h = L.lance_create_detached(b"", D, a.metric.encode(), b"bench_ivf", e, 2048)
    if not h:
        raise RuntimeError(e.value.decode())
    lance_hip.LanceHipSetOption(h, "storage", a.storage)
    # IVF_FLAT's bound scan streams the bf16 scan copy (the exact re-rank reads
    # the f32 rows); IVF_PQ scans codes only
    lance_hip.LanceHipSetOption(h, "scan_copy", a.scan_copy if a.index_type == "ivf_flat" else "off")
    lance_hip.LanceHipSetOption(h, "reserve_rows", str(N))
    lance_hip.LanceHipSetOption(h, "index_type", a.index_type)
    if a.index_type == "ivf_pq":
        lance_hip.LanceHipSetOption(h, "pq_query", a.pq_query or "f32")
        lance_hip.LanceHipSetOption(h, "pq_scan", a.pq_scan or "fast")
    for kv in a.opt:
        key, _, val = kv.partition("=")
        lance_hip.LanceHipSetOption(h, key, val)
    centers = cluster_centers(D, dev)
    t_gen = time.perf_counter()
    for lo in range(s0, s0 + N, 1 << 18):
        hi = min(s0 + N, lo + (1 << 18))
        X = gen_clustered(lo, hi, D, dev, centers)
        torch.cuda.synchronize()
        if L.lance_hip_add_batch_device(h, X.data_ptr(), hi - lo, D, e, 2048) < 0:
            raise RuntimeError(e.value.decode())
        del X
    t_build = time.perf_counter()
    if rank == 0:
        if L.lance_detached_create_index(h, a.nlist, a.m, e, 2048) != 0:
            raise RuntimeError(e.value.decode())
    if world > 1:
        nsub = a.m if a.index_type == "ivf_pq" else 0
        dsub = D // nsub if nsub else 0
        Cm = torch.empty((a.nlist, D), dtype=torch.float32, device=dev)
        CB = torch.empty((max(nsub, 1), 256, max(dsub, 1)), dtype=torch.float32, device=dev)
        if rank == 0:
            ex = lance_hip.LanceHipIvfExport(h)
            Cm.copy_(torch.from_numpy(ex["centroids"]))
            if nsub:
                CB.copy_(torch.from_numpy(ex["codebook"]))
        dist.broadcast(Cm, 0)
        dist.broadcast(CB, 0)
        if rank != 0:
            lance_hip.LanceHipIvfSetModel(h, a.index_type, Cm.cpu().numpy(), CB.cpu().numpy() if nsub else None)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t_build
    gen_s = t_build - t_gen
    g = torch.Generator(device=dev)
    g.manual_seed(5678)
    BG = B * world
    qids = torch.randint(0, NCENT, (BG,), generator=g, device=dev)
    Q = (centers[qids] + SIGMA * torch.randn((BG, D), generator=g, device=dev, dtype=torch.float32)).contiguous()
    from lance_hip.sharded import (AsyncPipeline, ShardedPipeline, ShardedSearch, hip_device_merge, hip_device_search,
                                   hip_packed_merge)

    searcher = ShardedSearch(hip_device_search(L, h, D, nprobes=a.nprobe, refine_factor=a.refine),
                             hip_device_merge(L), label_offset=s0, dist=dist, world=world,
                             force_exchange=a.exchange_rehearsal, merge_packed=hip_packed_merge(L))
    torch.cuda.synchronize()

    if a.api != "device" and world > 1:
        raise SystemExit("--api host_batch / per_call: one GPU (the host C-ABI is unsharded)")
    Qh_api = Q.cpu().numpy() if a.api != "device" else None
    call_i = [0]
    # device API: two searches in flight on the handle (lance_hip_search_batch_device_async:
    # the IVF search is enqueued whole, its completion — the fused coarse search's flags,
    # a rerun if one is set — at its wait inside the timed region); --sync: one
    # synchronous call per batch
    pipelined = a.api == "device" and not a.sync
    pipe = None
    if pipelined:
        pipe = AsyncPipeline(L, h, D, nprobes=a.nprobe, refine_factor=a.refine,
                             packed=(world > 1 or a.exchange_rehearsal) and a.exchange == "packed",
                             label_offset=s0, host_sync=a.submit_host_sync)
        if world > 1 or a.exchange_rehearsal:
            pipe = ShardedPipeline(pipe, searcher)
    last_out = [None]

    def step():
        if a.api == "host_batch":
            return lance_hip.LanceDetachedSearchBatch(h, Qh_api, K)
        if a.api == "per_call":
            i = call_i[0] % BG
            call_i[0] += 1
            return lance_hip.LanceDetachedSearch(h, Qh_api[i], D, K)
        if pipelined:
            r = pipe.step(Q, K)
            last_out[0] = r if r is not None else last_out[0]
            return r
        return searcher.search(Q, K, reuse_outputs=True)

    def sync():
        if pipelined:
            r = pipe.drain()
            last_out[0] = r if r is not None else last_out[0]
        torch.cuda.synchronize()

    settled = settle(step, sync, a.settle_s, dist, dev)
    for _ in range(a.warmup):
        step()
    sync()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = step()
    sync()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    t = float(elapsed.item())
    if pipelined:
        res = tuple(x.clone() for x in last_out[0])
    sync_leg = None
    if pipelined and world == 1 and not a.no_sync_leg:
        # the synchronous call beside it (one lance_hip_search_batch_device per batch)
        ts, rs, _ = timed_steps(lambda: searcher.search(Q, K, reuse_outputs=True), a.steps, a.warmup, None, dev,
                                torch.cuda.synchronize)
        sync_leg = {"value": round(BG * a.steps / ts, 1), "unit": "queries/s",
                    "ms_per_step": round(1000.0 * ts / a.steps, 4),
                    "api": "lance_hip_search_batch_device, one synchronous call per batch",
                    "ids_equal_pipelined": bool(np.array_equal(rs[0].cpu().numpy(), res[0].cpu().numpy()))}
    lance_hip.LanceHipSetOption(h, "time_kernels", "1")
    for _ in range(max(3, min(a.steps, 10))):
        step()
    torch.cuda.synchronize()
    kt = lance_hip.LanceHipKernelTimes(h)
    lance_hip.LanceHipSetOption(h, "time_kernels", "0")
    res_l = res[0].cpu().numpy()

    # the list-major 8-bit-LUT scan runs for m <= 96 and k * refine <= 512 (ivf.h FQ_MAX_M / FQ_MAX_KK)
    fast_pq = a.index_type == "ivf_pq" and (a.pq_scan or "fast") == "fast" and a.m <= 96 and K * a.refine <= 512
    recall = cpu = None
    recall_sweep = {}
    if rank == 0 and world == 1 and not a.no_recall:
        from oracle import c_oracle, flat_knn, ivf

        Xh = np.empty((N, D), np.float32)
        for lo in range(0, N, 1 << 18):
            hi = min(N, lo + (1 << 18))
            Xh[lo:hi] = gen_clustered(lo, hi, D, dev, centers).cpu().numpy()
        Qh = Q.cpu().numpy()
        nr = min(a.recall_queries or B, B)
        nthreads = cpu_threads(a)
        el, _, _ = c_oracle.flat_search_batch(Xh, Qh[:nr], K, a.metric, acc64=True, nthreads=nthreads)
        recall = flat_knn.recall_at_k(res_l[:nr], el, min(10, K))
        if a.index_type == "ivf_pq":
            # recall@10 against the refine factor (the exact re-rank window), same batch
            for rf in [int(x) for x in a.refine_sweep.split(",") if x]:
                sl = torch.empty((BG, K), dtype=torch.int64, device=dev)
                sd = torch.empty((BG, K), dtype=torch.float32, device=dev)
                sc = torch.empty((BG,), dtype=torch.int32, device=dev)
                r = L.lance_hip_search_batch_device(h, Q.data_ptr(), BG, D, K, a.nprobe, rf, sl.data_ptr(),
                                                    sd.data_ptr(), sc.data_ptr(), e, 2048)
                if r < 0:
                    raise RuntimeError(e.value.decode())
                torch.cuda.synchronize()
                recall_sweep[str(rf)] = flat_knn.recall_at_k(sl.cpu().numpy()[:nr], el, min(10, K))
        if not a.no_cpu_baseline:
            # the same IVF search on the host (oracle/flat_knn.c's IVF port over the
            # model and lists the GPU built), one query per call, f32 distances
            ex = lance_hip.LanceHipIvfExport(h)
            lay = c_oracle.IvfLayout(ex["lists"], ex["live"], a.nlist)
            kw = {}
            if a.index_type == "ivf_pq":
                _, T = ivf.pq_tables(ex["centroids"], ex["codebook"], Qh[:1], a.metric)
                kw = dict(codes=ex["codes"], codebook=ex["codebook"], T=T, refine_factor=a.refine,
                          lut="u8" if fast_pq else "f32", query_fp8=a.pq_query == "fp8")
            done, tc0 = 0, time.perf_counter()
            agree = 0
            while True:
                cl, _, _ = c_oracle.ivf_search_batch(Xh, ex["labels"], lay, ex["centroids"], Qh[done % B:done % B + 1],
                                                     K, a.nprobe, a.metric, acc64=False, nthreads=nthreads, **kw)
                agree += int(np.intersect1d(cl[0], res_l[done % B]).size)
                done += 1
                if time.perf_counter() - tc0 >= a.cpu_seconds and done >= 2:
                    break
            tcpu = time.perf_counter() - tc0
            cpu = {"value": done / tcpu, "unit": "queries/s", "cores": nthreads, "kind": "port",
                   "sample": f"{done} queries, one per call, {a.index_type} nprobes={a.nprobe} over the GPU-built "
                             f"model and lists of {N}x{D} rows, f32 distances ({tcpu:.1f} s, oracle/flat_knn.c IVF "
                             f"port, {nthreads} OpenMP threads)",
                   "id_overlap_with_gpu": round(agree / (done * K), 4), "host": host_cpus()}
        del Xh

    if rank == 0:
        value = BG * a.steps / t
        roof = None
        if kt["ivf_scan_launches"] > 0:
            avg_ms = kt["ivf_scan_ms_total"] / kt["ivf_scan_launches"]
            bytes_launch = kt["ivf_scan_bytes"] / kt["ivf_scan_launches"]
            ach = bytes_launch / (avg_ms * 1e-3) / 1e9
            bound_flat = a.index_type == "ivf_flat" and a.scan_copy == "on" and K <= 15 and \
                "ivf_flat_scan=exact" not in a.opt
            kname = (("flat_list_lb_kernel" if bound_flat else "flat_list_scan_kernel") if a.index_type == "ivf_flat" else
                     ("pq_fast_scan_bank_kernel" if a.m in (32, 64, 96) and os.environ.get("LANCE_HIP_PQ_LANE_ROWS") != "1"
                      else "pq_fast_scan_kernel") if fast_pq else "pq_query_scan_kernel")
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": ivf_traffic(a.config, N, D, BG, kname), "kernel": kname,
                    "avg_launch_ms": round(avg_ms, 4), "bytes_per_launch": int(bytes_launch),
                    "pair_rows_per_launch": int(kt["ivf_pair_rows"] / kt["ivf_scan_launches"]),
                    "coarse_ms_per_batch": round(kt["ivf_coarse_ms_total"] / kt["ivf_scan_launches"], 4)}
        what = "IVF-Flat" if a.index_type == "ivf_flat" else f"IVF-PQ m={a.m} nbits=8"
        line = {
            "metric": f"kNN queries/sec + recall@10, {what} nlist={a.nlist} nprobe={a.nprobe}, {N}x{D} f32 per GPU",
            "value": round(value, 1), "unit": "queries/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "settle": {"steps": settled, "seconds": a.settle_s},
            "ms_per_step": round(1000.0 * t / a.steps, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": a.storage,
            "data": f"synthetic clustered rows: {NCENT} Gaussian clusters (centers N(0,1), sigma {SIGMA}), queries "
                    "drawn the same way (seeded torch Philox)",
            "config": {"workload": f"{a.config.upper()} {what} nlist={a.nlist} nprobe={a.nprobe} refine={a.refine} "
                                   f"{N}x{D} f32 per GPU k={K} query-batch={BG}",
                       "n_per_gpu": N, "n_total": N * world, "dim": D, "k": K, "global_batch": BG,
                       "metric": a.metric, "index_type": a.index_type, "nlist": a.nlist, "nprobe": a.nprobe,
                       "m": a.m, "refine_factor": a.refine, "parallelism": f"rowshard{world}",
                       **exchange_note(a, world, pipelined),
                       **({"pq_query": a.pq_query or "f32", "pq_scan": a.pq_scan or "fast"}
                          if a.index_type == "ivf_pq" else {}),
                       **({"options": a.opt} if a.opt else {})},
            "recall_at_10": recall,
            **({"recall_at_10_by_refine": recall_sweep} if recall_sweep else {}),
            "roofline": roof,
            "cpu_baseline": cpu,
            **({"sync": sync_leg} if sync_leg else {}),
            "build_s": round(build_s, 2), "gen_s": round(gen_s, 2),
        }
        print(json.dumps(line), flush=True)
    L.lance_free_detached(h)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def main_c1(a):
    """C1 (BASELINE.json configs[0]): 10k x 128 f32, k = 10, one query per call
    through lance_detached_search with host query / result buffers — the
    lance_search() call pattern (lance_search.cpp:73-74 -> rust_ffi.cpp:130-139).
    Latency-bound by construction (one 5 MB dense scan per call); a step = one
    call.  Single GPU only."""
    from oracle import c_oracle

    torch.cuda.set_device(0)
    L = lance_hip.lib()
    N, D, K = a.n, a.dim, a.k
    rng = np.random.default_rng(1234)
    X = rng.standard_normal((N, D), dtype=np.float32)
    Q = np.random.default_rng(5678).standard_normal((max(a.steps, 64), D), dtype=np.float32)
    h = lance_hip.LanceCreateDetached("", D, a.metric, "c1")
    lance_hip.LanceDetachedAddBatch(h, X, N, D)
    ci = [0]

    def one():
        lance_hip.LanceDetachedSearch(h, Q[ci[0] % len(Q)], D, K)
        ci[0] += 1

    settled = settle(one, lambda: None, a.settle_s, None, "cpu")
    for i in range(a.warmup):
        lance_hip.LanceDetachedSearch(h, Q[i % len(Q)], D, K)
    got = []
    t0 = time.perf_counter()
    for i in range(a.steps):
        got.append(lance_hip.LanceDetachedSearch(h, Q[i % len(Q)], D, K)[0])
    t = time.perf_counter() - t0
    lance_hip.LanceHipSetOption(h, "time_kernels", "1")
    for i in range(10):
        lance_hip.LanceDetachedSearch(h, Q[i], D, K)
    kt = lance_hip.LanceHipKernelTimes(h)
    small = lance_hip.LanceHipLastSearchStats(h)["small_exact"]
    nthreads = cpu_threads(a)
    nr = min(16, a.steps)
    el, _, _ = c_oracle.flat_search_batch(X, Q[:nr], K, a.metric, acc64=True, nthreads=nthreads)
    exact = all((got[i] == el[i]).all() for i in range(nr))
    done, tc0 = 0, time.perf_counter()
    while time.perf_counter() - tc0 < min(a.cpu_seconds, 5.0) or done < 2:
        c_oracle.flat_search_batch(X, Q[done % len(Q):done % len(Q) + 1], K, a.metric, acc64=False, nthreads=nthreads)
        done += 1
    tcpu = time.perf_counter() - tc0
    roof = None
    if kt["dense_launches"]:
        ms = kt["dense_ms_total"] / kt["dense_launches"]
        ld = ((D + 63) // 64) * 64
        if small:
            # one-launch exact search: every row's dim f32 elements, its row-aux
            # word and label (f32 store, the small path reads the rows themselves)
            byts = N * (D * 4 + 4 + 8)
            kern = f"small_exact_kernel<{a.metric.upper()},f32>"
        else:
            byts = ((N + 255) // 256 * 256) * (ld * kt["scan_elem_bytes"] + 16) + 256 * ld * 2
            kern = "scan_kernel<L2,dense,bf16>"
        roof = {"bound": "hbm", "achieved": round(byts / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(byts / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": kern, "avg_launch_ms": round(ms, 4), "bytes_per_launch": int(byts),
                "note": "a 10k-row store is one short launch: latency, not bandwidth, sets the call time"}
    line = {"metric": "lance_search() queries/sec, 10kx128 f32 flat L2 k=10, one query per call (C1)",
            "value": round(a.steps / t, 1), "unit": "queries/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
            "settle": {"steps": settled, "seconds": a.settle_s},
            "ms_per_step": round(1000.0 * t / a.steps, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic N(0,1) rows and queries (numpy default_rng)",
            "config": {"workload": "C1 flat l2 10000x128 f32 k=10, lance_detached_search per query (host buffers)",
                       "n": N, "dim": D, "k": K, "global_batch": 1, "parallelism": "single"},
            "exact_ids": exact, "roofline": roof,
            "cpu_baseline": {"value": done / tcpu, "unit": "queries/s", "cores": nthreads, "kind": "port",
                             "sample": f"{done} queries, one per call, exact f32 l2 over {N}x{D} "
                                       f"({tcpu:.1f} s, oracle/flat_knn.c, {nthreads} OpenMP threads)"}}
    print(json.dumps(line), flush=True)
    lance_hip.LanceFreeDetached(h)


def main():
    a = parse()
    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1 and not a.inproc:
        # one process per GPU, started here (the driver may also start them with
        # torch.distributed.run, which sets WORLD_SIZE)
        return launch_ranks(a)
    if a.inproc and env_world is not None and int(env_world) > 1:
        raise SystemExit("--inproc: one process for every device (do not launch ranks)")
    if env_world is not None and int(env_world) != a.gpus and not a.inproc:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={env_world}: launch one rank per GPU")
    if a.dry_run:
        return main_dry_run(a)
    _load_lib()
    if a.config == "c1":
        return main_c1(a)
    if a.index_type:
        return main_ivf(a)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = init_dist(a, world, dev)
    L = lance_hip.lib()

    N, D, K, B = a.n, a.dim, a.k, a.batch
    s0, s1 = rank * N // world, (rank + 1) * N // world
    n_local = s1 - s0

    # ---- build the shard (device-resident base) --------------------------
    e = err_buf()
    h = L.lance_create_detached(b"", D, a.metric.encode(), b"bench", e, 2048)
    if not h:
        raise RuntimeError(e.value.decode())
    inproc_devs = None
    if a.inproc:
        inproc_devs = a.inproc_devices or ",".join(str(i) for i in range(a.gpus))
        if len(inproc_devs.split(",")) > 1:
            lance_hip.LanceHipSetOption(h, "devices", inproc_devs)
    lance_hip.LanceHipSetOption(h, "storage", a.storage)
    lance_hip.LanceHipSetOption(h, "scan_copy", a.scan_copy)
    lance_hip.LanceHipSetOption(h, "reserve_rows", str(n_local))
    if a.sample_div:
        lance_hip.LanceHipSetOption(h, "sample_div", str(a.sample_div))
    if a.cand_extra:
        lance_hip.LanceHipSetOption(h, "cand_extra", str(a.cand_extra))
    for kv in a.opt:
        key, _, val = kv.partition("=")
        lance_hip.LanceHipSetOption(h, key, val)
    for lo in range(s0, s1, 1 << 18):
        hi = min(s1, lo + (1 << 18))
        X = gen_rows(lo, hi, D, dev, normalize=a.normalize)
        torch.cuda.synchronize()
        r = L.lance_hip_add_batch_device(h, X.data_ptr(), hi - lo, D, e, 2048)
        if r < 0:
            raise RuntimeError(e.value.decode())
        del X
    # index preparation (outside any timing): the int8 scan copy is derived from the rows
    lance_hip.LanceHipSetOption(h, "prepare", "1")
    g = torch.Generator(device=dev)
    g.manual_seed(5678)
    # global batch: strong (default) = B in all, weak = B per rank (per-GPU flops fixed)
    BG = B * world if a.scaling == "weak" else B
    Q = torch.randn((BG, D), generator=g, device=dev, dtype=torch.float32)
    if a.normalize:
        Q /= torch.linalg.vector_norm(Q, dim=1, keepdim=True)
    from lance_hip.sharded import (AsyncPipeline, ShardedPipeline, ShardedSearch, hip_device_merge, hip_device_search,
                                   hip_packed_merge)

    searcher = ShardedSearch(hip_device_search(L, h, D), hip_device_merge(L), label_offset=s0, dist=dist,
                             world=world, force_exchange=a.exchange_rehearsal, merge_packed=hip_packed_merge(L))
    torch.cuda.synchronize()

    if a.api != "device" and world > 1:
        raise SystemExit("--api host_batch / per_call: one GPU (the host C-ABI is unsharded)")
    Qh_api = Q.cpu().numpy() if (a.api != "device" or (world == 1 and not a.no_host_batch)) else None
    call_i = [0]

    # device API: two batches in flight per rank (lance_hip_search_batch_device_async;
    # every batch completes — certified, reruns / fallbacks done — at its wait
    # inside the timed region; N > 1: batch i-1's all-gather + merge run while
    # batch i scans); --sync: one synchronous call (+ exchange) per batch
    pipelined = a.api == "device" and not a.sync
    pipe = None
    if pipelined:
        pipe = AsyncPipeline(L, h, D, packed=(world > 1 or a.exchange_rehearsal) and a.exchange == "packed",
                             label_offset=s0, host_sync=a.submit_host_sync)
        if world > 1 or a.exchange_rehearsal:
            pipe = ShardedPipeline(pipe, searcher)
    last_out = [None]

    def step():
        if a.api == "host_batch":
            return lance_hip.LanceDetachedSearchBatch(h, Qh_api, K)
        if a.api == "per_call":
            i = call_i[0] % BG
            call_i[0] += 1
            return lance_hip.LanceDetachedSearch(h, Qh_api[i], D, K)
        if pipelined:
            r = pipe.step(Q, K)
            last_out[0] = r if r is not None else last_out[0]
            return r
        return searcher.search(Q, K, reuse_outputs=True)

    def sync():
        if pipelined:
            r = pipe.drain()
            last_out[0] = r if r is not None else last_out[0]
        torch.cuda.synchronize()

    # settle (clocks), then warmup; for per_call the timed calls then start at
    # query 0 (the recall subset below)
    settled = settle(step, sync, a.settle_s, dist, dev)
    for _ in range(a.warmup):
        step()
    sync()
    call_i[0] = 0
    per_call_l = []

    def step_rec():
        r = step()
        if a.api == "per_call" and len(per_call_l) < BG:
            per_call_l.append(r[0])
        return r

    t, res, per = timed_steps(step_rec, a.steps, 0, dist, dev, sync)
    if pipelined:
        res = last_out[0]
    if a.api == "device":  # (the output buffers are reused by the legs below)
        res = tuple(x.clone() for x in res)
    st = lance_hip.LanceHipLastSearchStats(h)
    print(f"[bench] per-step ms: min {per.min():.4f} median {np.median(per):.4f} max {per.max():.4f}", file=sys.stderr)
    # extra legs (never `value`): the other multi-GPU scaling mode, and at N = 1
    # the host-buffer C-ABI (H2D queries + D2H results inside the step: SURVEY.md
    # §8(d)'s QPS definition) beside the device-resident figure
    other = None
    if world > 1 and a.api == "device" and not a.no_other_scaling:
        om = "weak" if a.scaling == "strong" else "strong"
        BO = B * world if om == "weak" else B
        Qo = torch.randn((BO, D), generator=g, device=dev, dtype=torch.float32)
        if a.normalize:
            Qo /= torch.linalg.vector_norm(Qo, dim=1, keepdim=True)
        to, _, _ = timed_steps(lambda: searcher.search(Qo, K), a.steps, a.warmup, dist, dev, torch.cuda.synchronize)
        other = {"scaling": om, "value": round(BO * a.steps / to, 1), "unit": "queries/s",
                 "ms_per_step": round(1000.0 * to / a.steps, 4), "global_batch": BO,
                 "rows_per_gpu": n_local}
        del Qo
    syncleg = None
    if pipelined:
        ts, rs, _ = timed_steps(lambda: searcher.search(Q, K, reuse_outputs=True), a.steps, a.warmup, dist, dev,
                                torch.cuda.synchronize)
        syncleg = {"value": round(BG * a.steps / ts, 1), "unit": "queries/s", "ms_per_step": round(1000.0 * ts / a.steps, 4),
                   "api": "lance_hip_search_batch_device, one synchronous call per batch",
                   "ids_equal_pipelined": bool((rs[0].cpu() == res[0].cpu()).all())}
    hostb = None
    if world == 1 and a.api == "device" and not a.no_host_batch:
        th, rh, _ = timed_steps(lambda: lance_hip.LanceDetachedSearchBatch(h, Qh_api, K), a.steps, a.warmup, None,
                                dev, torch.cuda.synchronize)
        hostb = {"value": round(BG * a.steps / th, 1), "unit": "queries/s", "ms_per_step": round(1000.0 * th / a.steps, 4),
                 "api": "lance_detached_search_batch (host query / result buffers, H2D + D2H timed)",
                 "ids_equal_device": bool((rh[0] == res[0].cpu().numpy()).all())}
    # the scan kernel's own duration (HIP events on the stream it runs on),
    # from separate steps so the event calls stay out of the timed loop above
    lance_hip.LanceHipSetOption(h, "time_kernels", "1")
    for _ in range(max(3, min(a.steps, 10))):
        step()
    sync()
    kt = lance_hip.LanceHipKernelTimes(h)
    lance_hip.LanceHipSetOption(h, "time_kernels", "0")
    if a.api == "device":
        res_l = res[0].cpu().numpy()
        res_d = res[1].cpu().numpy()
    elif a.api == "host_batch":
        res_l, res_d = res[0], res[1]
    else:  # per call: the results of the first calls, one query each
        res_l = np.stack(per_call_l)
        res_d = None

    # ---- recall@10 vs exact (CPU oracle, float64) on a query subset ----------
    recall = None
    cpu = None
    if rank == 0 and not a.no_recall:
        sys.path.insert(0, ROOT)
        from oracle import c_oracle, flat_knn

        Xh = np.empty((N, D), np.float32)
        for lo in range(0, N, 1 << 18):
            hi = min(N, lo + (1 << 18))
            Xr = gen_rows(lo, hi, D, dev, normalize=a.normalize)
            if a.storage == "bf16":  # the stored rows: nearest-even bf16 of the added rows
                Xr = Xr.to(torch.bfloat16).float()
            Xh[lo:hi] = Xr.cpu().numpy()
            del Xr
        Qh = Q.cpu().numpy()
        nr = min(a.recall_queries or BG, BG, len(res_l))
        nthreads = cpu_threads(a)
        el, ed, _ = c_oracle.flat_search_batch(Xh, Qh[:nr], K, a.metric, acc64=True, nthreads=nthreads)
        recall = flat_knn.recall_at_k(res_l[:nr], el, min(10, K))
        recall_k = flat_knn.recall_at_k(res_l[:nr], el, K)
        exact_ids = bool((res_l[:nr] == el).all())
        max_rel = (float(np.max(np.abs(res_d[:nr] - ed) / np.maximum(np.abs(ed), 1e-30)))
                   if res_d is not None else None)
        if world == 1 and not a.no_cpu_baseline:
            # bounded sample: one query per call (the reference API, lance_search.cpp:73-74)
            done, t_cpu0 = 0, time.perf_counter()
            while True:
                c_oracle.flat_search_batch(Xh, Qh[done % B:done % B + 1], K, a.metric, acc64=False,
                                           nthreads=nthreads)
                done += 1
                if time.perf_counter() - t_cpu0 >= a.cpu_seconds and done >= 2:
                    break
            t_cpu = time.perf_counter() - t_cpu0
            # batched leg: one call for a block of queries (each 64-row block of the
            # base reused from cache by every query of the call), bounded likewise
            nbq = 8
            while True:
                tb0 = time.perf_counter()
                c_oracle.flat_search_batch(Xh, Qh[:nbq], K, a.metric, acc64=False, nthreads=nthreads)
                t_b = time.perf_counter() - tb0
                if t_b >= a.cpu_seconds / 3 or nbq >= B:
                    break
                nbq = min(B, nbq * 4)
            cpu = {"value": done / t_cpu, "unit": "queries/s", "cores": nthreads, "kind": "port",
                   "sample": f"{done} queries, one per call (the reference API), each an exact f32 {a.metric} scan "
                             f"of all {N}x{D} rows ({t_cpu:.1f} s, oracle/flat_knn.c, {nthreads} OpenMP threads)",
                   "batched": {"value": nbq / t_b, "unit": "queries/s", "queries_per_call": nbq,
                               "seconds": round(t_b, 2)},
                   "host": host_cpus()}
        del Xh

    if rank == 0:
        ms_step = 1000.0 * t / a.steps
        value = (1 if a.api == "per_call" else BG) * a.steps / t
        roof = None
        if kt["scan_launches"] > 0:
            ld = ((D + 63) // 64) * 64
            esz = kt.get("scan_elem_bytes") or (2 if a.storage == "bf16" else 4)
            avg_ms = kt["scan_ms_total"] / kt["scan_launches"]
            # algorithmic bytes per launch: every base row (ld elements + 16 B row aux) + the query tile
            # (bf16; int8 with the int8 scan copy)
            if kt["scan_kernel"] == "scan8_kernel":
                # scan8 reads, per row, its int8 k-chunks and its alpha (the other row
                # terms are per 256-row tile: 16 B), and the int8 query tile once
                tiles = (kt["scan_rows"] + 255) // 256
                bytes_launch = kt["scan_rows"] * (ld + 4) + tiles * 16 + kt["scan_qpad"] * ld
            else:
                bytes_launch = kt["scan_rows"] * (ld * esz + 16) + kt["scan_qpad"] * ld * (1 if esz == 1 else 2)
            xname = {1: "i8", 2: "bf16"}.get(esz, "f32")
            # dense MFMA peak of the scan's operand type (int8: 2x bf16)
            mfma_peak = MFMA_BF16_PEAK_TFS * (2 if esz == 1 else 1)
            ach = bytes_launch / (avg_ms * 1e-3) / 1e9
            kstr = f"{kt['scan_kernel']}<{ {'l2': 'L2', 'dot': 'DOT', 'cosine': 'COSINE'}[a.metric]},append,{xname}>"
            # (per store: a rank's shard, or with --inproc one of the handle's device stores)
            n_stores = world * (len(inproc_devs.split(",")) if inproc_devs else 1)
            traffic = measured_traffic(N // n_stores, D, BG, esz, kstr)
            mfma_tfs = 2.0 * kt["scan_rows"] * D * BG / (avg_ms * 1e-3) / 1e12
            kname = {"l2": "L2", "dot": "DOT", "cosine": "COSINE"}[a.metric]
            # the bounding roof: HBM time of the bytes vs dense-bf16 MFMA time of the flops
            # (N = 1: HBM; at N > 1 a 1/N shard meets N x the queries and MFMA can bind)
            mfma_bound = (2.0 * kt["scan_rows"] * D * BG) / (mfma_peak * 1e12) > bytes_launch / (HBM_PEAK_GBS * 1e9)
            if mfma_bound:
                roof = {"bound": "mfma", "achieved": round(mfma_tfs, 1), "peak": mfma_peak, "unit": "TFLOP/s",
                        "frac": round(mfma_tfs / mfma_peak, 4), "traffic": traffic,
                        "hbm_gbs": round(ach, 1), "hbm_frac": round(ach / HBM_PEAK_GBS, 4)}
            else:
                roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic}
            # context only (never `achieved`): the rate at which the scan covers the f32 base's own bytes
            roof["f32_equivalent_gbs"] = round(kt["scan_rows"] * ld * 4 / (avg_ms * 1e-3) / 1e9, 1)
            roof.update({
                    "kernel": f"{kt['scan_kernel']}<{kname},append,{xname}>",
                    "avg_launch_ms": round(avg_ms, 4), "bytes_per_launch": int(bytes_launch),
                    "mfma_tflops": round(mfma_tfs, 1), "mfma_frac": round(mfma_tfs / mfma_peak, 4)})
        api_note = {"device": "", "host_batch": ", lance_detached_search_batch on host buffers (H2D + D2H timed)",
                    "per_call": ", one lance_detached_search per query (host buffers; the DuckDB call pattern)"}[a.api]
        if a.config == "c2":
            metric_name = "kNN queries/sec + recall@10, 1Mx768 f32 flat; GB/s vs HBM roofline"
        elif a.config == "nstar":
            metric_name = f"kNN queries/sec + recall@10, {N // 1_000_000}Mx{D} f32 flat L2 (north_star); GB/s vs HBM roofline"
        else:
            metric_name = (f"kNN queries/sec + recall@{K}, {N // 1_000_000}Mx{D} {a.storage} flat "
                           f"{'IP' if a.metric == 'dot' else a.metric}; GB/s vs HBM roofline")
        line = {
            "metric": metric_name,
            "value": round(value, 1),
            "unit": "queries/s",
            "n_gpus": len(inproc_devs.split(",")) if inproc_devs else world,
            "steps": a.steps,
            "warmup": a.warmup,
            "settle": {"steps": settled, "seconds": a.settle_s,
                       "why": "untimed steps before the warmup: the GPU clocks up over its first ~50 steps"},
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": a.storage,
            "data": "synthetic N(0,1) base (seeded torch Philox), independent N(0,1) queries"
                    + (", rows and queries L2-normalized; base stored as bf16 (RNE)" if a.config == "c3" else ""),
            "config": {"workload": f"{a.config.upper()} flat {a.metric} {N}x{D} {a.storage} k={K} "
                                   f"query-batch={1 if a.api == 'per_call' else BG}{api_note}",
                       "api": a.api,
                       "n": N, "dim": D, "k": K, "global_batch": BG, "batch_per_gpu": B, "metric": a.metric, "storage": a.storage,
                       "parallelism": (f"inproc-rowshard{len(inproc_devs.split(','))}" if inproc_devs
                                       else f"rowshard{world}"),
                       **({"devices": inproc_devs} if inproc_devs else {}),
                       **exchange_note(a, world, pipelined),
                       "scan_copy": a.scan_copy,
                       **({"options": a.opt} if a.opt else {})},
            "recall_at_10": recall,
            "recall_queries": None if recall is None else nr,
            "roofline": roof,
            "cpu_baseline": cpu,
            "search_stats": st,
        }
        if other:
            line[f"{other['scaling']}_scaling"] = other
        if pipelined and inproc_devs:
            line["config"]["pipeline"] = ("multi-device handle: every shard's pass enqueued before the first wait "
                                          "(shards scan concurrently), partial lists merged on the first device")
            line["sync"] = syncleg
        elif pipelined:
            line["config"]["pipeline"] = ("async: 2 batches in flight on the handle's stream "
                                          "(lance_hip_search_batch_device_async / lance_hip_search_wait)"
                                          + ("; batch i-1's all-gather + merge overlap batch i's scan" if world > 1 else ""))
            line["sync"] = syncleg
        if hostb:
            line["host_batch"] = hostb
            # SURVEY.md §8(d)'s QPS: the C-ABI search_batch wall time WITH the H2D of the
            # queries and the D2H of the results (base resident); `value` is device-resident
            line["qps_8d"] = {"value": hostb["value"], "unit": "queries/s",
                              "definition": "lance_detached_search_batch on host buffers, H2D + D2H timed (SURVEY §8d)"}
        if recall is not None:
            line[f"recall_at_{K}"] = recall_k
            line["exact_ids_on_recall_subset"] = exact_ids
            line["max_rel_dist_err"] = max_rel
        print(json.dumps(line), flush=True)
    L.lance_free_detached(h)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
