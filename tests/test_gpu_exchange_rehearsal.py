"""GPU: the multi-rank exchange on a real RCCL process group.

The driver's N > 1 runs (one rank per GPU) have each rank's search write its
top-k lists into one packed int32 row, all-gather the rows over RCCL
(``ShardedSearch.exchange``) and merge them with ``lance_hip_merge_topk_packed``
(``--exchange generic``: pack with torch ops, ``lance_hip_merge_topk_device``).
The one-GPU boxes of this pool cannot
start two RCCL ranks on one device, so ``bench.py --exchange-rehearsal`` runs a
one-rank ``nccl`` group and forces that exchange on every pipelined batch: the
packed rows, ``all_gather_into_tensor`` on device tensors and the device
merge all run on the GPU, and the ids must stay exact."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("exchange", ["packed", "generic"])
def test_bench_exchange_rehearsal_keeps_exact_ids(exchange):
    env = dict(os.environ)
    for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--n", "300000", "--steps", "6", "--warmup", "2",
                        "--settle-s", "0", "--no-cpu-baseline", "--no-host-batch", "--recall-queries", "64",
                        "--exchange-rehearsal", "--exchange", exchange],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["config"]["exchange"].startswith("rehearsal: one-rank RCCL group, " + exchange)
    assert line["recall_at_10"] == 1.0
    assert line["exact_ids_on_recall_subset"] is True
