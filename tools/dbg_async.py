import sys, numpy as np, torch
sys.path.insert(0, "duckdb-lancedb_amd"); sys.path.insert(0, ".")
import lance_hip as hip
from lance_hip.sharded import AsyncPipeline
torch.cuda.init()
rng = np.random.default_rng(505)
n, d, k = 120_000, 128, 10
X = rng.standard_normal((n, d), dtype=np.float32)
QA = rng.standard_normal((65, d), dtype=np.float32)
QB = rng.standard_normal((256, d), dtype=np.float32)
h = hip.LanceCreateDetached("", d, "cosine", "t")
hip.LanceDetachedAddBatch(h, X, n, d)
hip.LanceHipSetOption(h, "sample_div", "100000")
hip.LanceDetachedSearchBatch(h, QA, k); print("sync", hip.LanceHipLastSearchStats(h))
pipe = AsyncPipeline(hip.lib(), h, d)
tA = pipe.submit(torch.from_numpy(QA).cuda(), k); print("after submit A", hip.LanceHipLastSearchStats(h))
tB = pipe.submit(torch.from_numpy(QB).cuda(), k); print("after submit B", hip.LanceHipLastSearchStats(h))
pipe.wait(tA); print("after wait A", hip.LanceHipLastSearchStats(h))
pipe.wait(tB); print("after wait B", hip.LanceHipLastSearchStats(h))
tA = pipe.submit(torch.from_numpy(QA).cuda(), k); pipe.wait(tA); print("A alone", hip.LanceHipLastSearchStats(h))
