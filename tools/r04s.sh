#!/bin/bash
# IVF_PQ fast scan: seeded bounds (release) parity + C5 line; phase stamps of the seeded
# scan and of timing ablations (no liveness read, no lookups) and 48-lookup batches
source tools/gpu_step.sh
T=${1:-r04s}
step ${T}_pytest 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ivf_params.py tests/test_gpu_ivf.py
step ${T}_bench_c5 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
for v in pqprof pq_lb3 pq_noalive pq_nolookup; do
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_$v.so step ${T}_$v 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-recall
done
