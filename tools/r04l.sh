#!/bin/bash
# round 4 (session 2): full GPU suite with one HIP runtime per process; pool_refine /
# scan8 phase stamps at C2 (diagnostic builds); north_star, C3 and per-rank shapes
source tools/gpu_step.sh
T=${1:-r04l}
step ${T}_pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_prprof.so step ${T}_prprof 200 python -u bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_s8prof.so step ${T}_s8prof 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-recall --no-host-batch --sync
step ${T}_bench_nstar 300 python -u bench.py --config nstar --steps 10 --recall-queries 64 --no-cpu-baseline --no-host-batch
step ${T}_rank_c2s8 200 python -u bench.py --n 125000 --steps 30 --no-cpu-baseline --no-host-batch
step ${T}_rank_nstar8 200 python -u bench.py --n 1250000 --steps 30 --no-cpu-baseline --no-host-batch
step ${T}_bench_c3 400 python -u bench.py --config c3 --steps 10 --recall-queries 64 --no-cpu-baseline --no-host-batch
