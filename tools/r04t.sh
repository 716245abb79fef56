#!/bin/bash
# IVF_PQ fast scan with two code buffers (no per-round wait on its own prefetch): parity,
# C5 line + phases; then the round-4 PMC traffic passes of every config's dominant kernel
source tools/gpu_step.sh
T=${1:-r04t}
step ${T}_pytest 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ivf_params.py tests/test_gpu_ivf.py
step ${T}_bench_c5 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_pqprof.so step ${T}_pqprof 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-recall
step ${T}_pmc 1000 bash tools/r04_pmc.sh
