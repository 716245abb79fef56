#!/bin/bash
# cold-row gather probe; scan8 phases at C2 (printf-light profile build); C2 / north_star with auto sample_div
source tools/gpu_step.sh
T=${1:-r04j}
step ${T}_probe_cold 120 duckdb-lancedb_amd/lib_dev/gather_probe 1000000 1 1
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_s8prof.so step ${T}_s8prof 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-recall --no-host-batch --sync
step ${T}_bench_c2 200 python -u bench.py --steps 30 --no-cpu-baseline
step ${T}_bench_nstar 300 python -u bench.py --config nstar --steps 10 --recall-queries 64 --no-cpu-baseline --no-host-batch
