#!/bin/bash
# PQ fast scan phase stamps (diagnostic build): 8-query vs 4-query form at C5
source tools/gpu_step.sh
T=${1:-r05h}
export LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_pqprof.so
step ${T}_c5_g8 400 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-recall
step ${T}_c5_g4 400 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-recall --opt pq_group=4
grep -h PROF gpurun_out/${T}_c5_g8.log gpurun_out/${T}_c5_g4.log
