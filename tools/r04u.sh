#!/bin/bash
# round 4: one query per call A/B (scan8 QB = 1 geometry vs the 128-query geometry, same box,
# interleaved), then the C3 and C4 lines of the validated tree
# (lib_qb8.so was a development build of a 16-query scan8 geometry, measured slower and since removed)
source tools/gpu_step.sh
T=${1:-r04u}
QB8=duckdb-lancedb_amd/lib_dev/lib_qb8.so
PC="python -u bench.py --api per_call --steps 500 --warmup 3 --no-cpu-baseline"
step ${T}_pc_c2_qb1a 200 $PC
LANCE_HIP_LIB=$QB8 step ${T}_pc_c2_qb8a 200 $PC
step ${T}_pc_c2_qb1b 200 $PC
LANCE_HIP_LIB=$QB8 step ${T}_pc_c2_qb8b 200 $PC
PN="python -u bench.py --config nstar --api per_call --steps 100 --warmup 3 --no-cpu-baseline"
step ${T}_pc_nstar_qb1 300 $PN
LANCE_HIP_LIB=$QB8 step ${T}_pc_nstar_qb8 300 $PN
step ${T}_bench_c3 400 python -u bench.py --config c3 --steps 10 --recall-queries 64 --no-cpu-baseline --no-host-batch
step ${T}_bench_c4 400 python -u bench.py --config c4 --steps 10 --no-cpu-baseline
