#!/bin/bash
# pool_refine phase stamps (LHIP_PR_PROF diagnostic builds): round-3 kernel vs the NI path
source tools/gpu_step.sh
T=${1:-r04c}
for v in r03 new; do
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_prprof_$v.so step ${T}_prprof_$v 300 python -u bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch
done
