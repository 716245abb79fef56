#!/bin/bash
# C5 per-phase cycles (LHIP_PQ_PROF dev builds lib_dev/lib_NAME.so) of the PQ fast scan
source tools/gpu_step.sh
T=$1; shift
for v in "$@"; do
	export LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_$v.so
	step ${T}_prof_$v 300 python -u bench.py --config c5 --steps 3 --no-cpu-baseline --no-recall --no-host-batch
	echo "$v: $(grep -h PQPROF gpurun_out/${T}_prof_$v.log)"
done
