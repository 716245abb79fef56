#!/bin/bash
# C5 A/B of development builds (lib_dev/lib_NAME.so; "base" = the in-tree library): PQ scan launch time
source tools/gpu_step.sh
T=$1; shift
for v in "$@"; do
	if [ "$v" = base ]; then unset LANCE_HIP_LIB; else export LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_$v.so; fi
	step ${T}_ab_$v 300 python -u bench.py --config c5 --steps 10 --no-cpu-baseline --no-recall --no-host-batch
	grep -ho '"avg_launch_ms": [0-9.]*' gpurun_out/${T}_ab_$v.log
done
