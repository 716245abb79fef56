#!/bin/bash
# round 6: the PQ scan with the L2 prefetch of the next item (release) against without it
# (lib_dev/lib_nol2pre.so), interleaved on one box; IVF tests
source tools/gpu_step.sh
T=$1
for rep in 1 2; do
for v in base nol2pre; do
	if [ "$v" = base ]; then unset LANCE_HIP_LIB; else export LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_$v.so; fi
	step ${T}_ab_${v}_$rep 300 python -u bench.py --config c5 --steps 20 --no-cpu-baseline --no-recall --no-sync-leg
	grep -ho '"avg_launch_ms": [0-9.]*\|"value": [0-9.]*' gpurun_out/${T}_ab_${v}_$rep.log | tr '\n' ' '; echo
done
done
unset LANCE_HIP_LIB
step ${T}_ivf 900 python -u -m pytest tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py -x -q --timeout 300 --timeout-method thread
