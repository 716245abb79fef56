#!/bin/bash
# round 6: IVF_FLAT bound scan with the bound words in the query rows' LDS (3 workgroups per
# CU) and an item -> block table; A/B against round 5's layout (lib_dev/lib_flv1.so); IVF tests
source tools/gpu_step.sh
T=$1
step ${T}_ivf 900 python -u -m pytest tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py tests/test_gpu_ivf_shard.py -x -q --timeout 300 --timeout-method thread
for rep in 1 2; do
for v in base flv1; do
	if [ "$v" = base ]; then unset LANCE_HIP_LIB; else export LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_$v.so; fi
	step ${T}_ab_${v}_$rep 300 python -u bench.py --config c4 --steps 10 --no-cpu-baseline --no-recall --no-sync-leg
	grep -ho '"avg_launch_ms": [0-9.]*\|"value": [0-9.]*' gpurun_out/${T}_ab_${v}_$rep.log | tr '\n' ' '; echo
done
done
unset LANCE_HIP_LIB
step ${T}_c4 400 python -u bench.py --config c4 --steps 10 --no-cpu-baseline
grep -ho '"avg_launch_ms": [0-9.]*\|"value": [0-9.]*\|"recall_at_10": [0-9.]*' gpurun_out/${T}_c4.log | tr '\n' ' '; echo
