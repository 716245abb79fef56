#!/bin/bash
# round 6: the next item's round-0 codes requested in the PQ scan's last round: IVF tests and an
# interleaved C5 A/B against requesting them at the item start (lib_dev/lib_noxpre.so)
source tools/gpu_step.sh
T=$1
step ${T}_ivf 900 python -u -m pytest tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py tests/test_gpu_ivf_shard.py -x -q --timeout 300 --timeout-method thread
for rep in 1 2; do
for v in base noxpre; do
	if [ "$v" = base ]; then unset LANCE_HIP_LIB; else export LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_$v.so; fi
	step ${T}_ab_${v}_$rep 300 python -u bench.py --config c5 --steps 20 --no-cpu-baseline --no-recall --no-sync-leg
	grep -ho '"avg_launch_ms": [0-9.]*\|"value": [0-9.]*' gpurun_out/${T}_ab_${v}_$rep.log | tr '\n' ' '; echo
done
done
unset LANCE_HIP_LIB
