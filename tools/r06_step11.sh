#!/bin/bash
# round 6: pool_refine on 256 threads with a 4096-entry pool (two workgroups per CU:
# lib_dev/lib_pr256.so) against the release geometry: parity subset on the variant, then
# interleaved C2 / per-rank C2 / north_star lines
source tools/gpu_step.sh
T=$1
export LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_pr256.so
step ${T}_par_pr256 600 python -u -m pytest tests/test_gpu_scan8.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread
unset LANCE_HIP_LIB
for rep in 1 2; do
for v in base pr256; do
	if [ "$v" = base ]; then unset LANCE_HIP_LIB; else export LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_$v.so; fi
	step ${T}_c2_${v}_$rep 300 python -u bench.py --steps 40 --no-cpu-baseline --no-host-batch --no-recall
	step ${T}_rank_${v}_$rep 300 python -u bench.py --n 125000 --steps 40 --no-cpu-baseline --no-host-batch --no-recall
	grep -ho '"value": [0-9.]*' gpurun_out/${T}_c2_${v}_$rep.log gpurun_out/${T}_rank_${v}_$rep.log | tr '\n' ' '; echo
done
done
for v in base pr256; do
	if [ "$v" = base ]; then unset LANCE_HIP_LIB; else export LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_$v.so; fi
	step ${T}_nstar_${v} 400 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-host-batch --no-recall
	grep -ho '"value": [0-9.]*' gpurun_out/${T}_nstar_${v}.log | tr '\n' ' '; echo
done
unset LANCE_HIP_LIB
