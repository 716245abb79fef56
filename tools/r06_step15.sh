#!/bin/bash
# round 6: pool_refine's pool gather spread over every thread (release) against a thread per
# segment (lib_dev/lib_nospread.so): parity subset, then interleaved C2 / per-rank C2 / per-call /
# north_star lines
source tools/gpu_step.sh
T=$1
step ${T}_par 700 python -u -m pytest tests/test_gpu_scan8.py tests/test_gpu_parity.py tests/test_gpu_nstar.py -x -q --timeout 400 --timeout-method thread
for rep in 1 2; do
for v in base nospread; do
	if [ "$v" = base ]; then unset LANCE_HIP_LIB; else export LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_$v.so; fi
	step ${T}_c2_${v}_$rep 300 python -u bench.py --steps 40 --no-cpu-baseline --no-host-batch --no-recall
	step ${T}_rank_${v}_$rep 300 python -u bench.py --n 125000 --steps 40 --no-cpu-baseline --no-host-batch --no-recall
	grep -ho '"value": [0-9.]*' gpurun_out/${T}_c2_${v}_$rep.log gpurun_out/${T}_rank_${v}_$rep.log | head -2 | tr '\n' ' '; echo
done
done
for v in base nospread; do
	if [ "$v" = base ]; then unset LANCE_HIP_LIB; else export LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_$v.so; fi
	step ${T}_pc_${v} 300 python -u bench.py --api per_call --steps 256 --warmup 16 --no-cpu-baseline --no-recall
	step ${T}_nstar_${v} 400 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-host-batch --no-recall
	grep -ho '"value": [0-9.]*' gpurun_out/${T}_pc_${v}.log gpurun_out/${T}_nstar_${v}.log | tr '\n' ' '; echo
done
unset LANCE_HIP_LIB
