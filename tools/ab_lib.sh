#!/bin/bash
# interleaved A/B of the release library against a development variant on one box
# (usage: tools/ab_lib.sh TAG VARIANT [parity]): C2, the per-rank C2 / north_star shapes, twice each;
# "parity": first the flat GPU parity files under the variant
source tools/gpu_step.sh
T=$1 V=$2
VL=duckdb-lancedb_amd/lib_dev/lib_$V.so
if [ "$3" = parity ]; then
	LANCE_HIP_LIB=$VL step ${T}_${V}_parity 900 python -u -m pytest tests/test_gpu_scan8.py tests/test_gpu_parity.py tests/test_gpu_nstar.py -m gpu -x -q --timeout 300 --timeout-method thread
fi
B="--no-cpu-baseline --no-host-batch"
for r in 1 2; do
	for lib in rel $V; do
		if [ $lib = rel ]; then unset LANCE_HIP_LIB; else export LANCE_HIP_LIB=$VL; fi
		step ${T}_${lib}_c2_$r 300 python -u bench.py --steps 20 $B
		step ${T}_${lib}_rank_$r 300 python -u bench.py --n 125000 --steps 30 $B
		step ${T}_${lib}_nrank_$r 300 python -u bench.py --n 1250000 --steps 30 $B
	done
done
unset LANCE_HIP_LIB
for f in gpurun_out/${T}_*_[0-9].log; do grep -h '^{' $f | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$(basename $f .log)', d['value'], d['ms_per_step'], d.get('exact_ids_on_recall_subset'))"; done
