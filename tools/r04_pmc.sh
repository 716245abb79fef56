#!/bin/bash
# round 4 PMC traffic passes (MI355X_MICROARCH.md 'HBM': one counter per rocprofv3 run,
# no trace domains): FETCH_SIZE / WRITE_SIZE of the dominant kernel of C2, north_star,
# C3 (scan8 append), C4 (IVF_FLAT bound scan over list-order rows), C5 (PQ fast scan)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
run() { # tag counter bench-args...
	local tag=$1 ctr=$2; shift 2
	timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc4_${tag}_${ctr} -o run -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu-baseline --no-recall --no-host-batch --sync > $O/pmc4_${tag}_${ctr}.log 2>&1 || { echo "pmc $tag $ctr FAILED"; tail -5 $O/pmc4_${tag}_${ctr}.log; exit 1; }
	echo "pmc $tag $ctr ok"
}
# usage: tools/r04_pmc.sh [COUNTER...] (default both; one gpurun call each keeps a call short;
# the summaries below need both passes under gpurun_out/ and also run on the CPU side)
for ctr in ${@:-FETCH_SIZE WRITE_SIZE}; do
	run c2 $ctr
	run nstar $ctr --config nstar
	run c3 $ctr --config c3
	run c4 $ctr --config c4
	run c5 $ctr --config c5
done
S8="scan8_kernel<12, 4, 2, 0, 0>"
[ -d $O/pmc4_c5_FETCH_SIZE ] && [ -d $O/pmc4_c5_WRITE_SIZE ] || exit 0
python3 tools/pmc_traffic.py $O/pmc4_c2_FETCH_SIZE $O/pmc4_c2_WRITE_SIZE $O/r04_c2_scan_traffic.json --n 1000000 --dim 768 --batch 256 --elem-bytes 1 --kernel "$S8" --bench-kernel "scan8_kernel<L2,append,i8>"
python3 tools/pmc_traffic.py $O/pmc4_nstar_FETCH_SIZE $O/pmc4_nstar_WRITE_SIZE $O/r04_nstar_scan_traffic.json --n 10000000 --dim 768 --batch 256 --elem-bytes 1 --kernel "$S8" --bench-kernel "scan8_kernel<L2,append,i8>"
python3 tools/pmc_traffic.py $O/pmc4_c3_FETCH_SIZE $O/pmc4_c3_WRITE_SIZE $O/r04_c3_scan_traffic.json --n 10000000 --dim 768 --batch 256 --elem-bytes 1 --kernel "$S8" --bench-kernel "scan8_kernel<DOT,append,i8>"
python3 tools/pmc_traffic.py $O/pmc4_c4_FETCH_SIZE $O/pmc4_c4_WRITE_SIZE $O/r04_c4_ivf_traffic.json --n 12500000 --dim 768 --batch 256 --kernel "flat_list_lb_kernel" --bench-kernel "flat_list_lb_kernel"
python3 tools/pmc_traffic.py $O/pmc4_c5_FETCH_SIZE $O/pmc4_c5_WRITE_SIZE $O/r04_c5_ivf_traffic.json --n 12500000 --dim 768 --batch 256 --kernel "pq_fast_scan_kernel" --bench-kernel "pq_fast_scan_kernel"
