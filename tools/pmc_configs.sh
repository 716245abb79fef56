#!/bin/bash
# PMC traffic passes (MI355X_MICROARCH.md 'HBM': one counter per rocprofv3 run, no trace
# domains): FETCH_SIZE / WRITE_SIZE of the dominant kernel of each listed config.
# usage: tools/pmc_configs.sh TAG CONFIG... (configs: c2 nstar c3 c4 c5); summaries -> gpurun_out/TAG_<cfg>_*_traffic.json
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=$1
shift
run() { # cfg counter
	local cfg=$1 ctr=$2
	timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc5_${T}_${cfg}_${ctr} -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-recall --no-host-batch --sync > $O/pmc5_${T}_${cfg}_${ctr}.log 2>&1 || { echo "pmc $cfg $ctr FAILED"; tail -5 $O/pmc5_${T}_${cfg}_${ctr}.log; exit 1; }
	echo "pmc $cfg $ctr ok"
}
S8="scan8_kernel<12, 4, 2, 0, 0>"
for cfg in "$@"; do
	run $cfg FETCH_SIZE
	run $cfg WRITE_SIZE
	F=$O/pmc5_${T}_${cfg}_FETCH_SIZE W=$O/pmc5_${T}_${cfg}_WRITE_SIZE
	case $cfg in
	c2) python3 tools/pmc_traffic.py $F $W $O/${T}_c2_scan_traffic.json --n 1000000 --dim 768 --batch 256 --elem-bytes 1 --kernel "$S8" --bench-kernel "scan8_kernel<L2,append,i8>" ;;
	nstar) python3 tools/pmc_traffic.py $F $W $O/${T}_nstar_scan_traffic.json --n 10000000 --dim 768 --batch 256 --elem-bytes 1 --kernel "$S8" --bench-kernel "scan8_kernel<L2,append,i8>" ;;
	c3) python3 tools/pmc_traffic.py $F $W $O/${T}_c3_scan_traffic.json --n 10000000 --dim 768 --batch 256 --elem-bytes 1 --kernel "$S8" --bench-kernel "scan8_kernel<DOT,append,i8>" ;;
	c4) python3 tools/pmc_traffic.py $F $W $O/${T}_c4_ivf_traffic.json --n 12500000 --dim 768 --batch 256 --kernel "flat_list_lb_kernel" --bench-kernel "flat_list_lb_kernel" ;;
	c5) python3 tools/pmc_traffic.py $F $W $O/${T}_c5_ivf_traffic.json --n 12500000 --dim 768 --batch 256 --kernel "pq_fast_scan_bank_kernel" --bench-kernel "pq_fast_scan_bank_kernel" --fetch-factor 1.918 ;;
	esac
	rm -rf $F $W  # (the raw CSVs: gpurun returns at most 64 MiB)
done
