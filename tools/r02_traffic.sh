#!/bin/bash
# GPU box: PQ parity tests, C5 bench, then FETCH_SIZE / WRITE_SIZE passes (one
# counter per run) over C4, C5 and north_star + summaries (bench roofline.traffic).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py tests/test_gpu_filter.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/tr_pytest.log 2>&1 || { tail -30 $O/tr_pytest.log; exit 1; }
tail -1 $O/tr_pytest.log
timeout -k 10 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline > $O/tr_bench_c5.json 2> $O/tr_bench_c5.err || { tail -20 $O/tr_bench_c5.err; exit 1; }
python -c "import json;d=json.load(open('$O/tr_bench_c5.json'));r=d['roofline'];print('c5',d['value'],d['recall_at_10_by_refine'],r['avg_launch_ms'])"
timeout -k 10 400 python -u bench.py --config nstar --n 1250000 --no-cpu-baseline > $O/tr_bench_nstar_rank8.json 2> $O/tr_bench_nstar_rank8.err || { tail -20 $O/tr_bench_nstar_rank8.err; exit 1; }
python -c "import json;d=json.load(open('$O/tr_bench_nstar_rank8.json'));r=d['roofline'];print('nstar per-rank 1.25M',d['value'],d['ms_per_step'],r['avg_launch_ms'])"
for cfg in c4 c5 nstar; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/tr_${cfg}_pmc_${ctr} -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-recall > $O/tr_${cfg}_${ctr}.log 2>&1 || { echo "pmc $cfg $ctr FAILED"; tail -5 $O/tr_${cfg}_${ctr}.log; exit 1; }
    echo "pmc $cfg $ctr ok"
  done
done
echo done
