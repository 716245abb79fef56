#!/bin/bash
# Development-only (GPU box): int8 scan parity tests, then C2 / north_star benches with and without it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_scan_i8.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/i8_pytest.log 2>&1 || { tail -40 gpurun_out/i8_pytest.log; exit 1; }
tail -1 gpurun_out/i8_pytest.log
for b in c2i8:--steps,20 nstari8:--config,nstar,--steps,10,--no-recall c2bf:--steps,20,--opt,scan_i8=off ; do
  name=${b%%:*}; args=${b#*:}; args=${args//,/ }
  timeout -k 10 400 python -u bench.py --no-cpu-baseline $args > gpurun_out/i8_bench_$name.json 2> gpurun_out/i8_bench_$name.err || { tail -20 gpurun_out/i8_bench_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/i8_bench_$name.json'));r=d.get('roofline') or {};print('$name',d['value'],d.get('ms_per_step'),d.get('recall_at_10'),r.get('kernel'),r.get('avg_launch_ms'),r.get('frac'),d.get('search_stats'))"
done
