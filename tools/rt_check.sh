#!/bin/bash
# Development-only (GPU box): full GPU suite, then C2 / north_star / per-rank shapes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rt_pytest.log 2>&1 || { tail -30 gpurun_out/rt_pytest.log; exit 1; }
tail -1 gpurun_out/rt_pytest.log
for b in c2:--steps,20 nstar:--config,nstar,--steps,10,--no-recall strong8:--n,125000,--batch,256 nstar8:--config,nstar,--n,1250000,--steps,20,--no-recall; do
  name=${b%%:*}; args=${b#*:}; args=${args//,/ }
  timeout -k 10 400 python -u bench.py --no-cpu-baseline $args > gpurun_out/rt_bench_$name.json 2> gpurun_out/rt_bench_$name.err || { tail -20 gpurun_out/rt_bench_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/rt_bench_$name.json'));r=d.get('roofline') or {};print('$name',d['value'],d.get('ms_per_step'),d.get('recall_at_10'),r.get('avg_launch_ms'),d.get('search_stats'))"
done
