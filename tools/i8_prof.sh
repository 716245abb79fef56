#!/bin/bash
# Development-only (GPU box): C2 / north_star benches on the default (int8) scan + C2 kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in c2:--steps,20 nstar:--config,nstar,--steps,10,--no-recall ; do
  name=${b%%:*}; args=${b#*:}; args=${args//,/ }
  timeout -k 10 400 python -u bench.py --no-cpu-baseline $args > gpurun_out/i8p_bench_$name.json 2> gpurun_out/i8p_bench_$name.err || { tail -20 gpurun_out/i8p_bench_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/i8p_bench_$name.json'));r=d.get('roofline') or {};print('$name',d['value'],d.get('ms_per_step'),d.get('recall_at_10'),r.get('kernel'),r.get('avg_launch_ms'),r.get('frac'),d.get('search_stats'))"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/i8p_prof_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall > gpurun_out/i8p_prof_c2.log 2>&1 || { tail -20 gpurun_out/i8p_prof_c2.log; exit 1; }
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/i8p_prof_c2/**/run_kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]: print(r['Name'][:70], r['Calls'], r['AverageNs'])
PY
