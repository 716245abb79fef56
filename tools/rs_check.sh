#!/bin/bash
# GPU box: rscan parity tests + C2 / north_star / C3 benches with the register-streamed scan on and off.
# usage: tools/rs_check.sh TAG
set -o pipefail
T=${1:-rs}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
echo "== pytest rscan"
timeout -k 10 300 python -u -m pytest tests/test_gpu_rscan.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/${T}_pytest.log 2>&1 || { tail -30 $O/${T}_pytest.log; exit 1; }
tail -1 $O/${T}_pytest.log
for b in c2:--opt,rscan=1 c2s:--opt,rscan=0 nstar:--config,nstar,--steps,10,--opt,rscan=1 c3:--config,c3,--steps,10,--opt,rscan=1; do
  name=${b%%:*}; args=${b#*:}; args=${args//,/ }
  echo "== bench $name ($args)"
  timeout -k 10 400 python -u bench.py --no-cpu-baseline $args > $O/${T}_bench_$name.json 2> $O/${T}_bench_$name.err || { tail -20 $O/${T}_bench_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${T}_bench_$name.json'));r=d['roofline'];print('$name',d['value'],d.get('recall_at_10'),r['kernel'],r['avg_launch_ms'],r['frac'],d['search_stats']['fallback_queries'])"
done
echo "== rocprof c2 rscan"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --opt rscan=1 > $O/${T}_prof_c2.log 2>&1 || { tail -20 $O/${T}_prof_c2.log; exit 1; }
grep -i scan_kernel $O/${T}_prof_c2/run_kernel_stats.csv | cut -c1-60,200-400
echo done
