#!/bin/bash
# GPU box, round 2 end-to-end check: every GPU test, smoke, the bench lines of
# C1-C5 + north_star (+ the 8-GPU per-rank strong-scaling shape) and kernel stats.
# usage: tools/r02_final.sh TAG     (outputs under gpurun_out/TAG_*)
set -o pipefail
T=${1:-r02f}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
echo "== pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest.log 2>&1 || { tail -30 $O/${T}_pytest.log; exit 1; }
tail -1 $O/${T}_pytest.log
echo "== smoke"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
for b in c2:--config,c2 nstar:--config,nstar,--steps,10 c3:--config,c3,--steps,10 c4:--config,c4,--steps,10 c5:--config,c5,--steps,10 c1:--config,c1 strong8:--n,125000,--batch,256,--no-cpu-baseline weak8:--n,125000,--batch,2048,--no-cpu-baseline; do
  name=${b%%:*}; args=${b#*:}; args=${args//,/ }
  echo "== bench $name ($args)"
  timeout -k 10 600 python -u bench.py $args > $O/${T}_bench_$name.json 2> $O/${T}_bench_$name.err || { tail -20 $O/${T}_bench_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${T}_bench_$name.json'));r=d.get('roofline') or {};print('$name',d['value'],d.get('ms_per_step'),d.get('recall_at_10'),r.get('kernel'),r.get('avg_launch_ms'),r.get('frac'),(d.get('cpu_baseline') or {}).get('value'))"
done
for c in c2 c4 c5; do
  echo "== rocprof $c"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_$c -o run -- python3 bench.py --config $c --steps 10 --no-cpu-baseline --no-recall > $O/${T}_prof_$c.log 2>&1 || { tail -20 $O/${T}_prof_$c.log; exit 1; }
done
echo done
