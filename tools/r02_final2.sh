#!/bin/bash
# GPU box, round 2 closing check (int8 scan default): every GPU test, smoke, the
# bench lines of C1-C5 + north_star (+ the 8-GPU per-rank shapes), rocprof kernel
# stats, and PMC passes of the flat scan at C2 / north_star.
# usage: tools/r02_final2.sh TAG     (outputs under gpurun_out/TAG_*)
set -o pipefail
T=${1:-r02z}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
echo "== pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest.log 2>&1 || { tail -30 $O/${T}_pytest.log; exit 1; }
tail -1 $O/${T}_pytest.log
echo "== smoke"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
for b in c2:--steps,20 nstar:--config,nstar,--steps,10 c3:--config,c3,--steps,10 c4:--config,c4,--steps,10 c5:--config,c5,--steps,10 c1:--config,c1 strong8:--n,125000,--batch,256,--no-cpu-baseline weak8:--n,125000,--batch,2048,--no-cpu-baseline nstar8:--config,nstar,--n,1250000,--no-cpu-baseline c2bf16:--steps,20,--no-cpu-baseline,--opt,scan_i8=off; do
  name=${b%%:*}; args=${b#*:}; args=${args//,/ }
  echo "== bench $name ($args)"
  timeout -k 10 600 python -u bench.py $args > $O/${T}_bench_$name.json 2> $O/${T}_bench_$name.err || { tail -20 $O/${T}_bench_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${T}_bench_$name.json'));r=d.get('roofline') or {};print('$name',d['value'],d.get('ms_per_step'),d.get('recall_at_10'),r.get('kernel'),r.get('avg_launch_ms'),r.get('frac'),(d.get('cpu_baseline') or {}).get('value'))"
done
for c in c2:--steps,20 nstar:--config,nstar,--steps,10 c4:--config,c4,--steps,10 c5:--config,c5,--steps,10; do
  name=${c%%:*}; args=${c#*:}; args=${args//,/ }
  echo "== rocprof $name"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_$name -o run -- python3 bench.py $args --no-cpu-baseline --no-recall > $O/${T}_prof_$name.log 2>&1 || { tail -20 $O/${T}_prof_$name.log; exit 1; }
done
echo "== pmc"
bash tools/pmc_scan.sh ${T}_c2 -- --steps 5 --warmup 2 || exit 1
bash tools/pmc_scan.sh ${T}_nstar -- --config nstar --steps 3 --warmup 1 || exit 1
echo done
