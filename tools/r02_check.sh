#!/bin/bash
# GPU box, round 2: tests + smoke + C2 / north_star benches + C2 kernel stats.
# usage: tools/r02_check.sh TAG [benches...]   (outputs under gpurun_out/TAG_*)
set -o pipefail
T=${1:-r02}
shift
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
echo "== pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/${T}_pytest.log 2>&1 || { tail -30 $O/${T}_pytest.log; exit 1; }
tail -1 $O/${T}_pytest.log
echo "== smoke"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
for b in "$@"; do
  name=${b%%:*}; args=${b#*:}; args=${args//,/ }
  echo "== bench $name ($args)"
  timeout -k 10 600 python -u bench.py $args > $O/${T}_bench_$name.json 2> $O/${T}_bench_$name.err || { tail -20 $O/${T}_bench_$name.err; exit 1; }
  cut -c1-400 $O/${T}_bench_$name.json
done
echo "== rocprof c2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall > $O/${T}_prof_c2.log 2>&1 || { tail -20 $O/${T}_prof_c2.log; exit 1; }
echo done
