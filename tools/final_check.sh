#!/bin/bash
# GPU box: the round-end checks (tests, smoke, every bench config, C2 rocprof, 8-GPU per-rank rehearsal).
# usage: tools/final_check.sh TAG   (outputs under gpurun_out/TAG_*)
set -o pipefail
T=${1:-final}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1"; }
step pytest
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/${T}_pytest.log 2>&1 || { tail -30 $O/${T}_pytest.log; exit 1; }
tail -1 $O/${T}_pytest.log
step smoke
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
for c in c2 c3 c1 c4 c5; do
  step bench_$c
  extra=""
  [ $c = c3 ] && extra="--steps 10 --cpu-seconds 5"
  [ $c = c1 ] && extra="--steps 2000 --warmup 50"
  [ $c = c4 ] || [ $c = c5 ] && extra="--steps 10 --cpu-seconds 8"
  timeout -k 10 500 python -u bench.py --config $c $extra > $O/${T}_bench_$c.json 2> $O/${T}_bench_$c.err || { tail -20 $O/${T}_bench_$c.err; exit 1; }
  cut -c1-200 $O/${T}_bench_$c.json
done
step rehearsal_n8
timeout -k 10 300 python -u bench.py --n 125000 --batch 2048 --steps 20 --no-cpu-baseline > $O/${T}_rehearsal_n8.json 2>/dev/null || exit 1
cut -c1-200 $O/${T}_rehearsal_n8.json
step rocprof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall > $O/${T}_prof_c2.log 2>&1 || { tail -20 $O/${T}_prof_c2.log; exit 1; }
step rocprof_c1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_c1 -o run -- python3 bench.py --config c1 --steps 2000 --warmup 50 --no-cpu-baseline > $O/${T}_prof_c1.log 2>&1 || { tail -20 $O/${T}_prof_c1.log; exit 1; }
echo done
