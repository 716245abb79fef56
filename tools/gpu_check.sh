#!/bin/bash
# GPU box: parity tests, C2 + C3 bench lines, rocprofv3 kernel stats of the C2 bench.
# usage: tools/gpu_check.sh TAG   (outputs under gpurun_out/TAG_*)
set -o pipefail
T=${1:-chk}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/${T}_pytest.log 2>&1 || { echo "pytest FAILED"; tail -30 $O/${T}_pytest.log; exit 1; }
tail -3 $O/${T}_pytest.log
timeout -k 10 300 python -u bench.py > $O/${T}_bench_c2.json 2> $O/${T}_bench_c2.err || { echo "bench c2 FAILED"; tail -20 $O/${T}_bench_c2.err; exit 1; }
cat $O/${T}_bench_c2.json
timeout -k 10 400 python -u bench.py --config c3 --steps 10 --cpu-seconds 5 > $O/${T}_bench_c3.json 2> $O/${T}_bench_c3.err || { echo "bench c3 FAILED"; tail -20 $O/${T}_bench_c3.err; exit 1; }
cat $O/${T}_bench_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall > $O/${T}_prof_c2.log 2>&1 || { echo "rocprof FAILED"; tail -20 $O/${T}_prof_c2.log; exit 1; }
echo done
