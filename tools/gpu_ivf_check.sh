#!/bin/bash
# GPU box: IVF parity tests, then the IVF bench lines.  usage: tools/gpu_ivf_check.sh TAG [bench args]
set -o pipefail
T=${1:-ivf}
shift
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ivf.py tests/test_gpu_filter.py tests/test_distributed.py -x -v --timeout 120 --timeout-method thread > $O/${T}_pytest.log 2>&1 || { echo "ivf pytest FAILED"; tail -40 $O/${T}_pytest.log; exit 1; }
tail -3 $O/${T}_pytest.log
bash tools/gpu_ivf_bench.sh $T "$@"
if [ -n "$IVF_PROF" ]; then
  for c in c4 c5; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_$c -o run -- python3 bench.py --config $c --steps 10 --no-cpu-baseline --no-recall > $O/${T}_prof_$c.log 2>&1 || { echo "rocprof $c FAILED"; tail -20 $O/${T}_prof_$c.log; exit 1; }
  done
  echo profiled
fi
