#!/bin/bash
# round 4 (session 2): full GPU suite + smoke on the restored tree, C2 line, C2 kernel stats
source tools/gpu_step.sh
T=${1:-r04k}
step ${T}_pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ${T}_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step ${T}_bench_c2 300 python -u bench.py --steps 30
step ${T}_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch
