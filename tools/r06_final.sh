#!/bin/bash
# round 6 final: the C5 line + its pipelined-step trace on the final tree, then the GPU suite
# and smoke (closing_check A)
source tools/gpu_step.sh
T=$1
step ${T}_bench_c5 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
step ${T}_prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --no-cpu-baseline --no-recall --no-host-batch --no-sync-leg
python3 tools/trace_kernels.py gpurun_out/${T}_prof_c5/run_kernel_trace.csv 10 10 > gpurun_out/${T}_c5_step_kernels.txt 2>&1
rm -f gpurun_out/${T}_prof_*/run_kernel_trace.csv
step ${T}_pytest 1100 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread
step ${T}_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
