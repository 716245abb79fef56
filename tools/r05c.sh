#!/bin/bash
# full GPU suite + C2 bench (after the async drain fix) + a kernel trace of the C2 steps
source tools/gpu_step.sh
T=${1:-r05c}
step ${T}_pytest 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread
step ${T}_bench_c2 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step ${T}_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch
python3 tools/trace_kernels.py gpurun_out/${T}_prof_c2/run_kernel_trace.csv 20 > gpurun_out/${T}_c2_step_kernels.txt 2>&1
step ${T}_rank_nstar8 200 python -u bench.py --n 1250000 --steps 30 --no-cpu-baseline --no-host-batch
