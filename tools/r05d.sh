#!/bin/bash
# two pass streams: async tests, C2 bench + its kernel trace, per-rank north_star shape
source tools/gpu_step.sh
T=${1:-r05d}
step ${T}_pytest 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scan8.py tests/test_gpu_threads.py tests/test_distributed.py
step ${T}_bench_c2 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
step ${T}_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch
python3 tools/trace_kernels.py gpurun_out/${T}_prof_c2/run_kernel_trace.csv 20 > gpurun_out/${T}_c2_step_kernels.txt 2>&1
step ${T}_rank_nstar8 200 python -u bench.py --n 1250000 --steps 30 --no-cpu-baseline --no-host-batch
step ${T}_rank_c2s8 200 python -u bench.py --n 125000 --steps 30 --no-cpu-baseline --no-host-batch
