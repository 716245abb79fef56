#!/bin/bash
# round 4: async pipelined search + tau-mode NI path
source tools/gpu_step.sh
T=${1:-r04e}
step ${T}_pytest 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_scan8.py tests/test_gpu_parity.py
step ${T}_bench_c2 300 python -u bench.py --steps 30 --no-cpu-baseline
step ${T}_tr_c2 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch
python3 tools/trace_kernels.py gpurun_out/${T}_tr_c2/run_kernel_trace.csv 20 > gpurun_out/${T}_tr_c2.txt 2>&1
