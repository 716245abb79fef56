#!/bin/bash
# round 6: the one-query-per-call path after the fused small-batch prep: GPU parity subset,
# the Python per-call bench line, its kernel trace, and the C++ (torch-free) per-call timing
source tools/gpu_step.sh
T=$1
step ${T}_par 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scan8.py tests/test_gpu_abi_process.py -x -q --timeout 300 --timeout-method thread
step ${T}_percall_c2 300 python -u bench.py --api per_call --steps 256 --warmup 16 --no-cpu-baseline
step ${T}_cpp_percall 600 python -u tools/cpp_percall.py
step ${T}_prof_pc 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_pc -o run -- python3 bench.py --api per_call --steps 64 --warmup 8 --no-cpu-baseline --no-recall
python3 tools/trace_kernels.py gpurun_out/${T}_prof_pc/run_kernel_trace.csv 64 > gpurun_out/${T}_pc_step_kernels.txt 2>&1
rm -f gpurun_out/${T}_prof_*/run_kernel_trace.csv
cat gpurun_out/${T}_pc_step_kernels.txt
