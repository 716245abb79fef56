#!/bin/bash
# round 6: coarse bounds with its operand chunks requested two chunks ahead: IVF tests, C5 / C4
# lines and the C5 trace of the pipelined steps
source tools/gpu_step.sh
T=$1
step ${T}_ivf 900 python -u -m pytest tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py -x -q --timeout 300 --timeout-method thread
step ${T}_c5 400 python -u bench.py --config c5 --steps 20 --no-cpu-baseline --no-recall
step ${T}_prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --no-cpu-baseline --no-recall --no-host-batch --no-sync-leg
python3 tools/trace_kernels.py gpurun_out/${T}_prof_c5/run_kernel_trace.csv 10 10 > gpurun_out/${T}_c5_step_kernels.txt 2>&1
rm -f gpurun_out/${T}_prof_*/run_kernel_trace.csv
grep -ho '"avg_launch_ms": [0-9.]*\|"value": [0-9.]*' gpurun_out/${T}_c5.log | tr '\n' ' '; echo
cat gpurun_out/${T}_c5_step_kernels.txt
