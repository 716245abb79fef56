#!/bin/bash
# C4 step: bench line and rocprofv3 kernel trace of the timed steps
source tools/gpu_step.sh
T=$1
step ${T}_c4 300 python -u bench.py --config c4 --steps 10 --no-cpu-baseline
step ${T}_prof_c4 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c4 -o run -- python3 bench.py --config c4 --steps 10 --no-cpu-baseline --no-recall --no-host-batch
python3 tools/trace_kernels.py gpurun_out/${T}_prof_c4/run_kernel_trace.csv 10 > gpurun_out/${T}_c4_step_kernels.txt 2>&1
rm -f gpurun_out/${T}_prof_c4/run_kernel_trace.csv
cat gpurun_out/${T}_c4_step_kernels.txt
