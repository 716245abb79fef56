#!/bin/bash
# C5 step: IVF parity tests, bench line, rocprofv3 kernel trace of the timed steps
source tools/gpu_step.sh
T=$1
step ${T}_pytest 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_ivf_params.py tests/test_gpu_ivf.py}
step ${T}_c5 300 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
step ${T}_prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --no-cpu-baseline --no-recall --no-host-batch
python3 tools/trace_kernels.py gpurun_out/${T}_prof_c5/run_kernel_trace.csv 10 > gpurun_out/${T}_c5_step_kernels.txt 2>&1
rm -f gpurun_out/${T}_prof_c5/run_kernel_trace.csv
cat gpurun_out/${T}_c5_step_kernels.txt
