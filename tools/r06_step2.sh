#!/bin/bash
# round 6: IVF suite + C5 step after the deferred coarse-flag check and the run select;
# the per-call C2 path's kernel trace (usage: tools/r06_step2.sh TAG)
source tools/gpu_step.sh
T=$1
step ${T}_ivf 700 python -u -m pytest tests/test_gpu_ivf.py -x -q --timeout 300 --timeout-method thread
step ${T}_c5 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
step ${T}_prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --no-cpu-baseline --no-recall --no-host-batch
python3 tools/trace_kernels.py gpurun_out/${T}_prof_c5/run_kernel_trace.csv 10 > gpurun_out/${T}_c5_step_kernels.txt 2>&1
step ${T}_prof_pc 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_pc -o run -- python3 bench.py --api per_call --steps 64 --warmup 8 --no-cpu-baseline --no-recall
python3 tools/trace_kernels.py gpurun_out/${T}_prof_pc/run_kernel_trace.csv 64 > gpurun_out/${T}_pc_step_kernels.txt 2>&1
rm -f gpurun_out/${T}_prof_*/run_kernel_trace.csv
cat gpurun_out/${T}_c5_step_kernels.txt gpurun_out/${T}_pc_step_kernels.txt
