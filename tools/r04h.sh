#!/bin/bash
# DVFS probe (final refine on an idle GPU) and the scan8 phase / workgroup timeline at C2
source tools/gpu_step.sh
T=${1:-r04h}
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_idle.so step ${T}_tr_idle 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_idle -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
python3 tools/trace_kernels.py gpurun_out/${T}_tr_idle/run_kernel_trace.csv 20 > gpurun_out/${T}_tr_idle.txt 2>&1
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_s8prof.so step ${T}_s8prof 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-recall --no-host-batch --sync
