#!/bin/bash
# C2 after the spill fix; sample_div A/B; DVFS probe (final refine on an idle GPU);
# scan8 phase / workgroup timeline
source tools/gpu_step.sh
T=${1:-r04h}
step ${T}_bench_c2 200 python -u bench.py --steps 30 --no-cpu-baseline
for sd in 8 16; do
step ${T}_bench_c2_sd$sd 200 python -u bench.py --steps 30 --no-cpu-baseline --no-host-batch --sample-div $sd
done
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_idle.so step ${T}_tr_idle 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_idle -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
python3 tools/trace_kernels.py gpurun_out/${T}_tr_idle/run_kernel_trace.csv 20 > gpurun_out/${T}_tr_idle.txt 2>&1
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_s8prof.so step ${T}_s8prof 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-recall --no-host-batch --sync
