#!/bin/bash
# scan8 prologue with every query load in flight: scan8 / tilemin parity + C2 line and
# kernel trace; pool_refine stamps to device memory (host-printed, no in-kernel printf)
source tools/gpu_step.sh
T=${1:-r04m}
step ${T}_pytest 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scan8.py tests/test_gpu_scan_i8.py
step ${T}_bench_c2 200 python -u bench.py --steps 30 --no-cpu-baseline
step ${T}_tr_c2 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
python3 tools/trace_kernels.py gpurun_out/${T}_tr_c2/run_kernel_trace.csv 20 > gpurun_out/${T}_tr_c2.txt 2>&1
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_prprof.so step ${T}_prprof 200 python -u bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_s8prof.so step ${T}_s8prof 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-recall --no-host-batch --sync
