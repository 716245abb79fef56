#!/bin/bash
# IVF_PQ fast scan with two code buffers; pool_refine small later rounds; scan8 tilemin
# score: parity (IVF + flat), C2 line + kernel trace, C5 line + phases; then the round-4
# PMC traffic passes of every config's dominant kernel
source tools/gpu_step.sh
T=${1:-r04t}
step ${T}_pytest 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ivf_params.py tests/test_gpu_ivf.py tests/test_gpu_scan8.py tests/test_gpu_parity.py
step ${T}_bench_c2 200 python -u bench.py --steps 30 --no-cpu-baseline
step ${T}_tr_c2 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
python3 tools/trace_kernels.py gpurun_out/${T}_tr_c2/run_kernel_trace.csv 20 > gpurun_out/${T}_tr_c2.txt 2>&1
step ${T}_bench_c5 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_pqprof.so step ${T}_pqprof 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-recall
step ${T}_pmc 1000 bash tools/r04_pmc.sh
