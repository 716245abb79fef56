#!/bin/bash
# release candidate: full GPU suite; C2 trace; pool_refine stamps; C4 / C5 lines and the
# PQ scan's phase breakdown (diagnostic build)
source tools/gpu_step.sh
T=${1:-r04r}
step ${T}_pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ${T}_bench_c2 200 python -u bench.py --steps 30 --no-cpu-baseline
step ${T}_tr_c2 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
python3 tools/trace_kernels.py gpurun_out/${T}_tr_c2/run_kernel_trace.csv 20 > gpurun_out/${T}_tr_c2.txt 2>&1
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_prprof.so step ${T}_prprof 200 python -u bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
step ${T}_bench_c4 400 python -u bench.py --config c4 --steps 10 --no-cpu-baseline
step ${T}_bench_c5 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_pqprof.so step ${T}_pqprof 400 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-recall
