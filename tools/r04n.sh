#!/bin/bash
# pool_refine: wave-argmin merge (k <= 32), SGPR-addressed half-pipelined exact rows with
# transpose-reduced sums, segment entries loaded with their counts; full GPU suite + C2
source tools/gpu_step.sh
T=${1:-r04n}
step ${T}_pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ${T}_bench_c2 200 python -u bench.py --steps 30 --no-cpu-baseline
step ${T}_tr_c2 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
python3 tools/trace_kernels.py gpurun_out/${T}_tr_c2/run_kernel_trace.csv 20 > gpurun_out/${T}_tr_c2.txt 2>&1
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_prprof.so step ${T}_prprof 200 python -u bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
step ${T}_bench_c3 400 python -u bench.py --config c3 --steps 10 --recall-queries 64 --no-cpu-baseline --no-host-batch
