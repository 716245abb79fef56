#!/bin/bash
# scan8 per-lane append entries + pool_refine radix merge / split refine paths:
# full GPU suite, then an interleaved A/B against the previous commit on one box
source tools/gpu_step.sh
T=${1:-r04o}
step ${T}_pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for rep in 1 2; do
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_base.so step ${T}_ab_base$rep 200 python -u bench.py --steps 30 --no-cpu-baseline --no-host-batch --no-recall
step ${T}_ab_new$rep 200 python -u bench.py --steps 30 --no-cpu-baseline --no-host-batch
done
step ${T}_tr_c2 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
python3 tools/trace_kernels.py gpurun_out/${T}_tr_c2/run_kernel_trace.csv 20 > gpurun_out/${T}_tr_c2.txt 2>&1
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_prprof.so step ${T}_prprof 200 python -u bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_s8prof.so step ${T}_s8prof 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-recall --no-host-batch --sync
step ${T}_bench_nstar 300 python -u bench.py --config nstar --steps 10 --recall-queries 64 --no-cpu-baseline --no-host-batch
