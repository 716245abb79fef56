#!/bin/bash
# pool_refine final-mode ablations (row loads off / f32 math) + the async test
source tools/gpu_step.sh
T=${1:-r04f}
step ${T}_pytest 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_scan8.py::test_async_pipeline_matches_sync
for v in nol f32m nolf32m; do
  LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_$v.so step ${T}_tr_$v 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_$v -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
  python3 tools/trace_kernels.py gpurun_out/${T}_tr_$v/run_kernel_trace.csv 20 > gpurun_out/${T}_tr_$v.txt 2>&1
done
