#!/bin/bash
# pool_refine geometry variants (development builds in lib_dev/), kernel traces of C2 steps
source tools/gpu_step.sh
T=${1:-r04d}
step ${T}_probe_rand 200 duckdb-lancedb_amd/lib_dev/gather_probe 1000000 1
for v in default ni0 pw12 nomerge ni0nomerge; do
  if [ $v = default ]; then L=duckdb-lancedb_amd/lib/liblancedb_hip.so; else L=duckdb-lancedb_amd/lib_dev/lib_$v.so; fi
  LANCE_HIP_LIB=$L step ${T}_tr_$v 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_$v -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch
  python3 tools/trace_kernels.py gpurun_out/${T}_tr_$v/run_kernel_trace.csv 20 > gpurun_out/${T}_tr_$v.txt 2>&1
done
