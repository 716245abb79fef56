#!/bin/bash
# round 6: invert + item layout in one faster launch; A/B of round 0's rows issued after the
# LUT reads (lib_dev/lib_rowslast.so); IVF GPU tests; C5 trace of the pipelined steps
source tools/gpu_step.sh
T=$1
step ${T}_ivf 700 python -u -m pytest tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py tests/test_gpu_ivf_shard.py -x -q --timeout 300 --timeout-method thread
for rep in 1 2; do
for v in base rowslast; do
	if [ "$v" = base ]; then unset LANCE_HIP_LIB; else export LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_$v.so; fi
	step ${T}_ab_${v}_$rep 300 python -u bench.py --config c5 --steps 20 --no-cpu-baseline --no-recall --no-sync-leg
	grep -ho '"avg_launch_ms": [0-9.]*\|"value": [0-9.]*' gpurun_out/${T}_ab_${v}_$rep.log | tr '\n' ' '; echo
done
done
unset LANCE_HIP_LIB
step ${T}_prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --no-cpu-baseline --no-recall --no-host-batch --no-sync-leg
python3 tools/trace_kernels.py gpurun_out/${T}_prof_c5/run_kernel_trace.csv 10 10 > gpurun_out/${T}_c5_step_kernels.txt 2>&1
rm -f gpurun_out/${T}_prof_*/run_kernel_trace.csv
cat gpurun_out/${T}_c5_step_kernels.txt
