#!/bin/bash
# round 6 C5 step: FETCH_SIZE calibration of the PQ scan's dwordx3 row stream,
# IVF parity, interleaved A/B of the C5 line (lib_dev/lib_NAME.so; base = in-tree)
source tools/gpu_step.sh
T=$1; shift
step ${T}_probe 120 tools/_fetch_probe
step ${T}_probe_pmc 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_probe_pmc -o run -- tools/_fetch_probe
python3 tools/fetch_calib.py gpurun_out/${T}_probe_pmc gpurun_out/${T}_probe.log gpurun_out/${T}_fetch_calib.json
step ${T}_ivf_pytest 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py tests/test_gpu_ivf_shard.py}
for rep in 1; do
for v in "$@"; do
	if [ "$v" = base ]; then unset LANCE_HIP_LIB; else export LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_$v.so; fi
	step ${T}_ab_${v}_$rep 300 python -u bench.py --config c5 --steps 10 --no-cpu-baseline --no-host-batch
	grep -ho '"avg_launch_ms": [0-9.]*\|"value": [0-9.]*' gpurun_out/${T}_ab_${v}_$rep.log | tr '\n' ' '; echo
done
done
unset LANCE_HIP_LIB
step ${T}_prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --no-cpu-baseline --no-recall --no-host-batch
python3 tools/trace_kernels.py gpurun_out/${T}_prof_c5/run_kernel_trace.csv 10 > gpurun_out/${T}_c5_step_kernels.txt 2>&1
rm -f gpurun_out/${T}_prof_c5/run_kernel_trace.csv
cat gpurun_out/${T}_c5_step_kernels.txt
