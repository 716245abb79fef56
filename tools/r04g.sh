#!/bin/bash
# round 4: scan8 tilemin sample pass, IVF_FLAT list-order rows, PQ LUT loads
source tools/gpu_step.sh
T=${1:-r04g}
step ${T}_pytest 700 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_scan8.py tests/test_gpu_parity.py tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py
step ${T}_bench_c2 200 python -u bench.py --steps 30 --no-cpu-baseline
step ${T}_tr_c2 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
python3 tools/trace_kernels.py gpurun_out/${T}_tr_c2/run_kernel_trace.csv 20 > gpurun_out/${T}_tr_c2.txt 2>&1
