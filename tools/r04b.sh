#!/bin/bash
# round 4: pool_refine with every row load of a round in flight (NI path)
source tools/gpu_step.sh
T=${1:-r04b}
step ${T}_pytest 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_scan8.py tests/test_gpu_scan_i8.py
step ${T}_bench_c2 300 python -u bench.py --steps 20 --no-cpu-baseline
step ${T}_bench_c2_prf64 300 python -u bench.py --steps 20 --no-cpu-baseline --no-host-batch --opt pr_first=64
step ${T}_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-recall --no-host-batch
