#!/bin/bash
# PQ fast scan with 8 queries per item: IVF parity tests, C5 A/B (pq_group 8 vs 4), rocprof of the C5 bench
source tools/gpu_step.sh
T=${1:-r05g}
step ${T}_pytest 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py
step ${T}_c5_g8 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
step ${T}_c5_g4 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline --opt pq_group=4
step ${T}_prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --no-cpu-baseline --no-recall
