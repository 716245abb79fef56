#!/bin/bash
# PQ fast scan: XCD-major item claims + two rounds of codes in flight; IVF tests, C5 bench, C5 PMC traffic
source tools/gpu_step.sh
T=${1:-r05i}
step ${T}_pytest 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py
step ${T}_c5 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
step ${T}_pmc 900 bash tools/r05_pmc.sh ${T} c5
