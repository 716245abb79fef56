#!/bin/bash
# IVF_FLAT bound scan with list-order row terms: IVF tests, C4 bench, C4 PMC traffic
source tools/gpu_step.sh
T=${1:-r05k}
step ${T}_pytest 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py tests/test_gpu_filter.py
step ${T}_c4 400 python -u bench.py --config c4 --steps 10 --no-cpu-baseline
step ${T}_pmc 900 bash tools/r05_pmc.sh ${T} c4
