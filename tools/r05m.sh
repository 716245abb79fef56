#!/bin/bash
# IVF_FLAT bound scan with list-order row terms + live bitmap: IVF / filter / multi-device tests, C4 bench + PMC
source tools/gpu_step.sh
T=${1:-r05m}
step ${T}_pytest 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py tests/test_gpu_filter.py tests/test_gpu_multidevice.py
step ${T}_c4 400 python -u bench.py --config c4 --steps 10 --no-cpu-baseline
step ${T}_pmc 900 bash tools/r05_pmc.sh ${T} c4
