#!/bin/bash
# round 4, first GPU check: the new / changed parity tests and the C2 line
source tools/gpu_step.sh
T=${1:-r04a}
step ${T}_pytest_new 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_scan8.py::test_split_div_progressive_threshold tests/test_gpu_scan8.py::test_release_build_rejects_development_knobs tests/test_distributed.py -m gpu tests/test_gpu_ivf_params.py::test_c4_ivf_flat_nlist4096_nprobe64
step ${T}_bench_c2 300 python -u bench.py --steps 20
