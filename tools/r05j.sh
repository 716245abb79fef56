#!/bin/bash
# PQ fast scan (bound read lagged one round) and IVF_FLAT bound scan (XCD-major (block, group) items):
# IVF parity tests, C4 / C5 benches, PQ phase stamps, PMC traffic of both
source tools/gpu_step.sh
T=${1:-r05j}
step ${T}_pytest 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py tests/test_gpu_multidevice.py
step ${T}_c5 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
step ${T}_c4 400 python -u bench.py --config c4 --steps 10 --no-cpu-baseline
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_pqprof.so step ${T}_c5_prof 400 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-recall
grep -h PROF gpurun_out/${T}_c5_prof.log
step ${T}_pmc 900 bash tools/r05_pmc.sh ${T} c4 c5
