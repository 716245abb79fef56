#!/bin/bash
# PQ fast scan: parity tests, C5 launch time, per-phase cycles (lib_dev/lib_pqprof.so)
source tools/gpu_step.sh
T=$1
step ${T}_pytest 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_ivf_params.py tests/test_gpu_ivf.py}
bash tools/r05_ab.sh $T base && bash tools/r05_prof.sh $T pqprof
