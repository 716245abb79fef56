#!/bin/bash
# scan8 pair coupling: GPU parity of the coupled scan, then an interleaved A/B at
# the north_star shape (one 10M x 768 store, tools/ab_opts.py)
source tools/gpu_step.sh
T=$1; shift
step ${T}_couple_pytest 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_scan8.py -k couple
step ${T}_couple_ab 600 python -u tools/ab_opts.py --reps 2 --steps 20 "$@"
cat gpurun_out/${T}_couple_ab.log | grep setting
