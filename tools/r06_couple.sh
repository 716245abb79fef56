#!/bin/bash
# round 6: scan8 pair coupling parity, then interleaved option A/Bs on one store per shape
# (tools/ab_opts.py): north_star 10M, the per-rank north_star shape 1.25M, C2 1M
source tools/gpu_step.sh
T=$1
step ${T}_couple_pytest 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_scan8.py -k couple
step ${T}_ab_nstar 500 python -u tools/ab_opts.py --n 10000000 --reps 2 --steps 20 s8_couple=0 s8_couple=8 s8_couple=32
step ${T}_ab_rank 300 python -u tools/ab_opts.py --n 1250000 --reps 3 --steps 40 s8_couple=0,split_div=0 s8_couple=8,split_div=0 s8_couple=0,split_div=4 s8_couple=0,split_div=8
step ${T}_ab_c2 300 python -u tools/ab_opts.py --n 1000000 --reps 3 --steps 40 s8_couple=0,split_div=0 s8_couple=8,split_div=0 s8_couple=0,split_div=4
grep -h setting gpurun_out/${T}_ab_*.log
