#!/bin/bash
# round 6 bench pass: the driver's C2 command, the north_star line and per-rank shapes, the C5 step trace
source tools/gpu_step.sh
T=$1
step ${T}_bench_c2 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step ${T}_bench_nstar 300 python -u bench.py --config nstar --steps 10 --recall-queries 64 --no-cpu-baseline --no-host-batch
step ${T}_rank_nstar8 200 python -u bench.py --n 1250000 --steps 30 --no-cpu-baseline --no-host-batch
step ${T}_rank_c2s8 200 python -u bench.py --n 125000 --steps 30 --no-cpu-baseline --no-host-batch
CFG=c5 bash tools/closing_check.sh S $T
grep -ho '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*' gpurun_out/${T}_bench_*.log gpurun_out/${T}_rank_*.log gpurun_out/${T}_c5.log
