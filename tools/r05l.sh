#!/bin/bash
# A/B: progressive threshold (split_div) at north_star and C2, interleaved
source tools/gpu_step.sh
T=${1:-r05l}
for i in 1 2; do
for sd in 0 4 8; do
step ${T}_nstar_sd${sd}_$i 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall --no-host-batch --opt split_div=$sd
done
done
for sd in 0 4 8; do
step ${T}_c2_sd${sd} 200 python -u bench.py --steps 30 --no-cpu-baseline --no-recall --no-host-batch --opt split_div=$sd
step ${T}_n8_sd${sd} 200 python -u bench.py --n 1250000 --steps 30 --no-cpu-baseline --no-recall --no-host-batch --opt split_div=$sd
done
