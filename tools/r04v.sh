#!/bin/bash
# round 4: sample_div A/B after the cheaper tilemin score (no code change: index option),
# interleaved on one box -- C2 (default 16), per-rank north_star shape (16), north_star (32)
source tools/gpu_step.sh
T=${1:-r04v}
B="python -u bench.py --steps 50 --no-cpu-baseline --no-host-batch --recall-queries 32"
for r in a b; do
	for sd in 8 12 16 24; do step ${T}_c2_sd${sd}${r} 120 $B --sample-div $sd; done
done
for sd in 8 16 32; do step ${T}_r8_sd${sd} 120 $B --n 1250000 --sample-div $sd; done
for sd in 16 32 48; do step ${T}_ns_sd${sd} 200 python -u bench.py --config nstar --steps 10 --recall-queries 32 --no-cpu-baseline --no-host-batch --sample-div $sd; done
