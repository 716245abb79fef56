#!/bin/bash
# round 4: IVF benches (C4 list-order rows, C5 LUT loads) and the north_star line
source tools/gpu_step.sh
T=${1:-r04i}
step ${T}_bench_c4 400 python -u bench.py --config c4 --steps 10 --no-cpu-baseline
step ${T}_bench_c5 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
step ${T}_bench_nstar 300 python -u bench.py --config nstar --steps 10 --recall-queries 64 --no-cpu-baseline --no-host-batch
