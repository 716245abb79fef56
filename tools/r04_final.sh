#!/bin/bash
# round-4 closing check on one MI355X: the committed tree's GPU suite and smoke, the
# driver's bench command, its rocprofv3 kernel stats, north_star / C3 lines, per-rank shapes
source tools/gpu_step.sh
T=${1:-r04z}
step ${T}_pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ${T}_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step ${T}_bench_c2 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step ${T}_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch
python3 tools/trace_kernels.py gpurun_out/${T}_prof_c2/run_kernel_trace.csv 20 > gpurun_out/${T}_c2_step_kernels.txt 2>&1
step ${T}_bench_nstar 300 python -u bench.py --config nstar --steps 10 --recall-queries 64 --no-cpu-baseline --no-host-batch
step ${T}_rank_c2s8 200 python -u bench.py --n 125000 --steps 30 --no-cpu-baseline --no-host-batch
step ${T}_rank_nstar8 200 python -u bench.py --n 1250000 --steps 30 --no-cpu-baseline --no-host-batch
step ${T}_bench_c3 400 python -u bench.py --config c3 --steps 10 --recall-queries 64 --no-cpu-baseline --no-host-batch
step ${T}_bench_c4 400 python -u bench.py --config c4 --steps 10 --no-cpu-baseline
