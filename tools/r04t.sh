#!/bin/bash
# round-4 validation of the last kernel changes (PQ two code buffers, pool_refine small later
# rounds + one-pass later chunks, scan8 tilemin score): full GPU suite + smoke, the driver's
# C2 command and its kernel trace, C2 / north_star one query per call (scan8 QB = 1), C5 line + PQ phases, north_star, C3, C4, per-rank shapes
source tools/gpu_step.sh
T=${1:-r04t}
step ${T}_pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ${T}_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step ${T}_bench_c2 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step ${T}_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
python3 tools/trace_kernels.py gpurun_out/${T}_prof_c2/run_kernel_trace.csv 20 > gpurun_out/${T}_c2_step_kernels.txt 2>&1
step ${T}_bench_c2_percall 200 python -u bench.py --api per_call --steps 500 --warmup 3 --no-cpu-baseline
step ${T}_bench_c5 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_pqprof.so step ${T}_pqprof 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-recall
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_prprof.so step ${T}_prprof 200 python -u bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --sync
step ${T}_bench_nstar 300 python -u bench.py --config nstar --steps 10 --recall-queries 64 --no-cpu-baseline --no-host-batch
step ${T}_rank_c2s8 200 python -u bench.py --n 125000 --steps 30 --no-cpu-baseline --no-host-batch
step ${T}_rank_nstar8 200 python -u bench.py --n 1250000 --steps 30 --no-cpu-baseline --no-host-batch
step ${T}_bench_nstar_percall 200 python -u bench.py --config nstar --api per_call --steps 100 --warmup 3 --no-cpu-baseline
