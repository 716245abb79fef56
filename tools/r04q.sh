#!/bin/bash
# scan8 append: per-u flush loop (any number of entries), tail flush with every load in
# flight; parity + split bisect case; interleaved A/B incl. pr_first=128
source tools/gpu_step.sh
T=${1:-r04q}
step ${T}_pytest 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scan8.py tests/test_gpu_scan_i8.py tests/test_gpu_parity.py tests/test_gpu_nstar.py
step ${T}_split 300 python -u tools/dbg_split.py l2
for rep in 1 2; do
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_base.so step ${T}_ab_base$rep 200 python -u bench.py --steps 30 --no-cpu-baseline --no-host-batch --no-recall
step ${T}_ab_new$rep 200 python -u bench.py --steps 30 --no-cpu-baseline --no-host-batch --no-recall
step ${T}_ab_prf128_$rep 200 python -u bench.py --steps 30 --no-cpu-baseline --no-host-batch --no-recall --opt pr_first=128
done
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_s8prof.so step ${T}_s8prof 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-recall --no-host-batch --sync
