#!/bin/bash
# A/B: pool_refine at 1024 threads (dev lib) vs HEAD, interleaved; bench --inproc rehearsal (two shards on device 0)
source tools/gpu_step.sh
T=${1:-r05f}
DEV=duckdb-lancedb_amd/lib_dev/lib_pr1024.so
step ${T}_par1024 300 env LANCE_HIP_LIB=$DEV python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_scan8.py -k "c2_full_size or every_ld or split_div"
for i in 1 2; do
step ${T}_c2_head_$i 200 python -u bench.py --steps 30 --no-cpu-baseline --no-recall --no-host-batch
step ${T}_c2_pr1024_$i 200 env LANCE_HIP_LIB=$DEV python -u bench.py --steps 30 --no-cpu-baseline --no-recall --no-host-batch
step ${T}_n8_head_$i 200 python -u bench.py --n 1250000 --steps 30 --no-cpu-baseline --no-recall --no-host-batch
step ${T}_n8_pr1024_$i 200 env LANCE_HIP_LIB=$DEV python -u bench.py --n 1250000 --steps 30 --no-cpu-baseline --no-recall --no-host-batch
done
export LANCE_HIP_LIB=$DEV
step ${T}_prof_pr1024 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_pr1024 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch --opt pr_first=0
unset LANCE_HIP_LIB
step ${T}_inproc 300 python -u bench.py --inproc --inproc-devices 0,0 --steps 20 --no-cpu-baseline --no-host-batch
