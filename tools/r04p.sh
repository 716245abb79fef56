#!/bin/bash
# bisect the split_div failure: new scan8 only, new pool_refine only, both
source tools/gpu_step.sh
T=${1:-r04p}
for v in s8new knnnew base; do
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_$v.so step ${T}_split_$v 300 python -u tools/dbg_split.py l2
done
step ${T}_split_new 300 python -u tools/dbg_split.py l2 dot
