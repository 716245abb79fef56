#!/bin/bash
# Development-only (GPU box): the cosine regression tests on each named build
# (base = in-tree library, else abl/lib_NAME.so)
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
L=abl/lib_$v.so; [ "$v" = base ] && L=duckdb-lancedb_amd/lib/liblancedb_hip.so
LANCE_HIP_LIB=$L timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -k cosine -m gpu -q --timeout 60 --timeout-method thread > gpurun_out/cos_$v.log 2>&1; echo "$v rc=$?"; tail -1 gpurun_out/cos_$v.log; grep -E "query [0-9]+$|ACTUAL|DESIRED" gpurun_out/cos_$v.log | head -6
done
true
