#!/bin/bash
# Development-only (GPU box): int8 tests + a profiled C2 bench (int8 copy build time, scan time).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_scan_i8.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gs_pytest.log 2>&1 || { tail -30 gpurun_out/gs_pytest.log; exit 1; }
tail -1 gpurun_out/gs_pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gs_prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline > gpurun_out/gs_bench.json 2> gpurun_out/gs_bench.err || { tail gpurun_out/gs_bench.err; exit 1; }
grep -rh "rows_to_i8\|scan_kernel<0, 1, 2>" gpurun_out/gs_prof --include=run_kernel_stats.csv | cut -c1-160
python3 -c "import json;d=json.load(open('gpurun_out/gs_bench.json'));print(d['value'],d['recall_at_10'])"
