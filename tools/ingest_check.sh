#!/bin/bash
# Development-only (GPU box): full GPU suite, then a profiled C2 bench (ingest + int8 build kernel times).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ic_pytest.log 2>&1 || { tail -30 gpurun_out/ic_pytest.log; exit 1; }
tail -1 gpurun_out/ic_pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ic_prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline > gpurun_out/ic_bench.json 2> gpurun_out/ic_bench.err || { tail gpurun_out/ic_bench.err; exit 1; }
python3 - <<'PY'
import csv,glob,json
f=glob.glob('gpurun_out/ic_prof/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'rows_to_i8' in r['Name'] or 'rowaux_kernel' in r['Name'] or 'scan_kernel<0, 1, 2>' in r['Name']: print(r['Name'][:40], r['Calls'], r['AverageNs'])
d=json.load(open('gpurun_out/ic_bench.json')); print(d['value'], d['recall_at_10'])
PY
