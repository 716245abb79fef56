#!/bin/bash
# GPU box: C5 list-scan timing of each PQ ablation library (tools/pq_ablate.sh) + the product build.
set -o pipefail
O=gpurun_out; mkdir -p $O
T=${1:-pqabl}; shift
for v in base "$@"; do
  if [ $v = base ]; then lib=""; else lib="abl/lib_pq_$v.so"; fi
  LANCE_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-recall --steps 5 --n 4000000 > $O/${T}_$v.json 2> $O/${T}_$v.err || { echo "$v failed"; tail -5 $O/${T}_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${T}_$v.json'));r=d['roofline'];print('$v',d['value'],r['kernel'],r['avg_launch_ms'],r['pair_rows_per_launch'])"
done
