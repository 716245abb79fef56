#!/bin/bash
# GPU box: C2 bench timing of each rscan ablation library (tools/rs_ablate.sh) + the product build.
set -o pipefail
O=gpurun_out; mkdir -p $O
T=${1:-rsabl}; shift
for v in base "$@"; do
  if [ $v = base ]; then lib=""; else lib="abl/lib_rs_$v.so"; fi
  LANCE_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-recall --steps 10 --opt rscan=1 > $O/${T}_$v.json 2> $O/${T}_$v.err || { echo "$v failed"; tail -5 $O/${T}_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${T}_$v.json'));r=d['roofline'];print('$v',r['kernel'],r['avg_launch_ms'])"
done
