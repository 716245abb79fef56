#!/bin/bash
# Development-only (GPU box): the 8-GPU per-rank north_star shape (1.25M x 768, B = 256) under
# sample_div / cand_extra_i8 settings: step time vs the N = 1 step (fixed per-batch costs).
set -o pipefail
mkdir -p gpurun_out
for cfg in "32 0" "64 0" "128 0" "32 48" "64 48"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --config nstar --n 1250000 --steps 20 --no-cpu-baseline --no-recall --opt sample_div=$1 --opt cand_extra_i8=$2 > gpurun_out/rs_$1_$2.json 2>gpurun_out/rs_$1_$2.err || { tail gpurun_out/rs_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/rs_$1_$2.json'));r=d['roofline'];print('sd',$1,'ce',$2,d['value'],d['ms_per_step'],r['avg_launch_ms'],d['search_stats'])"
done
