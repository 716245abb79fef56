#!/bin/bash
# GPU box: PMC counter groups (tools/pmc_scan.sh) over C2, C3 and C5 plus the per-launch summaries.
set -o pipefail
bash tools/pmc_scan.sh r02p_c2 -- --config c2 --steps 5 --warmup 2 && \
python3 tools/pmc_summary.py r02p_c2 "scan_kernel<0, 1, true>" gpurun_out/r02p_c2_scan_pmc.json --meta config=c2 n=1000000 dim=768 batch=256 scan_elem_bytes=2 && \
bash tools/pmc_scan.sh r02p_c3 -- --config c3 --steps 3 --warmup 1 && \
python3 tools/pmc_summary.py r02p_c3 "scan_kernel<1, 1, true>" gpurun_out/r02p_c3_scan_pmc.json --meta config=c3 n=10000000 dim=768 batch=256 scan_elem_bytes=2 && \
bash tools/pmc_scan.sh r02p_c5 -- --config c5 --steps 3 --warmup 1 && \
python3 tools/pmc_summary.py r02p_c5 "pq_fast_scan_kernel" gpurun_out/r02p_c5_pq_pmc.json --meta config=c5 n=12500000 dim=768 batch=256 && \
echo all-ok
