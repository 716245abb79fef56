#!/bin/bash
# Development-only (GPU box): full GPU suite + smoke on the in-tree build, then the
# phase-timer breakdown of the int8 and bf16 scans (abl/lib_PROF.so).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fc_pytest.log 2>&1 || { tail -30 gpurun_out/fc_pytest.log; exit 1; }
tail -1 gpurun_out/fc_pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fc_smoke.log 2>&1 || { tail -20 gpurun_out/fc_smoke.log; exit 1; }
tail -1 gpurun_out/fc_smoke.log
for v in on off; do LANCE_HIP_LIB=abl/lib_PROF.so timeout -k 10 200 python tools/prof_scan.py --scan-i8 $v > gpurun_out/fc_prof_$v.txt 2>&1 || { tail gpurun_out/fc_prof_$v.txt; exit 1; }; cat gpurun_out/fc_prof_$v.txt; done
