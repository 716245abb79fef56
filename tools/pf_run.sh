#!/bin/bash
# Development-only (GPU box): scan parity tests on the in-tree library, then the
# prefetch-distance variants (tools/ablate.sh PF*) A/B on C2 and north_star.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -k cosine -m gpu -x -q --timeout 60 --timeout-method thread > gpurun_out/pf_cos.log 2>&1 || { tail -30 gpurun_out/pf_cos.log; exit 1; }
tail -1 gpurun_out/pf_cos.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scan_copy.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pf_pytest.log 2>&1 || { tail -30 gpurun_out/pf_pytest.log; exit 1; }
tail -1 gpurun_out/pf_pytest.log
tools/abl_run.sh -- base "$@" || exit 1
tools/abl_run.sh --config nstar -- base "$@" || exit 1
