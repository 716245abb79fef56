#!/bin/bash
# Development-only (GPU box): int8 + flat parity tests on the in-tree build, then TFOLD on/off A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scan_i8.py tests/test_gpu_parity.py tests/test_gpu_scan_copy.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tf_pytest.log 2>&1 || { tail -40 gpurun_out/tf_pytest.log; exit 1; }
tail -1 gpurun_out/tf_pytest.log
tools/abl_run.sh --steps 20 -- base TFOLD0 base TFOLD0 || exit 1
tools/abl_run.sh --config nstar -- base TFOLD0 || exit 1
