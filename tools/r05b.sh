#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_scan8.py::test_async_rerun_and_fallback_with_next_pass_in_flight" \
  "tests/test_gpu_nstar.py::test_c3_full_size_bf16_dot_k100" > gpurun_out/r05b_pytest.log 2>&1
rc=$?
tail -30 gpurun_out/r05b_pytest.log
exit $rc
