#!/bin/bash
# round 5: the new drop-in / threading / async / C3 full-size tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_abi_process.py tests/test_gpu_threads.py \
  "tests/test_gpu_scan8.py::test_async_pipeline_matches_sync" \
  "tests/test_gpu_scan8.py::test_async_rerun_and_fallback_with_next_pass_in_flight" \
  "tests/test_gpu_nstar.py::test_c3_full_size_bf16_dot_k100" > gpurun_out/r05a_pytest.log 2>&1
rc=$?
tail -30 gpurun_out/r05a_pytest.log
exit $rc
