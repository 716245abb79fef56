set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ivf.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ivf1.log 2>&1; rc=$?
tail -40 gpurun_out/ivf1.log
exit $rc
