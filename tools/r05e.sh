#!/bin/bash
# multi-device handles (two shards on device 0) in-process and in the torch-free C++ caller
source tools/gpu_step.sh
T=${1:-r05e}
step ${T}_pytest 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multidevice.py tests/test_gpu_abi_process.py
