#!/bin/bash
# round 6: the multi-rank exchange rehearsed on a one-rank RCCL group (test + the C2 line with it)
source tools/gpu_step.sh
T=$1
step ${T}_test 400 python -u -m pytest tests/test_gpu_exchange_rehearsal.py -x -q --timeout 300 --timeout-method thread
step ${T}_c2 400 python -u bench.py --steps 20 --no-cpu-baseline --no-host-batch --exchange-rehearsal
grep -ho '"value": [0-9.]*\|"exact_ids_on_recall_subset": [a-z]*\|"exchange": "[^"]*"' gpurun_out/${T}_c2.log | tr '\n' ' '; echo
