#!/bin/bash
# round 6: packed exchange — distributed GPU tests + rehearsal tests, and the IVF configs'
# one-rank RCCL rehearsal (packed / generic)
source tools/gpu_step.sh
T=$1
step ${T}_tests 700 python -u -m pytest tests/test_distributed.py tests/test_gpu_exchange_rehearsal.py -m gpu -x -q --timeout 300 --timeout-method thread
step ${T}_c5_packed 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline --exchange-rehearsal --no-sync-leg
step ${T}_c5_generic 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline --exchange-rehearsal --exchange generic --no-sync-leg --no-recall
step ${T}_c4_packed 400 python -u bench.py --config c4 --steps 10 --no-cpu-baseline --exchange-rehearsal --no-sync-leg
for f in c5_packed c5_generic c4_packed; do grep -h '^{' gpurun_out/${T}_$f.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$f', d['value'], d['ms_per_step'], d.get('recall_at_10'))"; done
