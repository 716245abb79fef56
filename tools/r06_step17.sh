#!/bin/bash
# round 6: the device merge without its host wait: distributed GPU tests, the rehearsal test,
# and the C2 line with and without the one-rank RCCL exchange
source tools/gpu_step.sh
T=$1
step ${T}_tests 600 python -u -m pytest tests/test_distributed.py tests/test_gpu_exchange_rehearsal.py -m gpu -x -q --timeout 300 --timeout-method thread
step ${T}_c2_rehearsal 400 python -u bench.py --steps 20 --no-cpu-baseline --no-host-batch --exchange-rehearsal
step ${T}_c2 400 python -u bench.py --steps 20 --no-cpu-baseline --no-host-batch
step ${T}_rank_rehearsal 400 python -u bench.py --n 125000 --steps 30 --no-cpu-baseline --no-host-batch --exchange-rehearsal
step ${T}_nstar_rank_rehearsal 400 python -u bench.py --n 1250000 --steps 30 --no-cpu-baseline --no-host-batch --exchange-rehearsal
for f in c2_rehearsal c2 rank_rehearsal nstar_rank_rehearsal; do grep -h '^{' gpurun_out/${T}_$f.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$f', d['value'], d['ms_per_step'], d.get('exact_ids_on_recall_subset'))"; done
