#!/bin/bash
# round 6: the packed exchange (search writes the rank's packed row, one all-gather +
# lance_hip_merge_topk_packed): merge kernel parity, distributed GPU tests, the rehearsal
# test, and the rehearsal lines packed vs generic beside the exchange-free C2 line
source tools/gpu_step.sh
T=$1
step ${T}_tests 700 python -u -m pytest tests/test_gpu_parity.py -k merge_topk tests/test_distributed.py tests/test_gpu_exchange_rehearsal.py -m gpu -x -q --timeout 300 --timeout-method thread
step ${T}_c2_packed 400 python -u bench.py --steps 20 --no-cpu-baseline --no-host-batch --exchange-rehearsal
step ${T}_c2_generic 400 python -u bench.py --steps 20 --no-cpu-baseline --no-host-batch --exchange-rehearsal --exchange generic
step ${T}_c2 400 python -u bench.py --steps 20 --no-cpu-baseline --no-host-batch
step ${T}_rank_packed 400 python -u bench.py --n 125000 --steps 30 --no-cpu-baseline --no-host-batch --exchange-rehearsal
step ${T}_rank_generic 400 python -u bench.py --n 125000 --steps 30 --no-cpu-baseline --no-host-batch --exchange-rehearsal --exchange generic
step ${T}_rank 400 python -u bench.py --n 125000 --steps 30 --no-cpu-baseline --no-host-batch
step ${T}_nstar_rank_packed 400 python -u bench.py --n 1250000 --steps 30 --no-cpu-baseline --no-host-batch --exchange-rehearsal
for f in c2_packed c2_generic c2 rank_packed rank_generic rank nstar_rank_packed; do grep -h '^{' gpurun_out/${T}_$f.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$f', d['value'], d['ms_per_step'], d.get('exact_ids_on_recall_subset'))"; done
