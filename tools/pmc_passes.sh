#!/bin/bash
# GPU box: separate rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) over the C2
# bench and the C4 / C5 IVF benches (MI355X_MICROARCH.md 'HBM': one counter
# group per run, no trace domains beside it).  Outputs under gpurun_out/pmc_*.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for cfg in c2 c4 c5; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_${cfg}_${ctr} -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-recall > $O/pmc_${cfg}_${ctr}.log 2>&1 || { echo "pmc $cfg $ctr FAILED"; tail -5 $O/pmc_${cfg}_${ctr}.log; exit 1; }
    echo "pmc $cfg $ctr ok"
  done
done
