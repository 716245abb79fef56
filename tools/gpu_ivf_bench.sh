#!/bin/bash
# GPU box: IVF bench lines (C4 IVF-Flat, C5 IVF-PQ, one 12.5M-row shard each).
# usage: tools/gpu_ivf_bench.sh TAG [extra bench args]
set -o pipefail
T=${1:-ivf}
shift
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --config c4 --steps 10 --cpu-seconds 8 "$@" > $O/${T}_c4.json 2> $O/${T}_c4.err || { echo "c4 FAILED"; tail -30 $O/${T}_c4.err; exit 1; }
cat $O/${T}_c4.json
timeout -k 10 500 python -u bench.py --config c5 --steps 10 --cpu-seconds 8 "$@" > $O/${T}_c5.json 2> $O/${T}_c5.err || { echo "c5 FAILED"; tail -30 $O/${T}_c5.err; exit 1; }
cat $O/${T}_c5.json
