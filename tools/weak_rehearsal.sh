set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline > $O/ws_n1.json 2> $O/ws_n1.err || exit 1
cat $O/ws_n1.json
for nb in "500000 512" "250000 1024" "125000 2048"; do set -- $nb
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --n $1 --batch $2 > $O/ws_$1.json 2> $O/ws_$1.err || exit 1
cat $O/ws_$1.json; done
