set -o pipefail
O=gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --config c1 --steps 2000 --warmup 50 > $O/c1.json 2>$O/c1.err || { tail -20 $O/c1.err; exit 1; }
cat $O/c1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c1prof -o c1 -- python3 bench.py --config c1 --steps 2000 --warmup 50 --no-cpu-baseline > $O/c1p.log 2>&1 || { tail -20 $O/c1p.log; exit 1; }
find $O/c1prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
