set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/f3_pytest.log 2>&1 || { tail -30 $O/f3_pytest.log; exit 1; }
tail -1 $O/f3_pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/f3_smoke.log 2>&1 || { tail -20 $O/f3_smoke.log; exit 1; }
tail -1 $O/f3_smoke.log
timeout -k 10 300 python -u bench.py --config c1 --steps 2000 --warmup 50 > $O/f3_bench_c1.json 2>$O/f3_c1.err || { tail -20 $O/f3_c1.err; exit 1; }
cut -c1-300 $O/f3_bench_c1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/f3_prof_c1 -o run -- python3 bench.py --config c1 --steps 2000 --warmup 50 --no-cpu-baseline > $O/f3_prof_c1.log 2>&1 || { tail -20 $O/f3_prof_c1.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline > $O/f3_bench_c2.json 2>/dev/null || exit 1
cut -c1-200 $O/f3_bench_c2.json
echo done
