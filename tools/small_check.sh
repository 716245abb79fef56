set -o pipefail
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/small_tests.log 2>&1 || { tail -40 $O/small_tests.log; exit 1; }
tail -3 $O/small_tests.log
timeout -k 10 300 python -u bench.py --config c1 > $O/c1.json 2>$O/c1.err || { tail -20 $O/c1.err; exit 1; }
cat $O/c1.json
