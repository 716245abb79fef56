set -o pipefail
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/retry_tests.log 2>&1 || { tail -30 $O/retry_tests.log; exit 1; }
tail -3 $O/retry_tests.log
for sd in 32 128; do
  timeout -k 10 300 python -u bench.py --config c3 --sample-div $sd --no-cpu-baseline --steps 10 > $O/sd.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$O/sd.json'));print('c3','sd',$sd,'ms',d['ms_per_step'],'stats',d['search_stats'],'exact',d['exact_ids_on_recall_subset'])"
done
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $O/c2.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/c2.json'));print('c2 ms',d['ms_per_step'],d['value'],d['search_stats'])"
