set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/sel_pytest.log 2>&1 || { tail -30 $O/sel_pytest.log; exit 1; }
tail -2 $O/sel_pytest.log
for shape in "1000000 256" "125000 2048" "500000 512"; do set -- $shape
  timeout -k 10 200 python -u bench.py --n $1 --batch $2 --steps 20 --no-cpu-baseline > $O/sel.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$O/sel.json'));print('n',$1,'b',$2,'qps',d['value'],'ms',d['ms_per_step'],'scan',d['roofline']['avg_launch_ms'],'fb',d['search_stats']['fallback_queries'],'exact',d['exact_ids_on_recall_subset'])"
done
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --no-cpu-baseline > $O/sel_c3.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/sel_c3.json'));print('c3 qps',d['value'],'ms',d['ms_per_step'],'fb',d['search_stats']['fallback_queries'],'exact',d['exact_ids_on_recall_subset'])"
