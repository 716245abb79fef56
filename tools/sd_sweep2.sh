set -o pipefail
O=gpurun_out
for cfg in c2 c3; do
  for sd in 16 32 64 128; do
    extra=""; [ $cfg = c3 ] && extra="--steps 10"
    timeout -k 10 300 python -u bench.py --config $cfg --sample-div $sd --no-cpu-baseline $extra > $O/sd.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$O/sd.json'));print('$cfg','sd',$sd,'ms',d['ms_per_step'],'scan',d['roofline']['avg_launch_ms'],'pool',d['search_stats']['max_pool'],'fb',d['search_stats']['fallback_queries'],'exact',d['exact_ids_on_recall_subset'])"
  done
done
