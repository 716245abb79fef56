#!/bin/bash
# GPU box: IVF parity tests (incl. C4/C5 parameters) + C5 benches (fast scan fp8 / f32 queries, f32-LUT scan).
# usage: tools/pq_check.sh TAG [quick]
set -o pipefail
T=${1:-pq}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
echo "== pytest ivf"
timeout -k 10 500 python -u -m pytest tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/${T}_pytest.log 2>&1 || { tail -40 $O/${T}_pytest.log; exit 1; }
grep -E "C5 params|C4 params|passed|failed" $O/${T}_pytest.log
for b in c5:--config,c5 c5f32q:--config,c5,--pq-query,f32,--no-cpu-baseline c5old:--config,c5,--pq-scan,exact_lut,--no-cpu-baseline,--refine-sweep,10; do
  name=${b%%:*}; args=${b#*:}; args=${args//,/ }
  echo "== bench $name ($args)"
  timeout -k 10 500 python -u bench.py --steps 10 $args > $O/${T}_bench_$name.json 2> $O/${T}_bench_$name.err || { tail -20 $O/${T}_bench_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${T}_bench_$name.json'));r=d['roofline'];print('$name',d['value'],d.get('recall_at_10'),d.get('recall_at_10_by_refine'),r['kernel'],r['avg_launch_ms'],r['frac'],(d.get('cpu_baseline') or {}).get('value'))"
done
echo "== rocprof c5"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --no-cpu-baseline --no-recall > $O/${T}_prof_c5.log 2>&1 || { tail -20 $O/${T}_prof_c5.log; exit 1; }
grep -E "pq_|ivf_" $O/${T}_prof_c5/run_kernel_stats.csv | cut -c1-70,200-330
echo done
