#!/bin/bash
# GPU box: IVF parity tests + C4 benches (bound scan / exact scan) + scan-kernel stage ablations.
set -o pipefail
T=${1:-ivf}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
echo "== pytest ivf"
timeout -k 10 500 python -u -m pytest tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/${T}_pytest.log 2>&1 || { tail -40 $O/${T}_pytest.log; exit 1; }
grep -E "C5 params|C4 params|passed|failed" $O/${T}_pytest.log
for b in c4:--config,c4 c4x:--config,c4,--opt,ivf_flat_scan=exact,--no-cpu-baseline; do
  name=${b%%:*}; args=${b#*:}; args=${args//,/ }
  echo "== bench $name ($args)"
  timeout -k 10 500 python -u bench.py --steps 10 $args > $O/${T}_bench_$name.json 2> $O/${T}_bench_$name.err || { tail -20 $O/${T}_bench_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${T}_bench_$name.json'));r=d['roofline'];print('$name',d['value'],d.get('recall_at_10'),r['kernel'],r['avg_launch_ms'],r['frac'],(d.get('cpu_baseline') or {}).get('value'))"
done
echo done
