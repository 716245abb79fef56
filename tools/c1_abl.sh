set -o pipefail
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_filter.py tests/test_gpu_bf16.py > $O/small_tests.log 2>&1 || { tail -40 $O/small_tests.log; exit 1; }
tail -2 $O/small_tests.log
for v in default; do
  if [ $v = default ]; then unset LANCE_HIP_LIB; else export LANCE_HIP_LIB=$PWD/abl/lib_$v.so; fi
  timeout -k 10 300 python -u bench.py --config c1 --steps 2000 --warmup 50 --no-cpu-baseline > $O/c1_$v.json 2>$O/c1.err || { tail -20 $O/c1.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c1_$v.json'));print('$v',d['ms_per_step'],d['roofline']['avg_launch_ms'],d['exact_ids'])"
done
unset LANCE_HIP_LIB
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c1prof -o c1 -- python3 bench.py --config c1 --steps 2000 --warmup 50 --no-cpu-baseline > $O/c1p.log 2>&1 || { tail -20 $O/c1p.log; exit 1; }
find $O/c1prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-100,180-260
