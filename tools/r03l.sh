source tools/gpu_step.sh
step r03l_scan8 600 python -u -m pytest tests/test_gpu_scan8.py -x -q --timeout 300 --timeout-method thread
step r03l_nstar 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall
step r03l_c2 300 python -u bench.py --steps 20 --no-cpu-baseline
B="python -u bench.py --config nstar --steps 5 --warmup 1 --no-cpu-baseline --no-recall"
step r03l_a24 300 $B --opt scan8_variant=24
step r03l_a22 300 $B --opt scan8_variant=22
step r03l_c2_percall 300 python -u bench.py --steps 300 --no-cpu-baseline --api per_call
