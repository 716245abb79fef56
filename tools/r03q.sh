source tools/gpu_step.sh
step r03q_nstar 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall
step r03q_c2 300 python -u bench.py --steps 20 --no-cpu-baseline
step r03q_scan8 600 python -u -m pytest tests/test_gpu_scan8.py -x -q --timeout 300 --timeout-method thread
