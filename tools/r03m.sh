source tools/gpu_step.sh
step r03m_nstar 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall
step r03m_c2 300 python -u bench.py --steps 20 --no-cpu-baseline
step r03m_a24 300 python -u bench.py --config nstar --steps 5 --warmup 1 --no-cpu-baseline --no-recall --opt scan8_variant=24
step r03m_scan8 600 python -u -m pytest tests/test_gpu_scan8.py tests/test_gpu_scan_i8.py -x -q --timeout 300 --timeout-method thread
