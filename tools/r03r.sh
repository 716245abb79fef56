source tools/gpu_step.sh
step r03r_nstar 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline
step r03r_nstar_nosplit 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall --opt split_div=0
step r03r_c2 300 python -u bench.py --steps 20 --no-cpu-baseline
step r03r_c2_nosplit 300 python -u bench.py --steps 20 --no-cpu-baseline --opt split_div=0
step r03r_c2_s4 300 python -u bench.py --steps 20 --no-cpu-baseline --no-recall --opt split_div=4
step r03r_tests 900 python -u -m pytest tests/test_gpu_scan8.py tests/test_gpu_scan_i8.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread
