source tools/gpu_step.sh
step r03u_scan8 600 python -u -m pytest tests/test_gpu_scan8.py -x -q --timeout 300 --timeout-method thread
step r03u_nstar 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline
step r03u_nstar_nosplit 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall --opt split_div=0
step r03u_c2 300 python -u bench.py --steps 20 --no-cpu-baseline
step r03u_c2_nosplit 300 python -u bench.py --steps 20 --no-cpu-baseline --no-recall --opt split_div=0
step r03u_a34 300 python -u bench.py --config nstar --steps 5 --warmup 1 --no-cpu-baseline --no-recall --opt scan8_variant=34
