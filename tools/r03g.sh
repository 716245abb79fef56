source tools/gpu_step.sh
step r03g_nstar 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall
step r03g_nstar_nosync 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall --opt scan8_sync=off
step r03g_c2 300 python -u bench.py --steps 20 --no-cpu-baseline
step r03g_c2_nosync 300 python -u bench.py --steps 20 --no-cpu-baseline --opt scan8_sync=off
step r03g_pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
