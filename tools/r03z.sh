source tools/gpu_step.sh
step r03z_k100 600 python -u -m pytest tests/test_gpu_scan8.py -x -v --timeout 300 --timeout-method thread -k "k100 or adversarial or c2_full"
step r03z_c3 600 python -u bench.py --config c3 --steps 10 --no-cpu-baseline --recall-queries 64
step r03z_c2 300 python -u bench.py --steps 20 --no-cpu-baseline --no-recall
step r03z_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
