source tools/gpu_step.sh
step r03b_c2 300 python -u bench.py --steps 20 --no-cpu-baseline
step r03b_nstar 400 python -u bench.py --config nstar --steps 10 --no-cpu-baseline
for v in 1 2 3 4 5 6; do
  step r03b_nstar_v$v 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall --opt scan8_variant=$v
done
step r03b_pytest 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
