# final check with the auto sample_div: GPU suite, smoke, C2 and north_star lines
source tools/gpu_step.sh
T=${1:-r03y}
step ${T}_pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ${T}_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step ${T}_bench_c2 300 python -u bench.py
step ${T}_bench_nstar 600 python -u bench.py --config nstar --steps 10 --recall-queries 64 --cpu-seconds 10
