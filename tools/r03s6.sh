# final check of the committed tree (in-tree library as the driver will load it)
source tools/gpu_step.sh
T=${1:-r03w}
step ${T}_pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ${T}_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step ${T}_bench_c2 300 python -u bench.py
