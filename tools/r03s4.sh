# pool_refine refine rounds: double-buffered row loads, 12 candidates per wave (in-tree)
# against the committed kernel (abl/lib_head.so), then the GPU suite on the in-tree library
source tools/gpu_step.sh
T=${1:-r03u}
step ${T}_new_c2 300 python -u bench.py --steps 30 --no-cpu-baseline --no-recall
LANCE_HIP_LIB=abl/lib_head.so step ${T}_head_c2 300 python -u bench.py --steps 30 --no-cpu-baseline --no-recall
step ${T}_new_c2b 300 python -u bench.py --steps 30 --no-cpu-baseline --no-recall
LANCE_HIP_LIB=abl/lib_head.so step ${T}_head_c2b 300 python -u bench.py --steps 30 --no-cpu-baseline --no-recall
step ${T}_new_nstar 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall
LANCE_HIP_LIB=abl/lib_head.so step ${T}_head_nstar 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall
step ${T}_new_c2s8 300 python -u bench.py --n 125000 --steps 40 --no-cpu-baseline --no-recall
LANCE_HIP_LIB=abl/lib_head.so step ${T}_head_c2s8 300 python -u bench.py --n 125000 --steps 40 --no-cpu-baseline --no-recall
step ${T}_pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ${T}_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step ${T}_bench_c2 300 python -u bench.py --steps 20
