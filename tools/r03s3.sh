# session-2 closing check: GPU suite + smoke on the pool_refine / host-status changes, the C2 and
# north_star lines, first-chunk A/B, per-rank shapes, host/per-call lines and kernel stats
source tools/gpu_step.sh
T=${1:-r03t}
step ${T}_pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ${T}_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step ${T}_bench_c2 300 python -u bench.py --steps 20
step ${T}_bench_nstar 600 python -u bench.py --config nstar --steps 10 --recall-queries 64 --cpu-seconds 10
for r in 64 80 128; do
  step ${T}_ab_c2_prf$r 300 python -u bench.py --steps 20 --no-cpu-baseline --no-recall --opt pr_first=$r
done
step ${T}_ab_nstar_prf128 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall --opt pr_first=128
step ${T}_rank_nstar8 300 python -u bench.py --config nstar --n 1250000 --steps 20 --no-cpu-baseline --no-recall
step ${T}_rank_c2s8 300 python -u bench.py --n 125000 --steps 40 --no-cpu-baseline --no-recall
step ${T}_bench_c2_host 300 python -u bench.py --steps 20 --no-cpu-baseline --api host_batch
step ${T}_bench_c2_percall 300 python -u bench.py --steps 500 --no-cpu-baseline --api per_call
step ${T}_bench_c3 600 python -u bench.py --config c3 --steps 10 --recall-queries 64 --cpu-seconds 10
step ${T}_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-recall
step ${T}_prof_nstar 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_nstar -o run -- python3 bench.py --config nstar --steps 5 --no-cpu-baseline --no-recall
