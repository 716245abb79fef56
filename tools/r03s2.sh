# session-2: pool_refine with gather-time statistics; C2 line with recall first, the first-chunk
# A/B, the step timelines (kernel trace) and pool_refine phase stamps, then the GPU suite
source tools/gpu_step.sh
T=${1:-r03s2}
step ${T}_bench_c2 300 python -u bench.py --steps 20
for r in 96 112 120; do
  step ${T}_c2_prf$r 300 python -u bench.py --steps 20 --no-cpu-baseline --no-recall --opt pr_first=$r
done
step ${T}_trace_c2 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_trace_c2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-recall
step ${T}_trace_c2s8 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_trace_c2s8 -o run -- python3 bench.py --n 125000 --steps 5 --warmup 2 --no-cpu-baseline --no-recall
LANCE_HIP_LIB=abl/lib_PRPROF.so step ${T}_prprof_c2 300 python3 -u bench.py --steps 5 --warmup 8 --no-cpu-baseline --no-recall
step ${T}_pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ${T}_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step ${T}_bench_nstar 600 python -u bench.py --config nstar --steps 10 --recall-queries 64 --cpu-seconds 10
