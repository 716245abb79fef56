#!/bin/bash
# closing check on one MI355X (usage: tools/closing_check.sh A|B|C|S TAG), in separate calls:
#   A: the committed tree's GPU suite and smoke
#   B: the driver's bench command, its rocprofv3 kernel stats, the other configs' lines, per-rank
#      shapes, the in-process two-shard form, the per-call legs (Python and torch-free C++), and
#      the C5 step's kernel stats
#   C: PMC traffic passes of each config's dominant kernel (tools/pmc_configs.sh)
#   S: one config's step: bench line + rocprofv3 kernel trace (CFG=c2|nstar|c4|c5, STEPS)
#   E: the multi-rank exchange rehearsed on one GPU (one-rank RCCL group): the rehearsal test, then
#      C2 / per-rank shapes / C5 with the packed and the generic exchange beside no exchange
source tools/gpu_step.sh
T=${2:-r06x}
case $1 in
A)
	step ${T}_pytest 1100 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread
	step ${T}_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
	;;
B)
	step ${T}_bench_c2 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
	step ${T}_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-recall --no-host-batch
	python3 tools/trace_kernels.py gpurun_out/${T}_prof_c2/run_kernel_trace.csv 20 > gpurun_out/${T}_c2_step_kernels.txt 2>&1
	step ${T}_bench_nstar 300 python -u bench.py --config nstar --steps 10 --recall-queries 64 --no-cpu-baseline --no-host-batch
	step ${T}_bench_c3 400 python -u bench.py --config c3 --steps 10 --recall-queries 64 --no-cpu-baseline --no-host-batch
	step ${T}_bench_c4 400 python -u bench.py --config c4 --steps 10 --no-cpu-baseline
	step ${T}_bench_c5 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
	step ${T}_bench_c1 300 python -u bench.py --config c1 --steps 20 --no-cpu-baseline
	step ${T}_rank_c2s8 200 python -u bench.py --n 125000 --steps 30 --no-cpu-baseline --no-host-batch
	step ${T}_rank_nstar8 200 python -u bench.py --n 1250000 --steps 30 --no-cpu-baseline --no-host-batch
	step ${T}_inproc 300 python -u bench.py --inproc --inproc-devices 0,0 --steps 20 --no-cpu-baseline --no-host-batch
	step ${T}_percall_c2 300 python -u bench.py --api per_call --steps 256 --warmup 16 --no-cpu-baseline
	step ${T}_percall_nstar 400 python -u bench.py --config nstar --api per_call --steps 64 --warmup 8 --no-cpu-baseline
	step ${T}_cpp_percall 600 python -u tools/cpp_percall.py
	step ${T}_prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c5 -o run -- python3 bench.py --config c5 --steps 10 --no-cpu-baseline --no-recall --no-host-batch --no-sync-leg
	python3 tools/trace_kernels.py gpurun_out/${T}_prof_c5/run_kernel_trace.csv 10 10 > gpurun_out/${T}_c5_step_kernels.txt 2>&1
	rm -f gpurun_out/${T}_prof_c*/run_kernel_trace.csv.gz
	;;
C)
	step ${T}_pmc 1100 bash tools/pmc_configs.sh $T c2 nstar c3 c4 c5
	;;
S)
	C=${CFG:-c2}
	N=${STEPS:-10}
	step ${T}_${C} 400 python -u bench.py --config $C --steps $N --no-cpu-baseline
	step ${T}_prof_${C} 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_${C} -o run -- python3 bench.py --config $C --steps $N --no-cpu-baseline --no-recall --no-host-batch
	python3 tools/trace_kernels.py gpurun_out/${T}_prof_${C}/run_kernel_trace.csv $N > gpurun_out/${T}_${C}_step_kernels.txt 2>&1
	rm -f gpurun_out/${T}_prof_${C}/run_kernel_trace.csv
	cat gpurun_out/${T}_${C}_step_kernels.txt
	;;
E)
	step ${T}_xtests 700 python -u -m pytest tests/test_distributed.py tests/test_gpu_exchange_rehearsal.py -m gpu -x -q --timeout 300 --timeout-method thread
	R="--no-cpu-baseline --no-host-batch --exchange-rehearsal"
	step ${T}_x_c2_packed 400 python -u bench.py --steps 20 $R
	step ${T}_x_c2_generic 400 python -u bench.py --steps 20 $R --exchange generic
	step ${T}_x_c2 400 python -u bench.py --steps 20 --no-cpu-baseline --no-host-batch
	step ${T}_x_rank_packed 400 python -u bench.py --n 125000 --steps 30 $R
	step ${T}_x_rank_generic 400 python -u bench.py --n 125000 --steps 30 $R --exchange generic
	step ${T}_x_rank 400 python -u bench.py --n 125000 --steps 30 --no-cpu-baseline --no-host-batch
	step ${T}_x_nstar_rank_packed 400 python -u bench.py --n 1250000 --steps 30 $R
	step ${T}_x_c5_packed 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline --exchange-rehearsal --no-sync-leg
	;;
esac
