# round-3 closing check on one MI355X: tests, every config's bench line, the
# per-rank scaling shapes, the host-API / per-call lines, kernel stats and the
# scan8 PMC passes (one counter group per rocprofv3 run, no trace domains)
source tools/gpu_step.sh
T=${1:-r03f}
PART=${2:-1}
if [ "$PART" = 1 ]; then
step ${T}_pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ${T}_bench_c2 300 python -u bench.py --steps 20
step ${T}_bench_nstar 600 python -u bench.py --config nstar --steps 10 --recall-queries 64 --cpu-seconds 10
step ${T}_bench_c1 300 python -u bench.py --config c1 --steps 2000
step ${T}_bench_c3 600 python -u bench.py --config c3 --steps 10 --recall-queries 64 --cpu-seconds 10
step ${T}_bench_c2_host 300 python -u bench.py --steps 20 --no-cpu-baseline --api host_batch
step ${T}_bench_c2_percall 300 python -u bench.py --steps 500 --no-cpu-baseline --api per_call
step ${T}_bench_nstar_percall 300 python -u bench.py --config nstar --steps 40 --no-cpu-baseline --api per_call --recall-queries 16
step ${T}_rank_nstar8 300 python -u bench.py --config nstar --n 1250000 --steps 20 --no-cpu-baseline --no-recall
step ${T}_rank_c2s8 300 python -u bench.py --n 125000 --steps 40 --no-cpu-baseline --no-recall
fi
if [ "$PART" = 2 ]; then
step ${T}_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-recall
step ${T}_prof_nstar 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_nstar -o run -- python3 bench.py --config nstar --steps 5 --no-cpu-baseline --no-recall
P="--kernel-include-regex scan8 --output-format csv"
for cfg in c2 nstar; do
  B="python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-recall"
  step ${T}_pmc_${cfg}_fetch 240 rocprofv3 --pmc FETCH_SIZE $P -d gpurun_out/${T}_pmc_${cfg}_fetch -o run -- $B
  step ${T}_pmc_${cfg}_write 240 rocprofv3 --pmc WRITE_SIZE $P -d gpurun_out/${T}_pmc_${cfg}_write -o run -- $B
  step ${T}_pmc_${cfg}_tcc 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum $P -d gpurun_out/${T}_pmc_${cfg}_tcc -o run -- $B
  step ${T}_pmc_${cfg}_sq 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE $P -d gpurun_out/${T}_pmc_${cfg}_sq -o run -- $B
  step ${T}_pmc_${cfg}_lds 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS $P -d gpurun_out/${T}_pmc_${cfg}_lds -o run -- $B
done
fi
if [ "$PART" = 3 ]; then
step ${T}_bench_c4 600 python -u bench.py --config c4 --steps 10
step ${T}_bench_c5 600 python -u bench.py --config c5 --steps 10
fi
