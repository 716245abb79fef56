source tools/gpu_step.sh
step r03f_scan8 600 python -u -m pytest tests/test_gpu_scan8.py -x -q --timeout 300 --timeout-method thread -k "every_ld or c2_full or query_batches"
step r03f_nstar 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall
step r03f_nstar_nosync 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall --opt scan8_sync=off
step r03f_c2 300 python -u bench.py --steps 20 --no-cpu-baseline
step r03f_c2_nosync 300 python -u bench.py --steps 20 --no-cpu-baseline --opt scan8_sync=off
P="--kernel-include-regex scan8 --output-format csv"
B="python3 bench.py --config nstar --steps 3 --warmup 1 --no-cpu-baseline --no-recall"
step r03f_pmc_tcc 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum $P -d gpurun_out/r03f_pmc_tcc -o run -- $B
step r03f_pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE $P -d gpurun_out/r03f_pmc_fetch -o run -- $B
