source tools/gpu_step.sh
step r03d_scan8 600 python -u -m pytest tests/test_gpu_scan8.py -x -v --timeout 300 --timeout-method thread
step r03d_c2 300 python -u bench.py --steps 20 --no-cpu-baseline
step r03d_nstar 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall
step r03d_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03d_prof_c2 -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-recall
step r03d_c1 300 python -u bench.py --config c1 --steps 2000
P="--kernel-include-regex scan8 --output-format csv"
B="python3 bench.py --config nstar --steps 3 --warmup 1 --no-cpu-baseline --no-recall"
step r03d_pmc_sq 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE $P -d gpurun_out/r03d_pmc_sq -o run -- $B
step r03d_pmc_lds 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS $P -d gpurun_out/r03d_pmc_lds -o run -- $B
