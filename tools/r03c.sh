source tools/gpu_step.sh
step r03c_c1 300 python -u bench.py --config c1 --steps 2000
step r03c_nstar_b128 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall --batch 128
step r03c_nstar_b64 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall --batch 64
step r03c_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03c_prof_c2 -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-recall
P="--kernel-include-regex scan8 --output-format csv"
B="python3 bench.py --config nstar --steps 3 --warmup 1 --no-cpu-baseline --no-recall"
step r03c_pmc_tcc 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum $P -d gpurun_out/r03c_pmc_tcc -o run -- $B
step r03c_pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE $P -d gpurun_out/r03c_pmc_fetch -o run -- $B
step r03c_pmc_sq 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE $P -d gpurun_out/r03c_pmc_sq -o run -- $B
step r03c_pmc_lds 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM $P -d gpurun_out/r03c_pmc_lds -o run -- $B
