source tools/gpu_step.sh
B="python -u bench.py --config nstar --steps 5 --warmup 1 --no-cpu-baseline --no-recall"
step r03i_base 300 $B
step r03i_a21 300 $B --opt scan8_variant=21
step r03i_a22 300 $B --opt scan8_variant=22
step r03i_a23 300 $B --opt scan8_variant=23
step r03i_prof_c1 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03i_prof_c1 -o run -- python3 bench.py --config c1 --steps 500 --no-cpu-baseline
