source tools/gpu_step.sh
B="python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall"
step r03p_base 300 $B
step r03p_v30 300 $B --opt scan8_variant=30
step r03p_v31 300 $B --opt scan8_variant=31
step r03p_v32 300 $B --opt scan8_variant=32
step r03p_v33 300 $B --opt scan8_variant=33
step r03p_c2_v30 300 python -u bench.py --steps 20 --no-cpu-baseline --opt scan8_variant=30
