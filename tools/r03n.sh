source tools/gpu_step.sh
B="python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall"
step r03n_base 300 $B
step r03n_v28 300 $B --opt scan8_variant=28
step r03n_v29 300 $B --opt scan8_variant=29
step r03n_c2_v28 300 python -u bench.py --steps 20 --no-cpu-baseline --opt scan8_variant=28
