source tools/gpu_step.sh
B="python -u bench.py --config nstar --steps 5 --warmup 1 --no-cpu-baseline --no-recall"
step r03s_base1 300 $B
step r03s_a34 300 $B --opt scan8_variant=34
step r03s_a24 300 $B --opt scan8_variant=24
step r03s_base2 300 $B
step r03s_a34b 300 $B --opt scan8_variant=34
