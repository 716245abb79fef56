source tools/gpu_step.sh
B="python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall"
step r03h_base 300 $B
step r03h_st64 300 $B --opt scan8_variant=1064
step r03h_st128 300 $B --opt scan8_variant=1128
step r03h_st192 300 $B --opt scan8_variant=1192
step r03h_v1 300 $B --opt scan8_variant=1
step r03h_v2 300 $B --opt scan8_variant=2
step r03h_v5 300 $B --opt scan8_variant=5
