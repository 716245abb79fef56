# sample-pass coverage A/B (option sample_div) on C2, its per-rank shape and north_star
source tools/gpu_step.sh
T=${1:-r03x}
for sd in 16 32 64; do
  step ${T}_c2_sd$sd 300 python -u bench.py --steps 30 --no-cpu-baseline --no-recall --sample-div $sd
  step ${T}_c2s8_sd$sd 300 python -u bench.py --n 125000 --steps 40 --no-cpu-baseline --no-recall --sample-div $sd
  step ${T}_nstar_sd$sd 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall --sample-div $sd
done
