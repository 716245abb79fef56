source tools/gpu_step.sh
step r03e_scan8 600 python -u -m pytest tests/test_gpu_scan8.py -x -q --timeout 300 --timeout-method thread -k "every_ld or c2_full or query_batches"
step r03e_nstar 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall
for v in 1 2 4 5; do
step r03e_nstar_v$v 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall --opt scan8_variant=$v
done
step r03e_c2 300 python -u bench.py --steps 20 --no-cpu-baseline
step r03e_nstar_b128 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall --batch 128
