source tools/gpu_step.sh
step r03j_probe 200 ./tools/_stream_probe 10000000
step r03j_tests 600 python -u -m pytest tests/test_gpu_scan8.py tests/test_gpu_scan_i8.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread
step r03j_c2 300 python -u bench.py --steps 20 --no-cpu-baseline
step r03j_nstar 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall
B="python -u bench.py --config nstar --steps 5 --warmup 1 --no-cpu-baseline --no-recall"
step r03j_a21 300 $B --opt scan8_variant=21
step r03j_a22 300 $B --opt scan8_variant=22
step r03j_a23 300 $B --opt scan8_variant=23
step r03j_c2_host 300 python -u bench.py --steps 20 --no-cpu-baseline --api host_batch
step r03j_c2_percall 300 python -u bench.py --steps 300 --no-cpu-baseline --api per_call
step r03j_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03j_prof_c2 -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-recall
step r03j_prof_c1 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03j_prof_c1 -o run -- python3 bench.py --config c1 --steps 500 --no-cpu-baseline
