source tools/gpu_step.sh
step r03a_i8tests 600 python -u -m pytest tests/test_gpu_scan_i8.py -x -q --timeout 200 --timeout-method thread
step r03a_c2 300 python -u bench.py --steps 20 --no-cpu-baseline
step r03a_nstar 400 python -u bench.py --config nstar --steps 10 --no-cpu-baseline
step r03a_prof_nstar 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03a_prof_nstar -o run -- python3 bench.py --config nstar --steps 5 --no-cpu-baseline --no-recall
