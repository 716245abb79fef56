source tools/gpu_step.sh
step r03v_graphs 600 python -u -m pytest tests/test_gpu_graphs.py -x -v --timeout 300 --timeout-method thread
step r03v_c2 300 python -u bench.py --steps 20 --no-cpu-baseline
step r03v_c2_nog 300 python -u bench.py --steps 20 --no-cpu-baseline --no-recall --opt graphs=off
step r03v_nstar 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall
step r03v_c2_host 300 python -u bench.py --steps 20 --no-cpu-baseline --no-recall --api host_batch
step r03v_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03v_prof_c2 -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-recall
step r03v_pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
