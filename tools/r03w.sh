source tools/gpu_step.sh
step r03w_small 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "small or c1 or exact"
step r03w_c1 300 python -u bench.py --config c1 --steps 2000
step r03w_prof_c1 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03w_prof_c1 -o run -- python3 bench.py --config c1 --steps 500 --no-cpu-baseline
step r03w_pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
