source tools/gpu_step.sh
step r03y_c3 600 python -u bench.py --config c3 --steps 10 --no-cpu-baseline --recall-queries 64
step r03y_c3_split 600 python -u bench.py --config c3 --steps 10 --no-cpu-baseline --no-recall --opt split_div=8
step r03y_c3_noi8 600 python -u bench.py --config c3 --steps 10 --no-cpu-baseline --no-recall --opt scan_i8=off
step r03y_tests 900 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_scan_i8.py tests/test_gpu_scan8.py -x -q --timeout 300 --timeout-method thread
