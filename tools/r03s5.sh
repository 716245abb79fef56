# host-side step anatomy: HIP runtime API trace + kernel trace of the C2 bench
source tools/gpu_step.sh
T=${1:-r03v}
step ${T}_hiptrace_c2 300 rocprofv3 --hip-runtime-trace --kernel-trace -d gpurun_out/${T}_hiptrace_c2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-recall
