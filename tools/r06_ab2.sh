#!/bin/bash
# round 6: interleaved A/Bs of the final refine's first chunk (pr_first) and the sample size at C2 and
# the per-rank north_star shape (tools/ab_opts.py, one store per shape)
source tools/gpu_step.sh
T=$1
step ${T}_ab_c2 300 python -u tools/ab_opts.py --n 1000000 --reps 3 --steps 60 pr_first=0,sample_div=0 pr_first=128,sample_div=0 pr_first=112,sample_div=0 pr_first=64,sample_div=0 pr_first=0,sample_div=12 pr_first=0,sample_div=24
step ${T}_ab_rank 300 python -u tools/ab_opts.py --n 1250000 --reps 3 --steps 60 pr_first=0,sample_div=0 pr_first=128,sample_div=0 pr_first=0,sample_div=12 pr_first=0,sample_div=24
grep -h setting gpurun_out/${T}_ab_*.log
