#!/bin/bash
# PQ fast scan A/B on one MI355X: IVF parity tests, C5 bench of both forms and their
# per-phase cycles (LHIP_PQ_PROF build); PMC=1: LDS / VALU counter passes for both forms
source tools/gpu_step.sh
T=${1:-r05r}
G="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE"
step ${T}_pytest 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_ivf.py tests/test_gpu_ivf_params.py tests/test_gpu_ivf_shard.py}
step ${T}_c5_bank 300 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
LANCE_HIP_PQ_LANE_ROWS=1 step ${T}_c5_lanes 300 python -u bench.py --config c5 --steps 10 --no-cpu-baseline
LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_pqprof.so step ${T}_prof_bank 300 python -u bench.py --config c5 --steps 3 --no-cpu-baseline --no-recall --no-host-batch
LANCE_HIP_PQ_LANE_ROWS=1 LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_pqprof.so step ${T}_prof_lanes 300 python -u bench.py --config c5 --steps 3 --no-cpu-baseline --no-recall --no-host-batch
grep -h PQPROF gpurun_out/${T}_prof_bank.log gpurun_out/${T}_prof_lanes.log
grep -ho '"avg_launch_ms": [0-9.]*' gpurun_out/${T}_c5_bank.log gpurun_out/${T}_c5_lanes.log
if [ "$PMC" = 1 ]; then
for f in bank lanes; do
	if [ $f = lanes ]; then export LANCE_HIP_PQ_LANE_ROWS=1; fi
	PMC_GROUPS="$G" step ${T}_pmc_$f 400 bash tools/pmc_scan.sh ${T}_$f -- --config c5 --steps 3 --warmup 1 --no-host-batch
	python3 tools/pmc_summary.py ${T}_$f pq_fast_scan gpurun_out/${T}_${f}_pq_pmc.json > /dev/null
	rm -rf gpurun_out/${T}_${f}_pmc[0-9]*/
done
fi
