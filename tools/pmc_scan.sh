#!/bin/bash
# GPU box: rocprofv3 counter passes over one bench configuration, one counter
# group per run (MI355X_MICROARCH.md 'rocprofv3 PMC slots': no trace domains
# beside --pmc, at most 8 SQ / 4 TCC counters per pass).
# usage: tools/pmc_scan.sh TAG -- <bench.py args>     (CSVs under gpurun_out/TAG_pmc<i>/)
# PMC_GROUPS='CTR CTR ...;CTR ...' replaces the default groups (';' between passes)
set -o pipefail
T=$1; shift; [ "$1" = "--" ] && shift
export TMPDIR=/tmp
O=gpurun_out
GROUPS_=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
)
if [ -n "$PMC_GROUPS" ]; then IFS=';' read -r -a GROUPS_ <<< "$PMC_GROUPS"; fi
i=0
for g in "${GROUPS_[@]}"; do
  timeout -s KILL 240 rocprofv3 --pmc $g --output-format csv -d $O/${T}_pmc$i -o run -- python3 bench.py "$@" --no-cpu-baseline --no-recall > $O/${T}_pmc$i.log 2>&1 || { echo "pmc group $i ($g) FAILED"; tail -5 $O/${T}_pmc$i.log; exit 1; }
  echo "pmc $i ok: $g"
  i=$((i+1))
done
