#!/bin/bash
# Development-only (GPU box): bench each named variant (base = the in-tree library)
# and print the scan kernel's average launch time and the step time.
# usage: tools/abl_run.sh [--config c3] -- base NAME1 NAME2 ...
extra=()
while [ "$1" != "--" ] && [ $# -gt 0 ]; do extra+=("$1"); shift; done
shift
for v in "$@"; do
	L=abl/lib_$v.so
	[ "$v" = base ] && L=duckdb-lancedb_amd/lib/liblancedb_hip.so
	LANCE_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-recall "${extra[@]}" \
		> gpurun_out/abl_$v.json 2> gpurun_out/abl_$v.err || { echo "$v FAILED"; exit 1; }
	echo "$v $(python -c "import json;d=json.load(open('gpurun_out/abl_$v.json'));print(d['roofline']['avg_launch_ms'], d['ms_per_step'], d['search_stats']['fallback_queries'])")"
done
