#!/bin/bash
# Development-only: timing-ablation variants of pq_fast_scan_kernel (ivf_kernels.hip)
# into abl/lib_pq_<NAME>.so (results are wrong by design; used as
# LANCE_HIP_LIB=abl/lib_pq_<NAME>.so python bench.py --config c5 ...)
set -e
cd "$(dirname "$0")/.."
D=duckdb-lancedb_amd
F="-DLHIP_ABLATION_BUILD -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-inline-asm -Wno-unused-result"
mkdir -p abl
make -s -C $D
OTHERS="$D/lib/knn_kernels.o $D/lib/rscan_kernels.o $D/lib/lance_hip_abi.o $D/lib/ivf_index.o $D/lib/meta.o"
for v in "$@"; do
	defs=""
	for f in ${v//+/ }; do defs="$defs -DLHIP_PQ_ABL_$f=1"; done
	hipcc $F $defs -c $D/csrc/ivf_kernels.hip -o abl/pq_$v.o
	hipcc -shared -o abl/lib_pq_$v.so abl/pq_$v.o $OTHERS
done
