#!/bin/bash
# Development-only library variants (diagnostic / A-B builds), never the product:
#   tools/devlib.sh NAME SOURCE DEFINES...   ->  duckdb-lancedb_amd/lib_dev/lib_NAME.so
# SOURCE (knn | scan8 | ivf: the <name>_kernels.hip file) is rebuilt with DEFINES; the other objects are the
# release ones (make first).  Run with LANCE_HIP_LIB=duckdb-lancedb_amd/lib_dev/lib_NAME.so.
set -e
cd "$(dirname "$0")/.."
D=duckdb-lancedb_amd
n=$1 src=$2
shift 2
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-inline-asm -Wno-unused-result"
make -s -C $D
mkdir -p $D/lib_dev
objs=""
for o in knn_kernels scan8_kernels ivf_kernels coarse_kernels lance_hip_abi ivf_index meta shards; do
	if [ "$o" = "${src}_kernels" ]; then
		/opt/rocm/bin/hipcc $F "$@" -c $D/csrc/$o.hip -o $D/lib_dev/${o}_$n.o
		objs="$objs $D/lib_dev/${o}_$n.o"
	else
		objs="$objs $D/lib/$o.o"
	fi
done
/opt/rocm/bin/hipcc -shared -Wl,--no-undefined -o $D/lib_dev/lib_$n.so $objs
echo built $D/lib_dev/lib_$n.so
