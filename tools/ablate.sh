#!/bin/bash
# Development-only: builds timing-ablation variants of the scan kernel into abl/
# (results are wrong by design; used with LANCE_HIP_LIB=abl/lib_<NAME>.so bench.py)
set -e
cd "$(dirname "$0")/.."
D=duckdb-lancedb_amd
F="-DLHIP_ABLATION_BUILD -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-inline-asm -Wno-unused-result"
mkdir -p abl
make -s -C $D  # the other objects of the library (lib/*.o)
OTHERS="$D/lib/scan8_kernels.o $D/lib/ivf_kernels.o $D/lib/lance_hip_abi.o $D/lib/ivf_index.o $D/lib/meta.o"
build() { # name defines...
	local n=$1; shift
	hipcc $F "$@" -c $D/csrc/knn_kernels.hip -o abl/k_$n.o
	hipcc -shared -o abl/lib_$n.so abl/k_$n.o $OTHERS
}
for v in "$@"; do
	case $v in
	NO_EPILOGUE) build NO_EPILOGUE -DLHIP_ABL_NO_EPILOGUE=1 ;;
	NO_MFMA) build NO_MFMA -DLHIP_ABL_NO_MFMA=1 ;;
	
	
	
	PROF) build PROF -DLHIP_PROF=1 ;;
	PROF_NOSLOW) build PROF_NOSLOW -DLHIP_PROF=1 -DLHIP_ABL_NO_SLOW=1 ;;
	PROF_NOFLUSH) build PROF_NOFLUSH -DLHIP_PROF=1 -DLHIP_ABL_NO_FLUSH=1 ;;
	NOSLOW) build NOSLOW -DLHIP_ABL_NO_SLOW=1 ;;
	NOREADS) build NOREADS -DLHIP_ABL_NO_READS=1 ;;
	NOMFMA_NOREADS) build NOMFMA_NOREADS -DLHIP_ABL_NO_MFMA=1 -DLHIP_ABL_NO_READS=1 ;;
	NOMFMA_NOREADS_NOEPI) build NOMFMA_NOREADS_NOEPI -DLHIP_ABL_NO_MFMA=1 -DLHIP_ABL_NO_READS=1 -DLHIP_ABL_NO_EPILOGUE=1 ;;
	NOFLUSH) build NOFLUSH -DLHIP_ABL_NO_FLUSH=1 ;;
	SNOFENCE) build SNOFENCE -DLHIP_ABL_SMALL_NOFENCE=1 ;;
	SLOW_NEVER) build SLOW_NEVER -DLHIP_ABL_SLOW_NEVER=1 ;;
	SLOW_UNROLL) build SLOW_UNROLL -DLHIP_SLOW_VALU=0 -DLHIP_SLOW_UNROLL=1 ;;
	SLOW_SWITCH) build SLOW_SWITCH -DLHIP_SLOW_VALU=0 ;;
	NOLISTWRITE) build NOLISTWRITE -DLHIP_ABL_NO_LISTWRITE=1 ;;
	DRAIN) build DRAIN -DLHIP_ABL_DRAIN_EPI=1 ;;
	PRIO) build PRIO -DLHIP_PRIO_HI_HALF=1 ;;
	SK32N3) build SK32N3 -DLHIP_SK_BF16=32 -DLHIP_NST_BF16_32=3 ;;
	SK32N4) build SK32N4 -DLHIP_SK_BF16=32 -DLHIP_NST_BF16_32=4 ;;
	SKEL_SK32N4) build SKEL_SK32N4 -DLHIP_SK_BF16=32 -DLHIP_NST_BF16_32=4 -DLHIP_ABL_NO_MFMA=1 -DLHIP_ABL_NO_READS=1 -DLHIP_ABL_NO_EPILOGUE=1 ;;
	NOSLOW_DRAIN) build NOSLOW_DRAIN -DLHIP_ABL_DRAIN_EPI=1 -DLHIP_ABL_NO_SLOW=1 ;;
	SKEL) build SKEL -DLHIP_ABL_NO_MFMA=1 -DLHIP_ABL_NO_READS=1 -DLHIP_ABL_NO_EPILOGUE=1 ;;
	SKEL_NOQ) build SKEL_NOQ -DLHIP_ABL_NO_MFMA=1 -DLHIP_ABL_NO_READS=1 -DLHIP_ABL_NO_EPILOGUE=1 -DLHIP_ABL_NO_QDMA=1 ;;
	SKEL_NOQ_NT0) build SKEL_NOQ_NT0 -DLHIP_ABL_NO_MFMA=1 -DLHIP_ABL_NO_READS=1 -DLHIP_ABL_NO_EPILOGUE=1 -DLHIP_ABL_NO_QDMA=1 -DLHIP_X_NT=0 ;;
	NOQ) build NOQ -DLHIP_ABL_NO_QDMA=1 -DLHIP_ABL_NO_SLOW=1 ;;
	SKEL_NT0) build SKEL_NT0 -DLHIP_ABL_NO_MFMA=1 -DLHIP_ABL_NO_READS=1 -DLHIP_ABL_NO_EPILOGUE=1 -DLHIP_X_NT=0 ;;
	NT0) build NT0 -DLHIP_X_NT=0 ;;
	NOQ_NT0) build NOQ_NT0 -DLHIP_ABL_NO_QDMA=1 -DLHIP_ABL_NO_SLOW=1 -DLHIP_X_NT=0 ;;
	
	
	
	
	TFOLD0) build TFOLD0 -DLHIP_I8_TFOLD=0 ;;
	PF0) build PF0 -DLHIP_PF=0 ;;
	PF1) build PF1 -DLHIP_PF=1 ;;
	PF2) build PF2 -DLHIP_PF=2 ;;
	PF4) build PF4 -DLHIP_PF=4 ;;
	PF6) build PF6 -DLHIP_PF=6 ;;
	PREV) # the committed (HEAD) kernel file, for same-box A/B timing
		git show HEAD:$D/csrc/knn_kernels.hip > abl/prev_kernels.hip
		hipcc $F -I$D/csrc -c abl/prev_kernels.hip -o abl/k_PREV.o
		hipcc -shared -o abl/lib_PREV.so abl/k_PREV.o $OTHERS ;;
	*) echo "unknown $v"; exit 1 ;;
	esac
done
