#!/bin/bash
# gpurun with retries ONLY while no GPU box / slot is free (exit 3: nothing ran,
# nothing charged); any other outcome ends it.  usage: tools/gpu_retry.sh OUT TIMEOUT 'cmd'
out=$1; to=$2; shift 2
for i in $(seq 1 ${GPU_RETRIES:-6}); do
	/usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
	rc=$?
	if [ $rc -ne 3 ] && ! grep -q "status=transient" "$out"; then exit $rc; fi
	sleep 150
done
exit $rc
