#!/bin/bash
# GPU box helper: run ONE step under its own time limit; stop the whole call on
# a timeout, a signal or a crash (status >= 124), keep going after an ordinary
# failure (a failed assertion) so the later steps still report.
# usage: source tools/gpu_step.sh; step NAME SECONDS cmd args...   (output: gpurun_out/NAME.log)
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
	local name=$1 secs=$2
	shift 2
	echo "== $name: $*"
	timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
	local rc=$?
	tail -3 "gpurun_out/$name.log"
	echo "== $name rc=$rc"
	if [ $rc -ge 124 ]; then
		echo "abnormal exit ($rc): stopping"
		exit $rc
	fi
	return 0
}
