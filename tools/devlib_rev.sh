#!/bin/bash
# Development-only: the library as built from git revision REV (A/B baseline):
#   tools/devlib_rev.sh REV NAME  ->  duckdb-lancedb_amd/lib_dev/lib_NAME.so
set -e
cd "$(dirname "$0")/.."
rev=$1 n=$2
W=/tmp/lhip_wt_$n
rm -rf $W
git worktree add -f --detach $W $rev > /dev/null
make -s -C $W/duckdb-lancedb_amd -j8 > /dev/null
mkdir -p duckdb-lancedb_amd/lib_dev
cp $W/duckdb-lancedb_amd/lib/liblancedb_hip.so duckdb-lancedb_amd/lib_dev/lib_$n.so
git worktree remove --force $W
echo built duckdb-lancedb_amd/lib_dev/lib_$n.so from $(git rev-parse --short $rev)
