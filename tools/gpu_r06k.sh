#!/bin/bash
# r06: kernel trace of the pool-16 tiled leg alone (verdict r05 item 7)
set -o pipefail
TAG=${1:-r06k}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
RDL_SHUTDOWN_LOG=1 RDL_SEGV_REPORT=$OUT/segv.txt timeout -k 10 400 rocprofv3 --kernel-trace --stats \
  -d $OUT/prof -o run -- python3 $R/tools/bench_legs.py tiled --reps 1 > $OUT/legs_tiled.jsonl 2> $OUT/legs_tiled.err
rc=$?
echo "rocprof tiled exit $rc"
tail -3 $OUT/legs_tiled.err
exit 0
