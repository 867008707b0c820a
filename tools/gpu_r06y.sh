#!/bin/bash
# r06: kernel trace of the pool-16 tiled leg after a one-worker pass (every
# kernel first dispatched from one thread)
set -o pipefail
TAG=${1:-r06y}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
RDL_SEGV_REPORT=$OUT/segv.txt timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv \
  -d $OUT/prof -o run -- python3 $R/tools/bench_legs.py tiled --reps 1 > $OUT/legs.jsonl 2> $OUT/legs.err
echo "rocprof exit $?"
exit 0
