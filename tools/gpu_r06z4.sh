#!/bin/bash
# r06: subimage assignment mode 3 (cost order dealt round robin) against 0 and 1
set -o pipefail
TAG=${1:-r06z4}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for q in 3 0 1 3 0 1; do
  RADLER_POOL_QUEUE=$q timeout -k 10 300 python -u tools/bench_legs.py tiled,joined_split --reps 2 >> $OUT/legs_q$q.jsonl 2>> $OUT/legs_q$q.err || exit $?
done
