#!/bin/bash
# r06: subimage queue modes with the stream pool (0 round-robin, 1 cost-ordered, 2 index-order queue)
set -o pipefail
TAG=${1:-r06z2}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for q in 2 0 1 2 0; do
  RADLER_POOL_QUEUE=$q timeout -k 10 300 python -u tools/bench_legs.py tiled,joined_split --reps 2 >> $OUT/legs_q$q.jsonl 2>> $OUT/legs_q$q.err || exit $?
done
