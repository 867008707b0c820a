#!/bin/bash
# r06: hardware queues with the stream pool (tiled + split joined legs)
set -o pipefail
TAG=${1:-r06u}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/bench_legs.py tiled,joined_split --reps 1 > $OUT/legs_q$q.jsonl 2> $OUT/legs_q$q.err || exit $?
done
