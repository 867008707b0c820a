#!/bin/bash
# r06: the cost-ordered subimage queue again, with the stream pool
set -o pipefail
TAG=${1:-r06z}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/bench_legs.py tiled,joined_split --reps 2 > $OUT/legs_rr.jsonl 2> $OUT/legs_rr.err || exit $?
RADLER_POOL_QUEUE=1 timeout -k 10 300 python -u tools/bench_legs.py tiled,joined_split --reps 2 > $OUT/legs_q.jsonl 2> $OUT/legs_q.err || exit $?
timeout -k 10 300 python -u tools/bench_legs.py tiled --reps 2 > $OUT/legs_rr2.jsonl 2> $OUT/legs_rr2.err || exit $?
