#!/bin/bash
# r06: stream pool — leg order with and without it
set -o pipefail
TAG=${1:-r06t}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/bench_legs.py joined,joined_split --reps 1 > $OUT/legs_order.jsonl 2> $OUT/legs_order.err || exit $?
timeout -k 10 300 python -u tools/bench_legs.py headline,tiled --reps 1 > $OUT/legs_ht.jsonl 2> $OUT/legs_ht.err || exit $?
RDL_STREAM_POOL=0 timeout -k 10 300 python -u tools/bench_legs.py joined,joined_split --reps 1 > $OUT/legs_order_nopool.jsonl 2> $OUT/legs_order_nopool.err || exit $?
timeout -k 10 300 python -u tools/bench_legs.py joined_split,tiled --reps 1 > $OUT/legs_first.jsonl 2> $OUT/legs_first.err || exit $?
