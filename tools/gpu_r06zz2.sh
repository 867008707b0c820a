#!/bin/bash
# r06 final: the tiled leg first and after other legs, three runs each
set -o pipefail
TAG=${1:-r06zz2}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/bench_legs.py tiled --reps 3 > $OUT/legs_first.jsonl 2> $OUT/legs_first.err || exit $?
timeout -k 10 300 python -u tools/bench_legs.py joined,headline,joined_split,tiled --reps 3 > $OUT/legs_after.jsonl 2> $OUT/legs_after.err || exit $?
