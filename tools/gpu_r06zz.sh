#!/bin/bash
# r06 final: leg-order independence with the final defaults (one job)
set -o pipefail
TAG=${1:-r06zz}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/bench_legs.py joined_split,tiled --reps 1 > $OUT/legs_first.jsonl 2> $OUT/legs_first.err || exit $?
timeout -k 10 300 python -u tools/bench_legs.py joined,headline,joined_split,tiled --reps 1 > $OUT/legs_after.jsonl 2> $OUT/legs_after.err || exit $?
