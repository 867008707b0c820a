#!/bin/bash
# r06: the split joined leg and the tiled leg after the session memset fix
set -o pipefail
TAG=${1:-r06r}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/bench_legs.py joined_split --reps 2 > $OUT/legs_js.jsonl 2> $OUT/legs_js.err || exit $?
timeout -k 10 300 python -u tools/bench_legs.py tiled --reps 2 > $OUT/legs_tiled.jsonl 2> $OUT/legs_tiled.err || exit $?
timeout -k 10 300 python -u tools/bench_legs.py joined,joined_split --reps 1 > $OUT/legs_order.jsonl 2> $OUT/legs_order.err || exit $?
