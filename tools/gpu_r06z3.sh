#!/bin/bash
# r06: the default subimage assignment per image-set size — parity and legs
set -o pipefail
TAG=${1:-r06z3}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 python -u -m pytest tests/test_tiling.py tests/test_deferred_result.py -m gpu -v $T > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/bench_legs.py tiled,joined_split --reps 2 > $OUT/legs.jsonl 2> $OUT/legs.err || exit $?
