#!/bin/bash
# A test subset, then the default bench and a short headline-only bench with
# an environment toggle (A/B).  Usage (on the box, via gpurun):
#   TEST_FILES="tests/a.py ..." TESTS="expr" AB_ENV="VAR=0" bash tools/gpu_ab.sh <tag>
set -o pipefail
TAG=${1:-ab}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TEST_FILES" ]; then
  timeout -k 10 720 python -u -m pytest $TEST_FILES -m gpu -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider -s ${TESTS:+-k "$TESTS"} > $OUT/tests.log 2>&1
  rc=$?
  tail -5 $OUT/tests.log
  [ $rc -le 1 ] || exit $rc
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 900 python -u bench.py ${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5} \
    > $OUT/bench.json 2> $OUT/bench.err || exit $?
  tail -1 $OUT/bench.json | cut -c1-300
fi
if [ -n "$AB_ENV" ]; then
  env $AB_ENV timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --tiled-reference 0 \
    --joined-reference 0 --c2-reference 0 --cpu-outer 0 > $OUT/bench_ab.json 2> $OUT/bench_ab.err || exit $?
  tail -1 $OUT/bench_ab.json | cut -c1-300
fi
