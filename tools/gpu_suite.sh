#!/bin/bash
# The -m gpu suite (optionally a -k selection) and then the driver's default
# bench command.  Usage (on the box, via gpurun): TESTS="expr" bash tools/gpu_suite.sh <tag>
set -o pipefail
TAG=${1:-suite}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 720 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -s ${TESTS:+-k "$TESTS"} > $OUT/gpu_tests.log 2>&1
rc=$?
tail -5 $OUT/gpu_tests.log
[ $rc -le 1 ] || exit $rc
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
  tail -1 $OUT/bench.json | cut -c1-400
fi
