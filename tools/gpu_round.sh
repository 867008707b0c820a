#!/bin/bash
# Round check on the GPU box: the -m gpu parity suite, then the driver's bench
# command.  Usage (on the box, via gpurun):  bash tools/gpu_round.sh [tag]
#   GPU_TESTS="tests/x.py ..."  run a subset of the suite
#   SKIP_TESTS=1                bench only
#   BENCH_ARGS="..."            bench arguments (default: the driver's)
set -o pipefail
TAG=${1:-round}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 840 python -u -m pytest ${GPU_TESTS:-tests} -m gpu -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider -s > $OUT/gpu_tests.log 2>&1 || exit $?
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5} \
  > $OUT/bench.json 2> $OUT/bench.err
