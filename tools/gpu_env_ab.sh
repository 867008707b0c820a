#!/bin/bash
# A/B of an environment setting on the GPU box: the parity subset with the
# setting, then a short headline-only bench without and with it.
#   ENV_B="VAR=value" TEST_FILES="..." TESTS="expr" bash tools/gpu_env_ab.sh <tag>
set -o pipefail
TAG=${1:-envab}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TEST_FILES" ]; then
  env $ENV_B timeout -k 10 720 python -u -m pytest $TEST_FILES -m gpu -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider -s ${TESTS:+-k "$TESTS"} > $OUT/tests_b.log 2>&1
  rc=$?
  tail -3 $OUT/tests_b.log
  [ $rc -le 1 ] || exit $rc
fi
LITE="--steps 10 --warmup 3 --tiled-reference 0 --joined-reference 0 --c2-reference 0 --cpu-outer 0"
timeout -k 10 400 python -u bench.py $LITE > $OUT/bench_a.json 2> $OUT/bench_a.err || exit $?
env $ENV_B timeout -k 10 400 python -u bench.py $LITE > $OUT/bench_b.json 2> $OUT/bench_b.err || exit $?
tail -1 $OUT/bench_a.json | cut -c1-200
tail -1 $OUT/bench_b.json | cut -c1-200
