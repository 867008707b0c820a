#!/bin/bash
# r06 ninth box run: t2k8 / h8kt end states, IUWT after the restrict change
set -o pipefail
TAG=${1:-r06i}
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
T="--timeout 900 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py -k "t2k8 or h8k_to_threshold" -m gpu -v -s $T \
  > $OUT/tests_ends.log 2>&1
rc=$?; tail -3 $OUT/tests_ends.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_iuwt.py tests/test_iuwt_algorithm.py -m gpu -q $T > $OUT/tests_iuwt.log 2>&1
rc=$?; tail -3 $OUT/tests_iuwt.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-outer 0 --tiled-reference 0 \
  --joined-reference 0 --c2-reference 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit $?
