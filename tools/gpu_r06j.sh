#!/bin/bash
# r06: IUWT row chains — bit-exact tests, then the C4 leg (chains vs rows)
set -o pipefail
TAG=${1:-r06j}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 python -u -m pytest tests/test_iuwt.py tests/test_iuwt_algorithm.py -m gpu -v $T \
  > $OUT/tests_iuwt.log 2>&1
rc=$?; tail -3 $OUT/tests_iuwt.log; [ $rc -le 1 ] || exit $rc
B="--steps 1 --warmup 1 --cpu-outer 0 --tiled-reference 0 --joined-reference 0 --c2-reference 0"
timeout -k 10 300 python -u bench.py $B > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit $?
RDL_IUWT_FUSED=1 timeout -k 10 300 python -u bench.py $B > $OUT/bench_c4_rows.json 2> $OUT/bench_c4_rows.err || exit $?
