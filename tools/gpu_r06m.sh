#!/bin/bash
# r06: IUWT in-place recurrences + default modes: tests, C4 leg per mode
set -o pipefail
TAG=${1:-r06m}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 python -u -m pytest tests/test_iuwt.py tests/test_iuwt_algorithm.py -m gpu -v $T \
  > $OUT/tests_iuwt.log 2>&1
rc=$?; tail -3 $OUT/tests_iuwt.log; [ $rc -le 1 ] || exit $rc
for cfg in "RDL_IUWT_NONE=1" "RDL_IUWT_FUSED=0" "RDL_IUWT_FUSED=3"; do
  env $cfg timeout -k 10 200 python -u tools/iuwt_run.py >> $OUT/iuwt_modes.jsonl 2>> $OUT/iuwt_modes.err || exit $?
done
