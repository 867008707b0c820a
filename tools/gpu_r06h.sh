#!/bin/bash
# r06 eighth box run: light peak kernel toggle, c2t / t2k8 end states, the C5
# rounding ensemble, then C5
set -o pipefail
TAG=${1:-r06h}
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
T="--timeout 900 --timeout-method thread -p no:cacheprovider"
RDL_PEAK_FINISH=0 timeout -k 10 300 python -u tools/bench_legs.py joined_split --reps 2 > $OUT/legs_nofinish.jsonl 2> $OUT/legs_nofinish.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py -k "t2k8 or c2_to_threshold" -m gpu -v -s $T \
  > $OUT/tests_t2k8_c2t.log 2>&1
rc=$?; tail -3 $OUT/tests_t2k8_c2t.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 700 python -u tools/end_state_spread.py c5 --ulp 3 --twopass 0 \
  > $OUT/spread_c5.json 2> $OUT/spread_c5.err || exit $?
cp $OUT/spread_c5.json profiles/r06_end_state_spread_c5.json
timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py -k "c5" -m gpu -v -s $T \
  > $OUT/tests_c5.log 2>&1
rc=$?; tail -3 $OUT/tests_c5.log; [ $rc -le 1 ] || exit $rc
