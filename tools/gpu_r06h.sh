#!/bin/bash
# r06 eighth box run: the C5 rounding ensemble, then C5 / t2k8 / c2t
set -o pipefail
TAG=${1:-r06h}
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
T="--timeout 900 --timeout-method thread -p no:cacheprovider"
if [ ! -f profiles/r06_end_state_spread_c5.json ]; then
  timeout -k 10 900 python -u tools/end_state_spread.py c5 --ulp 3 --twopass 0 \
    > $OUT/spread_c5.json 2> $OUT/spread_c5.err || exit $?
  cp $OUT/spread_c5.json profiles/r06_end_state_spread_c5.json
fi
timeout -k 10 1200 python -u -m pytest tests/test_configs_gpu.py -k "c5 or t2k8 or c2_to_threshold" -m gpu -v -s $T \
  > $OUT/tests_tiled.log 2>&1
rc=$?; tail -3 $OUT/tests_tiled.log; [ $rc -le 1 ] || exit $rc
