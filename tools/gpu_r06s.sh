#!/bin/bash
# r06: no null-stream uploads — FFT tests, then leg order
set -o pipefail
TAG=${1:-r06s}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 python -u -m pytest tests/test_fft_fast.py tests/test_conv64_tiled.py tests/test_scale_convs.py -m gpu -q $T > $OUT/tests_fft.log 2>&1
rc=$?; tail -2 $OUT/tests_fft.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/bench_legs.py joined,joined_split --reps 1 > $OUT/legs_order.jsonl 2> $OUT/legs_order.err || exit $?
timeout -k 10 300 python -u tools/bench_legs.py headline,tiled --reps 1 > $OUT/legs_ht.jsonl 2> $OUT/legs_ht.err || exit $?
