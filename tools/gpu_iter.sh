#!/bin/bash
# One iteration of the kernel work on the GPU box: parity subset, micro-
# benchmarks, sub-minor trace of the bench.  Usage: bash tools/gpu_iter.sh <tag>
#   TESTS="expr"      pytest -k selection (default: the kernel parity tests)
set -o pipefail
TAG=${1:-iter}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${TEST_FILES:-tests/test_gpu_kernels.py tests/test_configs_gpu.py} -m gpu -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider -s ${TESTS:+-k "$TESTS"} > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit $rc
if [ -n "$SUBMINOR_BENCH" ]; then
  RDL_BENCH_TAB=1 timeout -k 10 300 python -u tools/bench_subminor.py > $OUT/bench_subminor.txt 2>&1 || exit $?
fi
if [ -n "$FFT_BENCH" ]; then
  timeout -k 10 300 python -u tools/bench_fftk.py 10 $FFT_BENCH > $OUT/bench_fftk.txt 2>&1 || exit $?
fi
if [ -n "$TRACE" ]; then
  bash tools/gpu_subminor_trace.sh $TAG || exit $?
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py $BENCH > $OUT/bench.json 2> $OUT/bench.err || exit $?
fi
