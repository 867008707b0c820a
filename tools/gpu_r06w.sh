#!/bin/bash
# r06: row-kernel peak finish — kernel tests, C2/h8k traces, headline A/B
set -o pipefail
TAG=${1:-r06w}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 python -u -m pytest tests/test_fft_fast.py tests/test_rows_dma.py tests/test_gpu_kernels.py tests/test_multiscale_gpu.py -m gpu -q $T > $OUT/tests_k.log 2>&1
rc=$?; tail -2 $OUT/tests_k.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py -k "c2 or h8k" -m gpu -q -s $T > $OUT/tests_cfg.log 2>&1
rc=$?; tail -2 $OUT/tests_cfg.log; [ $rc -le 1 ] || exit $rc
B="--steps 10 --warmup 3 --cpu-outer 0 --tiled-reference 0 --joined-reference 0 --c2-reference 0 --iuwt-reference 0"
timeout -k 10 300 python -u bench.py $B > $OUT/bench_on.json 2> $OUT/bench_on.err || exit $?
RDL_ROWS_PEAK_FINISH=0 timeout -k 10 300 python -u bench.py $B > $OUT/bench_off.json 2> $OUT/bench_off.err || exit $?
timeout -k 10 300 python -u bench.py $B > $OUT/bench_on2.json 2> $OUT/bench_on2.err || exit $?
