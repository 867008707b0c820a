#!/bin/bash
# r06 seventh box run: atomic block argmax on the grid participants (parity +
# bins), deferred-result joined/pool tests, joined-split combined toggles,
# C5/t2k8 with the ensembles
set -o pipefail
TAG=${1:-r06g}
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
T="--timeout 900 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_multiscale_gpu.py \
  tests/test_deferred_result.py tests/test_iuwt.py tests/test_iuwt_algorithm.py -m gpu -q -x $T \
  > $OUT/tests_kernels.log 2>&1
rc=$?; tail -3 $OUT/tests_kernels.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py -k "c2_multi or h8k_headline or c3 or p8k" -m gpu -v -s $T \
  > $OUT/tests_configs.log 2>&1
rc=$?; tail -3 $OUT/tests_configs.log; [ $rc -le 1 ] || exit $rc
B="--steps 1 --warmup 1 --cpu-outer 0 --tiled-reference 0 --joined-reference 0 --c2-reference 0 --iuwt-reference 0 --device-resident 0"
RDL_TRACE_SUBMINOR=2 timeout -k 10 300 python -u bench.py $B > $OUT/trace2.json 2> $OUT/trace2.err || exit $?
python tools/subminor_stats.py $OUT/trace2.err --last-iterations 129505 > $OUT/subminor_bins.txt 2>&1
RDL_TRACE_SUBMINOR=1 timeout -k 10 300 python -u bench.py $B > $OUT/trace1.json 2> $OUT/trace1.err || exit $?
python tools/subminor_stats.py $OUT/trace1.err --last-iterations 129505 > $OUT/subminor_phases.txt 2>&1
RDL_ZERO_COPY=0 RDL_PEAK_FINISH=0 RDL_TABLE_ZERO=0 RDL_SEL_COUNT_COPY=1 timeout -k 10 300 \
  python -u tools/bench_legs.py joined_split --reps 2 > $OUT/legs_alltog.jsonl 2> $OUT/legs_alltog.err || exit $?
timeout -k 10 300 python -u tools/bench_legs.py joined_split --reps 2 > $OUT/legs_default.jsonl 2> $OUT/legs_default.err || exit $?
RDL_PEAK_FINISH=0 timeout -k 10 300 python -u tools/bench_legs.py joined_split --reps 2 > $OUT/legs_nofinish.jsonl 2> $OUT/legs_nofinish.err || exit $?
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-outer 0 --tiled-reference 0 \
  --joined-reference 0 --c2-reference 0 --device-resident 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit $?
