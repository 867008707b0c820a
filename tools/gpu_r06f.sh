#!/bin/bash
# r06 sixth box run: sub-minor atomic block argmax (parity + A/B), fused IUWT
# decomposition, joined-split state diagnostics with device time
set -o pipefail
TAG=${1:-r06f}
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
T="--timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_multiscale_gpu.py tests/test_iuwt.py \
  tests/test_deferred_result.py tests/test_stale_state.py -m gpu -q -x $T > $OUT/tests_kernels.log 2>&1
rc=$?; tail -3 $OUT/tests_kernels.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py -k "c2 or h8k_headline or c3 or c4" -m gpu -v -s $T \
  > $OUT/tests_configs.log 2>&1
rc=$?; tail -3 $OUT/tests_configs.log; [ $rc -le 1 ] || exit $rc
B="--steps 1 --warmup 1 --cpu-outer 0 --tiled-reference 0 --joined-reference 0 --c2-reference 0 --iuwt-reference 0 --device-resident 0"
for at in 1 0; do
  RDL_SUBMINOR_ATOMIC=$at RDL_TRACE_SUBMINOR=2 timeout -k 10 300 python -u bench.py $B \
    > $OUT/trace2_at$at.json 2> $OUT/trace2_at$at.err || exit $?
  python tools/subminor_stats.py $OUT/trace2_at$at.err --last-iterations 129505 > $OUT/subminor_at$at.txt 2>&1
done
RDL_TRACE_SUBMINOR=1 timeout -k 10 300 python -u bench.py $B > $OUT/trace1.json 2> $OUT/trace1.err || exit $?
for at in 1 0 1 0; do
  RDL_SUBMINOR_ATOMIC=$at timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-outer 0 \
    --tiled-reference 0 --joined-reference 0 --c2-reference 0 --iuwt-reference 0 \
    >> $OUT/bench_ab_at$at.json 2>> $OUT/bench_ab.err || exit $?
done
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-outer 0 --tiled-reference 0 \
  --joined-reference 0 --c2-reference 0 --device-resident 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit $?
timeout -k 10 400 python -u tools/bench_legs.py joined,joined_split --reps 1 --events 1 \
  > $OUT/legs_ev_slow.jsonl 2> $OUT/legs_ev_slow.err || exit $?
timeout -k 10 400 python -u tools/bench_legs.py joined_split,joined_split --reps 1 --events 1 \
  > $OUT/legs_ev_fast.jsonl 2> $OUT/legs_ev_fast.err || exit $?
(cd _bisect/365876d && timeout -k 10 300 python -u tools/bench_legs.py joined_split --reps 1 --events 1 \
    > $OUT/legs_ev_old.jsonl 2> $OUT/legs_ev_old.err) || exit $?
