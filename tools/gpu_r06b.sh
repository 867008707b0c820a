#!/bin/bash
# r06 second box run: teardown + profiler exit controls, leg order incl. the
# pre-regression build, end-state spread of c2t, float32 correction A/B
set -o pipefail
TAG=${1:-r06b}
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 python -u -m pytest tests/test_teardown.py -m gpu -v $T > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
# the float32 correction (RDL_CORR_F32=1): the reference's own 2e-6 tests, the
# multiscale kernel tests, and the C2 trace / c2t end state
RDL_CORR_F32=1 timeout -k 10 600 python -u -m pytest tests/test_radler_gpu.py tests/test_multiscale_gpu.py \
  tests/test_configs_gpu.py -k "not c3 and not c5 and not p8k and not h8k and not c4 and not c1" -m gpu -v $T \
  > $OUT/tests_f32.log 2>&1
rc=$?; tail -3 $OUT/tests_f32.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/end_state_spread.py c2t > $OUT/spread_c2t.json 2> $OUT/spread_c2t.err || exit $?
RDL_CORR_F32=1 timeout -k 10 300 python -u tools/end_state_spread.py c2t --ulp 0 --twopass 0 > $OUT/spread_c2t_f32.json 2> $OUT/spread_c2t_f32.err || exit $?
# headline A/B: float64 vs float32 correction (default families via --breakdown)
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --tiled-reference 0 --joined-reference 0 \
  --c2-reference 0 --cpu-outer 0 --breakdown > $OUT/bench_f64.json 2> $OUT/bench_f64.err || exit $?
RDL_CORR_F32=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --tiled-reference 0 --joined-reference 0 \
  --c2-reference 0 --cpu-outer 0 --breakdown > $OUT/bench_f32.json 2> $OUT/bench_f32.err || exit $?
# leg order as the bench runs it, then the pre-regression build
timeout -k 10 300 python -u tools/bench_legs.py joined,joined_split --reps 1 \
  > $OUT/legs_c.jsonl 2> $OUT/legs_c.err || exit $?
if [ -f _bisect/365876d/ska-sdp-func-radler_amd/lib/librdl_hip.so ]; then
  cp tools/bench_legs.py _bisect/365876d/tools/
  (cd _bisect/365876d && timeout -k 10 300 python -u tools/bench_legs.py joined_split,joined_split --reps 1 \
    > $OUT/legs_old.jsonl 2> $OUT/legs_old.err) || exit $?
fi
# profiler exit: control (torch only), then the bench with the atexit shutdown
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/prof_torch -o run -- \
  python3 -c "import torch; x = torch.ones(1 << 20, device='cuda'); print(float(x.sum()))" \
  > $OUT/prof_torch.out 2>&1
echo "rocprof torch-only exit $?"
RDL_SEGV_REPORT=$OUT/segv.txt RDL_SHUTDOWN_LOG=1 timeout -k 10 300 \
  rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 --cpu-outer 0 --joined-reference 0 \
  --c2-reference 0 --tiled-reference 0 > $OUT/prof_bench.json 2> $OUT/prof_bench.err
echo "rocprof bench exit $?"
