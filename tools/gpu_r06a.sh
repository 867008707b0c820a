#!/bin/bash
# r06 first box run: teardown tests, leg-order diagnostics, a profiled headline
set -o pipefail
TAG=${1:-r06a}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_teardown.py tests/test_deferred_result.py -m gpu -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider -s > $OUT/tests.log 2>&1
rc=$?
tail -5 $OUT/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/bench_legs.py joined_split,joined_split,tiled,joined_split --reps 1 \
  > $OUT/legs_a.jsonl 2> $OUT/legs_a.err || exit $?
timeout -k 10 300 python -u tools/bench_legs.py tiled,joined_split,joined_split --reps 1 \
  > $OUT/legs_b.jsonl 2> $OUT/legs_b.err || exit $?
cd /tmp && export TMPDIR=/tmp
RDL_SEGV_REPORT=$GRAFT_REPO_ROOT/$OUT/segv.txt RDL_SHUTDOWN_LOG=1 timeout -k 10 300 \
  rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --cpu-outer 0 --joined-reference 0 \
  --c2-reference 0 --tiled-reference 0 > $GRAFT_REPO_ROOT/$OUT/prof_bench.json 2> $GRAFT_REPO_ROOT/$OUT/prof_bench.err
echo "rocprof exit $?"
