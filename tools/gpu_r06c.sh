#!/bin/bash
# r06 third box run: end-state spread at 8192^2, leg order incl. the
# pre-regression build, profiler exit controls
set -o pipefail
TAG=${1:-r06c}
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u tools/end_state_spread.py h8kt > $OUT/spread_h8kt.json 2> $OUT/spread_h8kt.err || exit $?
timeout -k 10 300 python -u tools/bench_legs.py joined,joined_split --reps 1 \
  > $OUT/legs_c.jsonl 2> $OUT/legs_c.err || exit $?
cp tools/bench_legs.py _bisect/365876d/tools/
(cd _bisect/365876d && timeout -k 10 300 python -u tools/bench_legs.py joined_split,joined_split --reps 1 \
  > $OUT/legs_old.jsonl 2> $OUT/legs_old.err) || exit $?
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
cd $R && timeout -k 10 600 python -u -m pytest tests/test_distributed.py -k "channel_sharded" -m gpu -v \
  --timeout 500 --timeout-method thread -p no:cacheprovider -s > $OUT/tests_shard.log 2>&1
rc=$?; tail -3 $OUT/tests_shard.log; [ $rc -le 1 ] || exit $rc
