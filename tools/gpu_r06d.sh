#!/bin/bash
# r06 fourth box run: IUWT fused rows, c2t end state (ensemble tolerances),
# joined-split regression toggles and leg order, profiler exit controls
set -o pipefail
TAG=${1:-r06d}
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
T="--timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 python -u -m pytest tests/test_iuwt.py tests/test_teardown.py tests/test_iuwt_algorithm.py \
  -m gpu -v $T > $OUT/tests_iuwt.log 2>&1
rc=$?; tail -3 $OUT/tests_iuwt.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py -k "c2_to_threshold or c4" -m gpu -v -s $T \
  > $OUT/tests_c2t.log 2>&1
rc=$?; tail -3 $OUT/tests_c2t.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --cpu-outer 0 --tiled-reference 0 \
  --joined-reference 0 --c2-reference 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit $?
RDL_IUWT_FUSED=0 timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --cpu-outer 0 --tiled-reference 0 \
  --joined-reference 0 --c2-reference 0 > $OUT/bench_c4_old.json 2> $OUT/bench_c4_old.err || exit $?
for v in "RDL_TABLE_ZERO=0" "RDL_SEL_COUNT_COPY=1" "RDL_TABLE_ZERO=0 RDL_SEL_COUNT_COPY=1" "RDL_NONE=1"; do
  env $v timeout -k 10 300 python -u tools/bench_legs.py joined_split --reps 2 \
    > "$OUT/legs_tog_${v// /_}.jsonl" 2>/dev/null || exit $?
done
RDL_ALLOC_CACHE=0 timeout -k 10 300 python -u tools/bench_legs.py joined,joined_split --reps 1 \
  > $OUT/legs_nocache.jsonl 2> $OUT/legs_nocache.err || exit $?
timeout -k 10 400 python -u tools/bench_legs.py joined_split,joined,joined_split --reps 1 \
  > $OUT/legs_order.jsonl 2> $OUT/legs_order.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/prof_ctl_a -o run -- \
  python3 -c "import sys; sys.path.insert(0, '$R/tests'); import numpy as np; from rdl_lib import Session; s = Session(0); a = s.array(np.ones(1 << 20, np.float32)); print(s.find_peak(a, 1024, 1024))" \
  > $OUT/prof_ctl_a.out 2>&1
echo "rocprof control A (rdl_lib peak) exit $?"
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/prof_ctl_b -o run -- \
  python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $OUT/prof_ctl_b.out 2>&1
echo "rocprof control B (smoke) exit $?"
cd $R && timeout -k 10 300 python -u tools/end_state_spread.py t2k8 --ulp 4 --twopass 0 > $OUT/spread_t2k8.json 2> $OUT/spread_t2k8.err || exit $?
