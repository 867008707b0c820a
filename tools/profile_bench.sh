#!/bin/bash
# Kernel-trace profile of the default bench (rocprofv3 --kernel-trace --stats;
# the rocpd database -> tools/rocpd_stats.py summary). Usage on the GPU box:
#   bash tools/profile_bench.sh <tag> [bench args]   (gpurun_out/prof_<tag>/...)
# RDL_SEGV_REPORT makes librdl_hip append the pc, module, backtrace and module
# map of a crash of the profiled process to segv.txt (the profiler's exit).
set -e
TAG=${1:-bench}
shift || true
ARGS=${*:---cpu-outer 0 --tiled-reference 0 --joined-reference 0 --c2-reference 0}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rc=0
RDL_SEGV_REPORT=$OUT/segv.txt timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT -o run \
  -- python3 $R/bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || rc=$?
echo "rocprofv3 exit status $rc" >> $OUT/bench.err
python3 $R/tools/rocpd_stats.py $OUT/run_results.db --csv $OUT/kernel_stats.csv --top $OUT/kernel_stats_top.txt --title "rocprofv3 --kernel-trace --stats -- python3 bench.py $ARGS"
find $OUT -name "*kernel_stats.csv" | head -5
[ $rc -eq 0 ] || [ $rc -eq 139 ] || [ $rc -eq 134 ] || exit $rc
