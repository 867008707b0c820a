#!/bin/bash
# Kernel-trace profile of the default bench (rocprofv3 rocpd database ->
# tools/rocpd_stats.py summary). Usage on the GPU box:
#   bash tools/profile_bench.sh <tag>     (writes gpurun_out/prof_<tag>/...)
set -e
TAG=${1:-bench}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run -- python3 $R/bench.py --cpu-outer 0 --tiled-reference 0 > $OUT/bench.json 2> $OUT/bench.err || true
python3 $R/tools/rocpd_stats.py $OUT/run_results.db --csv $OUT/kernel_stats.csv --top $OUT/kernel_stats_top.txt --title "rocprofv3 --kernel-trace -- python3 bench.py --cpu-outer 0 --tiled-reference 0 (warmup 1 + 2 timed Perform steps + the HBM-resident warm-up and 2 steps)"
