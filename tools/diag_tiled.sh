#!/bin/bash
# Tiled-path diagnosis on the GPU box (one rocprofv3 pass, last):
#   bash tools/diag_tiled.sh <tag> <size> <grid> <threads> [hip]
# 1) host-profile run (RADLER_HOST_PROFILE=1): wall time per host section
# 2) rocprofv3 --kernel-trace (+ --hip-trace with "hip"), summarised here;
#    the database is deleted (gpurun_out is capped at 64 MiB)
set -e
TAG=${1:-tiled}; SIZE=${2:-8192}; GRID=${3:-4}; THR=${4:-1}; HIP=${5:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/diag_$TAG
mkdir -p $OUT
cd $R
export BENCH_TILED_RUNS=1
RADLER_HOST_PROFILE=1 RADLER_VERBOSE=3 timeout -k 10 300 python3 -u tools/bench_tiled.py $SIZE $GRID $THR > $OUT/host_profile.out 2> $OUT/verbose.err
grep -c '^\[ms\] it=' $OUT/verbose.err > $OUT/outer_iterations.txt || true
grep -v '^\[ms\] it=' $OUT/verbose.err | tail -50 > $OUT/verbose_tail.err || true
rm -f $OUT/verbose.err
cd /tmp && export TMPDIR=/tmp
EXTRA=""; [ "$HIP" = hip ] && EXTRA="--hip-trace"
timeout -k 10 400 rocprofv3 --kernel-trace $EXTRA -d $OUT/prof -o run -- python3 $R/tools/bench_tiled.py $SIZE $GRID $THR > $OUT/prof.out 2> $OUT/prof.err || true
python3 $R/tools/rocpd_stats.py $OUT/prof/run_results.db --csv $OUT/kernel_stats.csv --top $OUT/kernel_stats_top.txt --title "tiled $SIZE ${GRID}x$GRID threads $THR"
python3 $R/tools/rocpd_api_stats.py $OUT/prof/run_results.db --out $OUT/api_stats.txt || true
rm -rf $OUT/prof
