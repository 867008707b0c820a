#!/bin/bash
# Round-end measurement on the GPU box, ONE pass per gpurun call (this
# image's rocprofv3 segfaults at exit after writing its database, and no GPU
# step may follow a segfault in the same call):
#   bash tools/final_profile.sh <tag> trace   kernel-trace summary (profile_bench.sh)
#   bash tools/final_profile.sh <tag> fetch   --pmc FETCH_SIZE pass
#   bash tools/final_profile.sh <tag> write   --pmc WRITE_SIZE pass
#   bash tools/final_profile.sh <tag> bench   default bench line with its CPU baseline
# then, on the CPU:
#   python tools/pmc_traffic.py gpurun_out/final_<tag>/fetch/run_results.db \
#       gpurun_out/final_<tag>/write/run_results.db \
#       gpurun_out/final_<tag>/fetch/fams.json --out profiles/r01_traffic.json
set -e
TAG=${1:-final}
PASS=${2:-trace}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/final_$TAG
mkdir -p $OUT
case $PASS in
  trace)
    bash $R/tools/profile_bench.sh $TAG ;;
  fetch|write)
    COUNTER=$([ $PASS = fetch ] && echo FETCH_SIZE || echo WRITE_SIZE)
    mkdir -p $OUT/$PASS
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 400 rocprofv3 --pmc $COUNTER --kernel-trace -d $OUT/$PASS -o run -- \
      python3 $R/bench.py --warmup 0 --steps 1 --cpu-outer 0 --tiled-reference 0 --c2-reference 0 --joined-reference 0 --iuwt-reference 0 --device-resident 0 --timing-all \
      --dump-families $OUT/$PASS/fams.json > $OUT/$PASS/bench.json 2> $OUT/$PASS/bench.err ;;
  bench)
    cd $R
    timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err ;;
  *)
    echo "unknown pass $PASS" >&2; exit 2 ;;
esac
