#!/bin/bash
# Round-end measurement on the GPU box: kernel-trace profile, the two HBM
# PMC passes, and the default bench line with its CPU baseline.
#   bash tools/final_profile.sh <tag>   (writes gpurun_out/final_<tag>/...)
set -e
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/final_$TAG
mkdir -p $OUT/fetch $OUT/write
bash $R/tools/profile_bench.sh $TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run -- \
  python3 $R/bench.py --warmup 0 --steps 1 --cpu-sample 0 --timing-all \
  --dump-families $OUT/fetch/fams.json > $OUT/fetch/bench.json 2> $OUT/fetch/bench.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run -- \
  python3 $R/bench.py --warmup 0 --steps 1 --cpu-sample 0 --timing-all \
  --dump-families $OUT/write/fams.json > $OUT/write/bench.json 2> $OUT/write/bench.err
python3 $R/tools/pmc_traffic.py $OUT/fetch/run_results.db $OUT/write/run_results.db \
  $OUT/fetch/fams.json --out $OUT/traffic.json > $OUT/traffic.log 2>&1
cd $R
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
