#!/bin/bash
# Headline-only benches under several environment settings (A/B/C...):
#   ENVS="A=1;B=2 C=3" bash tools/gpu_env_multi.sh <tag>   (';' separates runs;
#   the first run is always the unset baseline)
set -o pipefail
TAG=${1:-envmulti}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
LITE="--steps 10 --warmup 3 --tiled-reference 0 --joined-reference 0 --c2-reference 0 --cpu-outer 0"
timeout -k 10 400 python -u bench.py $LITE > $OUT/bench_0.json 2> $OUT/bench_0.err || exit $?
tail -1 $OUT/bench_0.json | cut -c1-160
i=1
IFS=';' read -ra RUNS <<< "$ENVS"
for e in "${RUNS[@]}"; do
  env $e timeout -k 10 400 python -u bench.py $LITE > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit $?
  echo "$e: $(tail -1 $OUT/bench_$i.json | cut -c1-160)"
  i=$((i+1))
done
