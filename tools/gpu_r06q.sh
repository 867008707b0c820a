#!/bin/bash
# r06: split joined regression — session creation's memset / mapped buffer (devC toggles)
set -o pipefail
TAG=${1:-r06q}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
cp tools/bench_legs.py _bisect/devC/tools/
cd _bisect/devC
for cfg in "RDL_BIS_MEMSET=0" "RDL_BIS_MAPPED=0" "RDL_BIS_MEMSET=0 RDL_BIS_MAPPED=0" "RDL_BIS_NONE=1"; do
  n=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 300 python -u tools/bench_legs.py joined_split --reps 2 > $OUT/legs_$n.jsonl 2> $OUT/legs_$n.err || exit $?
done
