#!/bin/bash
# Joined-channel sub-minor grid size sweep (RDL_SUBMINOR_TARGET = pixels x
# images per workgroup).  Usage on the box: bash tools/gpu_joined_target.sh <tag>
set -o pipefail
TAG=${1:-jt}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
for t in 1024 4096 8192 16384; do
  RDL_SUBMINOR_TARGET=$t RDL_TRACE_SUBMINOR=2 timeout -k 10 300 python -u bench.py --workload joined \
    --steps 1 --warmup 1 --device-resident 0 > $OUT/t$t.json 2> $OUT/t$t.err || exit $?
done
