#!/bin/bash
# Sub-minor loop per-launch profile of the default 8192^2 bench (one warm-up
# + one timed Perform, no CPU leg): RDL_TRACE_SUBMINOR=2 (timing only) then =1
# (phase probes).  Usage on the box: bash tools/gpu_subminor_trace.sh <tag>
set -o pipefail
TAG=${1:-subminor}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
RDL_TRACE_SUBMINOR=2 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-outer 0 \
  --tiled-reference 0 --device-resident 0 > $OUT/trace2.json 2> $OUT/trace2.err || exit $?
RDL_TRACE_SUBMINOR=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-outer 0 \
  --tiled-reference 0 --device-resident 0 > $OUT/trace1.json 2> $OUT/trace1.err
