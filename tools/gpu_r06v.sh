#!/bin/bash
# r06: GPU rounding ensemble of the tiled 8192^2 run to threshold (p8kt)
set -o pipefail
TAG=${1:-r06v}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u tools/end_state_spread.py p8kt > $OUT/spread_p8kt.json 2> $OUT/spread_p8kt.err || exit $?
