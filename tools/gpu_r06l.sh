#!/bin/bash
# r06: IUWT chain strip widths and modes (C4 leg alone), then a kernel trace
# of the C4 algorithm
set -o pipefail
TAG=${1:-r06l}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for cfg in "RDL_IUWT_FUSED=1" "RDL_IUWT_CHAIN_WS=256" "RDL_IUWT_CHAIN_WS=512" "RDL_IUWT_CHAIN_WS=1024"; do
  env $cfg timeout -k 10 200 python -u tools/iuwt_run.py >> $OUT/iuwt_modes.jsonl 2>> $OUT/iuwt_modes.err || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $R/tools/iuwt_run.py > $OUT/prof_iuwt.json 2> $OUT/prof_iuwt.err
echo "rocprof exit $?"
exit 0
