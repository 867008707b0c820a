#!/bin/bash
# r06: split joined regression — 3c383ca's peak/session/header half on the old tree
set -o pipefail
TAG=${1:-r06o}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for t in 365876d devB; do cp tools/bench_legs.py _bisect/$t/tools/; done
(cd _bisect/devB && timeout -k 10 300 python -u tools/bench_legs.py joined_split --reps 2 \
  > $OUT/legs_devB.jsonl 2> $OUT/legs_devB.err) || exit $?
(cd _bisect/365876d && timeout -k 10 300 python -u tools/bench_legs.py joined_split --reps 2 \
  > $OUT/legs_old.jsonl 2> $OUT/legs_old.err) || exit $?
(cd _bisect/devB && RDL_ZERO_COPY=0 timeout -k 10 300 python -u tools/bench_legs.py joined_split --reps 2 \
  > $OUT/legs_devB_zc0.jsonl 2> $OUT/legs_devB_zc0.err) || exit $?
