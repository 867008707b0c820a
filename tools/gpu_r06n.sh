#!/bin/bash
# r06: split joined regression — the host half of 3c383ca on the old tree
set -o pipefail
TAG=${1:-r06n}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for t in 365876d hostA; do
  cp tools/bench_legs.py _bisect/$t/tools/
done
(cd _bisect/365876d && timeout -k 10 300 python -u tools/bench_legs.py joined_split --reps 2 \
  > $OUT/legs_old.jsonl 2> $OUT/legs_old.err) || exit $?
(cd _bisect/hostA && timeout -k 10 300 python -u tools/bench_legs.py joined_split --reps 2 \
  > $OUT/legs_hostA.jsonl 2> $OUT/legs_hostA.err) || exit $?
timeout -k 10 300 python -u tools/bench_legs.py joined_split --reps 2 > $OUT/legs_new.jsonl 2> $OUT/legs_new.err || exit $?
(cd _bisect/hostA && timeout -k 10 300 python -u tools/bench_legs.py joined_split --reps 2 \
  > $OUT/legs_hostA2.jsonl 2> $OUT/legs_hostA2.err) || exit $?
