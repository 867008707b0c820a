#!/bin/bash
# Table-kernel microbenchmark at forced workgroup sizes (256 / 512 / 1024
# threads).  Usage on the box: bash tools/gpu_tabthreads.sh <tag>
set -o pipefail
TAG=${1:-tabthreads}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
for t in 256 512 1024; do
  RDL_BENCH_TAB=1 RDL_SUBMINOR_TAB_THREADS=$t timeout -k 10 200 python -u tools/bench_subminor.py \
    > $OUT/threads$t.txt 2>&1 || exit $?
done
