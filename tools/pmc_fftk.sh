#!/bin/bash
# ONE PMC pass (counter group k) over a micro-benchmark, outputs under
# gpurun_out/<tag>/pmc_<k> (rocprofv3 may crash at exit after writing its
# database, so each pass is its own gpurun call).
#   bash tools/pmc_fftk.sh <tag> <k> [bench args...]     (default bench: fftk f64)
# k: 0 lists the counters; 1-2 SQ groups; 3 FETCH_SIZE; 4 WRITE_SIZE
TAG=${1:-pmc}
K=${2:-1}
shift 2
ARGS=${@:-tools/bench_fftk.py 3 f64}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
case $K in
  0) exec timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 ;;
  1) G="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" ;;
  2) G="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES" ;;
  3) G="FETCH_SIZE" ;;
  4) G="WRITE_SIZE" ;;
esac
timeout -s KILL 120 rocprofv3 --pmc $G --kernel-trace -d $OUT/pmc_$K -o run -- \
  python3 $R/$ARGS > $OUT/pmc_$K.log 2>&1
