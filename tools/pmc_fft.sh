#!/bin/bash
# PMC counters of the FFT kernels on one plane size (tools/bench_fft.py).
# Usage on the GPU box: bash tools/pmc_fft.sh W,H,F64 <tag>
set -e
CASE=${1:-8192,8192,0}
TAG=${2:-fft}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $R/gpurun_out/${TAG}_pmc1 -o run -- python3 $R/tools/bench_fft.py $CASE 2 > $R/gpurun_out/${TAG}_pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum -d $R/gpurun_out/${TAG}_pmc2 -o run -- python3 $R/tools/bench_fft.py $CASE 2 > $R/gpurun_out/${TAG}_pmc2.log 2>&1
