set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $R/gpurun_out/fpmc1 -o run -- python3 $R/tools/bench_fft.py 9216,9216,1 2 > $R/gpurun_out/fpmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum -d $R/gpurun_out/fpmc2 -o run -- python3 $R/tools/bench_fft.py 9216,9216,1 2 > $R/gpurun_out/fpmc2.log 2>&1 || true
timeout -s KILL 90 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
