set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
RADLER_FFT=lds RADLER_HOST_PROFILE=1 BENCH_TILED_RUNS=1 timeout -k 10 600 python -u tools/bench_tiled.py 8192 4 1 > gpurun_out/job2_tiled_lds.log 2>&1
bash tools/diag_tiled.sh t4x4b 8192 4 1
