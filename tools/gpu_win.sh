set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fft_fast.py tests/test_multiscale_gpu.py tests/test_tiling.py tests/test_gpu_kernels.py tests/test_kat_radler_gpu.py tests/test_distributed.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/win_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload tiled --grid 8 --steps 2 > gpurun_out/win_tiled8.json 2> gpurun_out/win_tiled8.err || exit $?
timeout -k 10 300 python -u bench.py --workload tiled --grid 4 --steps 1 > gpurun_out/win_tiled4.json 2> gpurun_out/win_tiled4.err || exit $?
