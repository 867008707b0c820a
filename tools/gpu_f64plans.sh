set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fft_fast.py tests/test_tiling.py tests/test_kat_radler_gpu.py tests/test_distributed.py tests/test_gpu_kernels.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/f64p_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload tiled --grid 8 --steps 2 > gpurun_out/f64p_tiled8.json 2> gpurun_out/f64p_tiled8.err || exit $?
timeout -k 10 300 python -u bench.py --cpu-outer 0 --tiled-reference 0 > gpurun_out/f64p_bench.json 2> gpurun_out/f64p_bench.err || exit $?
