set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_multiscale_gpu.py tests/test_radler_gpu.py tests/test_tiling.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/select_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --cpu-outer 0 --tiled-reference 0 > gpurun_out/select_bench1.json 2> gpurun_out/select_bench1.err || exit $?
RDL_SUBMINOR_SELECT=3 timeout -k 10 300 python -u bench.py --cpu-outer 0 --tiled-reference 0 > gpurun_out/select_bench3.json 2> gpurun_out/select_bench3.err || exit $?
