set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_configs_gpu.py tests/test_spectral.py tests/test_multiscale_gpu.py tests/test_radler_gpu.py tests/test_kat_image_set.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/regint_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload joined --steps 2 > gpurun_out/regint_joined.json 2> gpurun_out/regint_joined.err || exit $?
timeout -k 10 300 python -u bench.py --cpu-outer 0 --tiled-reference 0 > gpurun_out/regint_bench.json 2> gpurun_out/regint_bench.err || exit $?
