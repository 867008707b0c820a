set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_spectral.py tests/test_gpu_kernels.py tests/test_radler_gpu.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/logpoly_tests.log 2>&1 || exit $?
