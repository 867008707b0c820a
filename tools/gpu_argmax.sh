set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_multiscale_gpu.py tests/test_configs_gpu.py tests/test_spectral.py tests/test_radler_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/argmax_tests.log 2>&1 || exit $?
RDL_TRACE_SUBMINOR=2 timeout -k 10 300 python -u bench.py --cpu-outer 0 --tiled-reference 0 --device-resident 0 --steps 1 --warmup 0 > gpurun_out/argmax_trace.json 2> gpurun_out/argmax_trace.err || exit $?
timeout -k 10 300 python -u bench.py --cpu-outer 0 --tiled-reference 0 > gpurun_out/argmax_bench.json 2> gpurun_out/argmax_bench.err || exit $?
