set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fft_fast.py tests/test_multiscale_gpu.py tests/test_configs_gpu.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/fwdpair_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_fft.py 8192,8192,0 10 > gpurun_out/fwdpair_fft.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --cpu-outer 0 --tiled-reference 0 > gpurun_out/fwdpair_bench.json 2> gpurun_out/fwdpair_bench.err || exit $?
