set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fft_fast.py tests/test_gpu_kernels.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pad_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/bench_fft.py > gpurun_out/pad_fft.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --cpu-outer 0 --tiled-reference 0 \
  > gpurun_out/pad_bench.json 2> gpurun_out/pad_bench.err || exit $?
timeout -k 10 300 python -u bench.py --workload tiled --grid 8 --steps 1 --breakdown \
  > gpurun_out/pad_tiled8.json 2> gpurun_out/pad_tiled8.err || exit $?
