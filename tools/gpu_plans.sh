set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fft_fast.py tests/test_gpu_kernels.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider -k "fast or ms_transform" \
  > gpurun_out/plans_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload tiled --grid 8 --steps 1 --breakdown \
  > gpurun_out/tiled8_plans.json 2> gpurun_out/tiled8_plans.err || exit $?
timeout -k 10 300 python -u bench.py --workload tiled --grid 4 --steps 1 --breakdown \
  > gpurun_out/tiled4_plans.json 2> gpurun_out/tiled4_plans.err || exit $?
timeout -k 10 500 python -u bench.py --workload tiled --size 16384 --grid 8 --steps 1 --breakdown \
  > gpurun_out/bench_c5_plans.json 2> gpurun_out/bench_c5_plans.err || exit $?
