# GPU parity suite (optionally a subset: GPU_TESTS="tests/x.py ...") + bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest ${GPU_TESTS:-tests} -m gpu -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider -s > gpurun_out/gpu_tests.log 2>&1 || exit $?
RADLER_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --breakdown --cpu-outer 0 \
  > gpurun_out/bench_hostprof.json 2> gpurun_out/bench_hostprof.err || exit $?
if [ -n "$TILED" ]; then
  RADLER_HOST_PROFILE=1 timeout -k 10 400 python -u bench.py --workload tiled --grid 4 --pool 4 \
    --steps 1 --breakdown > gpurun_out/bench_tiled4.json 2> gpurun_out/bench_tiled4.err || exit $?
  RADLER_HOST_PROFILE=1 timeout -k 10 400 python -u bench.py --workload tiled --grid 8 --pool 8 \
    --steps 1 --breakdown > gpurun_out/bench_tiled8.json 2> gpurun_out/bench_tiled8.err || exit $?
fi
timeout -k 10 500 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
