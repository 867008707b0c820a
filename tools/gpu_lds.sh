set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/gpu_tests_lds.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload tiled --grid 8 --steps 1 --breakdown \
  > gpurun_out/tiled8_lds2.json 2> gpurun_out/tiled8_lds2.err || exit $?
timeout -k 10 300 python -u bench.py --workload tiled --grid 4 --steps 1 --breakdown \
  > gpurun_out/tiled4_lds2.json 2> gpurun_out/tiled4_lds2.err || exit $?
timeout -k 10 500 python -u bench.py --workload tiled --size 16384 --grid 8 --steps 1 --breakdown \
  > gpurun_out/bench_c5_lds.json 2> gpurun_out/bench_c5_lds.err || exit $?
