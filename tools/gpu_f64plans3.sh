set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fft_fast.py tests/test_tiling.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/f64p3_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload tiled --grid 4 --steps 1 > gpurun_out/f64p3_tiled4.json 2> gpurun_out/f64p3_tiled4.err || exit $?
timeout -k 10 500 python -u bench.py --workload tiled --size 16384 --grid 8 --steps 1 > gpurun_out/f64p3_c5.json 2> gpurun_out/f64p3_c5.err || exit $?
