set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fft_fast.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/f64p2_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --cpu-outer 0 --tiled-reference 0 > gpurun_out/f64p2_bench.json 2> gpurun_out/f64p2_bench.err || exit $?
timeout -k 10 500 python -u bench.py --workload tiled --size 16384 --grid 8 --steps 1 > gpurun_out/f64p2_c5.json 2> gpurun_out/f64p2_c5.err || exit $?
