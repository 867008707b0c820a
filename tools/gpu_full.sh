# full GPU parity suite, then the default bench line (as the driver runs it)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -s > gpurun_out/gpu_tests_full.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
