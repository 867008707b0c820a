set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -m gpu -x -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_dist.log 2>&1 || exit $?
RDL_TRACE_SUBMINOR=1 timeout -k 10 300 python -u bench.py --workload joined --steps 1 \
  --device-resident 0 > gpurun_out/joined_trace.json 2> gpurun_out/joined_trace.err || exit $?
export RADLER_HOST_PROFILE=1
timeout -k 10 300 python -u bench.py --workload tiled --grid 4 --pool 16 --steps 1 --breakdown \
  > gpurun_out/tiled4_p16.json 2> gpurun_out/tiled4_p16.err || exit $?
timeout -k 10 300 python -u bench.py --workload tiled --grid 8 --pool 16 --steps 1 --breakdown \
  > gpurun_out/tiled8_p16.json 2> gpurun_out/tiled8_p16.err || exit $?
