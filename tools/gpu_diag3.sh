set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "subminor" -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_subminor.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py -k "c3" -x -q -s --timeout 280 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_c3.log 2>&1 || exit $?
RDL_TRACE_SUBMINOR=1 timeout -k 10 300 python -u bench.py --workload joined --steps 1 --breakdown \
  --device-resident 0 > gpurun_out/joined2.json 2> gpurun_out/joined2.err || exit $?
export RADLER_HOST_PROFILE=1
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python -u bench.py --workload tiled --grid 4 --pool 16 --steps 1 --breakdown \
  > gpurun_out/tiled4_q16.json 2> gpurun_out/tiled4_q16.err || exit $?
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python -u bench.py --workload tiled --grid 8 --pool 16 --steps 1 --breakdown \
  > gpurun_out/tiled8_q16.json 2> gpurun_out/tiled8_q16.err || exit $?
