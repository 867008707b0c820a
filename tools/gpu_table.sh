set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_multiscale_gpu.py tests/test_configs_gpu.py tests/test_radler_gpu.py -k "subminor or multiscale or c2 or c3 or clark or joined" -x -q -s --timeout 280 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_table_tests.log 2>&1 || exit $?
RDL_SUBMINOR_TABLE_MAX=0 timeout -k 10 200 python -u bench.py --breakdown --cpu-outer 0 --tiled-reference 0 \
  > gpurun_out/bench_notable.json 2> gpurun_out/bench_notable.err || exit $?
timeout -k 10 200 python -u bench.py --breakdown --cpu-outer 0 --tiled-reference 0 \
  > gpurun_out/bench_table.json 2> gpurun_out/bench_table.err || exit $?
RDL_TRACE_SUBMINOR=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --cpu-outer 0 --tiled-reference 0 --device-resident 0 \
  > gpurun_out/bench_table_trace.json 2> gpurun_out/bench_table_trace.err || exit $?
timeout -k 10 300 python -u bench.py --workload joined --steps 1 --breakdown --device-resident 0 \
  > gpurun_out/joined_table.json 2> gpurun_out/joined_table.err || exit $?
