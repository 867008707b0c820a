set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_multiscale_gpu.py tests/test_configs_gpu.py tests/test_radler_gpu.py tests/test_fft_fast.py -k "subminor or multiscale or c2 or c3 or clark or joined or pipeline" -x -q -s --timeout 280 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_table_tests2.log 2>&1 || exit $?
for T in 2048 4096 8192; do
  RDL_SUBMINOR_TABLE_MAX=$T timeout -k 10 200 python -u bench.py --breakdown --cpu-outer 0 --tiled-reference 0 \
    > gpurun_out/bench_t$T.json 2> gpurun_out/bench_t$T.err || exit $?
done
RDL_TRACE_SUBMINOR=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --cpu-outer 0 --tiled-reference 0 --device-resident 0 \
  > gpurun_out/bench_t8192_trace.json 2> gpurun_out/bench_t8192_trace.err || exit $?
timeout -k 10 300 python -u bench.py --workload joined --steps 1 --breakdown --device-resident 0 \
  > gpurun_out/joined_t.json 2> gpurun_out/joined_t.err || exit $?
