set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_configs_gpu.py tests/test_spectral.py -k "subminor or c3 or joined or clark" -x -q -s --timeout 280 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_table_tests3.log 2>&1 || exit $?
for T in 8192 16384; do
  RDL_SUBMINOR_TABLE_MAX=$T timeout -k 10 200 python -u bench.py --breakdown --cpu-outer 0 --tiled-reference 0 \
    > gpurun_out/bench_u$T.json 2> gpurun_out/bench_u$T.err || exit $?
done
timeout -k 10 300 python -u bench.py --workload joined --steps 1 --breakdown --device-resident 0 \
  > gpurun_out/joined_u.json 2> gpurun_out/joined_u.err || exit $?
timeout -k 10 300 python -u bench.py --workload tiled --grid 8 --steps 1 --breakdown \
  > gpurun_out/tiled8_u.json 2> gpurun_out/tiled8_u.err || exit $?
RADLER_FFT=lds timeout -k 10 300 python -u bench.py --workload tiled --grid 8 --steps 1 --breakdown \
  > gpurun_out/tiled8_lds.json 2> gpurun_out/tiled8_lds.err || exit $?
timeout -k 10 500 python -u bench.py --workload tiled --size 16384 --grid 8 --steps 1 --breakdown \
  > gpurun_out/bench_c5_16384.json 2> gpurun_out/bench_c5_16384.err || exit $?
