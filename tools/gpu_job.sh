set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export RADLER_HOST_PROFILE=1
timeout -k 10 400 python -u bench.py --breakdown --cpu-single-thread 0 > gpurun_out/bench_fields.json 2> gpurun_out/bench_fields.err
timeout -k 10 400 python -u bench.py --workload tiled --grid 4 --pool 4 --steps 1 --breakdown > gpurun_out/bench_tiled4.json 2> gpurun_out/bench_tiled4.err
timeout -k 10 400 python -u bench.py --workload tiled --grid 8 --pool 8 --steps 1 --breakdown > gpurun_out/bench_tiled8.json 2> gpurun_out/bench_tiled8.err
