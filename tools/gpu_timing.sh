set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --cpu-outer 0 > gpurun_out/tim_default.json 2> gpurun_out/tim_default.err || exit $?
timeout -k 10 300 python -u bench.py --workload tiled --grid 8 --steps 2 > gpurun_out/tim_tiled8.json 2> gpurun_out/tim_tiled8.err || exit $?
