set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload tiled --grid 8 --steps 4 --warmup 1 > gpurun_out/tref_c.json 2> gpurun_out/tref_c.err || exit $?
