set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for p in 8 12 16; do
timeout -k 10 300 python -u bench.py --workload tiled --grid 8 --steps 3 --pool $p > gpurun_out/pool_$p.json 2> gpurun_out/pool_$p.err || exit $?
done
