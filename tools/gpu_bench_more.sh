# Tiled (C5-style) and joined-channel (C3) bench lines on one GPU, host profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export RADLER_HOST_PROFILE=1
for G in ${GRIDS:-4 8}; do
  timeout -k 10 400 python -u bench.py --workload tiled --grid $G --pool $G --steps 1 --breakdown \
    > gpurun_out/bench_tiled$G.json 2> gpurun_out/bench_tiled$G.err || exit $?
done
if [ -n "$JOINED" ]; then
  timeout -k 10 400 python -u bench.py --workload joined --steps 1 --breakdown \
    > gpurun_out/bench_joined.json 2> gpurun_out/bench_joined.err || exit $?
fi
