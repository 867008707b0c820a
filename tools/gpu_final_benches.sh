set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final_r02
O=gpurun_out/final_r02
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
timeout -k 10 300 python -u bench.py --workload tiled --grid 8 --steps 2 --breakdown > $O/tiled8.json 2> $O/tiled8.err || exit $?
timeout -k 10 300 python -u bench.py --workload tiled --grid 4 --steps 1 --breakdown > $O/tiled4.json 2> $O/tiled4.err || exit $?
timeout -k 10 300 python -u bench.py --workload joined --steps 2 > $O/joined.json 2> $O/joined.err || exit $?
timeout -k 10 500 python -u bench.py --workload tiled --size 16384 --grid 8 --steps 1 --breakdown > $O/c5.json 2> $O/c5.err || exit $?
