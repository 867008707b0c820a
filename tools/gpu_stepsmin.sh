set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 0 4096; do
RDL_FFT_STEPS_MIN=$v timeout -k 10 300 python -u bench.py --workload tiled --grid 4 --steps 1 > gpurun_out/smin4_$v.json 2> gpurun_out/smin4_$v.err || exit $?
RDL_FFT_STEPS_MIN=$v timeout -k 10 300 python -u bench.py --workload tiled --grid 8 --steps 2 > gpurun_out/smin8_$v.json 2> gpurun_out/smin8_$v.err || exit $?
done
