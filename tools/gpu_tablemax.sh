set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 16384 8192 6144; do
RDL_SUBMINOR_TABLE_MAX=$v timeout -k 10 300 python -u bench.py --cpu-outer 0 --tiled-reference 0 --device-resident 0 > gpurun_out/tmax$v.json 2> gpurun_out/tmax$v.err || exit $?
done
