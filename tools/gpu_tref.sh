set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --cpu-outer 0 --device-resident 0 > gpurun_out/tref_a.json 2> gpurun_out/tref_a.err || exit $?
RDL_ALLOC_CACHE=0 timeout -k 10 400 python -u bench.py --cpu-outer 0 --device-resident 0 > gpurun_out/tref_b.json 2> gpurun_out/tref_b.err || exit $?
