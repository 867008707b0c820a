set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
RDL_SUBMINOR_SELECT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "subminor or sub_minor" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/select2_tests.log 2>&1 || exit $?
for v in 2 1 3; do
RDL_SUBMINOR_SELECT=$v timeout -k 10 300 python -u bench.py --cpu-outer 0 --tiled-reference 0 --device-resident 0 > gpurun_out/selv$v.json 2> gpurun_out/selv$v.err || exit $?
done
