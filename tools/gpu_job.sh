set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dbg_c1.py > gpurun_out/dbg_c1.log 2>&1
