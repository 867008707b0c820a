cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04a
mkdir -p $OUT
timeout -k 10 720 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -s -k "not test_c5" > $OUT/gpu_tests.log 2>&1
rc=$?
tail -5 $OUT/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
