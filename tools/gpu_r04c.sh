cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04c
mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_fftk.py 10 f32 f64 f64_window > $OUT/fftk_tiled.txt 2>&1 || exit $?
RDL_FFT_STEPS_MIN=20000 timeout -k 10 300 python -u tools/bench_fftk.py 10 f32 > $OUT/fftk_rowmajor.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_fft_fast.py tests/test_configs_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -s -k "not test_c5" > $OUT/tests.log 2>&1
tail -3 $OUT/tests.log
cat $OUT/fftk_tiled.txt $OUT/fftk_rowmajor.txt
