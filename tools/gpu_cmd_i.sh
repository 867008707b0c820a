mkdir -p gpurun_out/r03_i
timeout -k 10 400 python -u -m pytest tests/test_fft_fast.py tests/test_configs_gpu.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider -s -k "not c3 and not c4 and not c5 and not c1" > gpurun_out/r03_i/tests.log 2>&1; tail -2 gpurun_out/r03_i/tests.log
timeout -k 10 200 python -u tools/bench_fftk.py 10 f32 f32_4096 > gpurun_out/r03_i/fftk_new.txt 2>&1 &&
RDL_FFT_ROWTW=0 timeout -k 10 200 python -u tools/bench_fftk.py 10 f32 f32_4096 > gpurun_out/r03_i/fftk_old.txt 2>&1
