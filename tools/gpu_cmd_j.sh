mkdir -p gpurun_out/r03_j
timeout -k 10 400 python -u -m pytest tests/test_fft_fast.py tests/test_configs_gpu.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider -s -k "not c3 and not c4 and not c5 and not c1 and not scale_conv" > gpurun_out/r03_j/tests.log 2>&1; tail -2 gpurun_out/r03_j/tests.log
timeout -k 10 200 python -u tools/bench_fftk.py 10 f32 f32_4096 > gpurun_out/r03_j/fftk.txt 2>&1
