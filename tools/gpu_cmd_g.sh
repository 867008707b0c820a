mkdir -p gpurun_out/r03_g
timeout -k 10 400 python -u -m pytest tests/test_fft_fast.py tests/test_gpu_kernels.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "masked_correction or convolutions_match or sparse_rows or table_kernel" > gpurun_out/r03_g/tests.log 2>&1; tail -2 gpurun_out/r03_g/tests.log
RDL_SUBMINOR_TAB_THREADS=256 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "table_kernel" > gpurun_out/r03_g/tests256.log 2>&1; tail -2 gpurun_out/r03_g/tests256.log
timeout -k 10 200 python -u tools/bench_fftk.py 10 f64 f64_dense > gpurun_out/r03_g/fftk_new.txt 2>&1 &&
RDL_FFT_CONVD=0 timeout -k 10 200 python -u tools/bench_fftk.py 10 f64 f64_dense > gpurun_out/r03_g/fftk_old.txt 2>&1 &&
RDL_SUBMINOR_TAB_THREADS=256 RDL_TRACE_SUBMINOR=1 RDL_BENCH_TAB=1 timeout -k 10 300 python -u tools/bench_subminor.py > gpurun_out/r03_g/b256.txt 2> gpurun_out/r03_g/b256.err &&
RDL_SUBMINOR_TAB_THREADS=512 RDL_BENCH_TAB=1 timeout -k 10 300 python -u tools/bench_subminor.py > gpurun_out/r03_g/b512.txt 2> gpurun_out/r03_g/b512.err
