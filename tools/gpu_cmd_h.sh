# table-kernel parity + phase profile; float64 column pass layouts
mkdir -p gpurun_out/r03_h
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "table_kernel or subminor_loop_bit_exact" > gpurun_out/r03_h/tests.log 2>&1; tail -2 gpurun_out/r03_h/tests.log
timeout -k 10 200 python -u tools/bench_fftk.py 10 f64 f64_colout > gpurun_out/r03_h/fftk.txt 2>&1 &&
RDL_TRACE_SUBMINOR=1 RDL_BENCH_TAB=1 timeout -k 10 300 python -u tools/bench_subminor.py > gpurun_out/r03_h/b.txt 2> gpurun_out/r03_h/b.err
