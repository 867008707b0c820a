# Timeline of one default bench step: kernel + HIP API + copy traces, the GPU
# busy fraction and what the host did during the idle gaps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/trace_${TAG:-bench}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d $OUT/prof -o run -- \
  python3 $R/bench.py --steps 1 --warmup 1 --cpu-outer 0 --device-resident 0 ${BENCH_ARGS:-} \
  > $OUT/bench.json 2> $OUT/bench.err || true
DB=$(ls $OUT/prof/*.db $OUT/prof/*/*.db 2>/dev/null | head -1)
python3 $R/tools/rocpd_api_stats.py $DB --out $OUT/api_stats.txt || true
python3 $R/tools/rocpd_stats.py $DB --csv $OUT/kernel_stats.csv --top $OUT/kernel_stats_top.txt --title "trace ${TAG:-bench}" || true
rm -rf $OUT/prof
