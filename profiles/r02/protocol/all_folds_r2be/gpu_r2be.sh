# r02 call BE: every P-role fold, interleaved on one box, all three workloads
# (the round's final table), then a kernel trace of the default fold on config 5.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2be; mkdir -p $O
timeout -k 10 900 python -u tools/proto_compare.py --rounds 6 --folds gpu_pipelined,gpu_batched,gpu_zero_copy,gpu_streamed,gpu_device_rows,gpu_staged,cpu_reference,noop > $O/proto_all.jsonl 2> $O/proto_all.err || { echo PROTO_FAIL; tail -20 $O/proto_all.err; exit 1; }
grep -h '"box"' $O/proto_all.jsonl; grep summary $O/proto_all.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/tools/proto_compare.py --rounds 2 --workloads c5_gen --folds gpu_pipelined --c5-stripes 400 > $O/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-220 | head -12
echo ALL_OK
