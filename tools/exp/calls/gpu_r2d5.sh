# r02 call D5: rebuild lanes -- the per-task rebuild with 1 (the reference's) and 12
# lanes per rank, every fold interleaved (threads), then rank processes (fold server).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2d5; mkdir -p $O
for L in 1 12; do
  timeout -k 10 400 python -u tools/proto_compare.py --rounds 5 --workloads c1_rebuild --rebuild-lanes $L --folds gpu_pipelined,gpu_batched,cpu_reference,noop > $O/threads_L$L.jsonl 2> $O/threads_L$L.err || { echo PC_FAIL $L; tail -20 $O/threads_L$L.err; exit 1; }
  echo "threads rebuild lanes $L"; grep summary $O/threads_L$L.jsonl | cut -c1-260
  timeout -k 10 400 python -u tools/proto_compare.py --procs --rounds 5 --workloads c1_rebuild --rebuild-lanes $L --folds gpu_batched,cpu_reference,noop > $O/procs_L$L.jsonl 2> $O/procs_L$L.err || { echo PC_PROCS_FAIL $L; tail -20 $O/procs_L$L.err; exit 1; }
  echo "procs rebuild lanes $L"; grep summary $O/procs_L$L.jsonl | cut -c1-260
done
echo ALL_OK
