# r02 call O: per-task protocol with ranks as PROCESSES (socketpair transport)
# and as threads, same box, same stores.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2o; mkdir -p $O
timeout -k 10 500 python -u tools/proto_compare.py --procs --rounds 6 --folds gpu_batched,gpu_zero_copy,cpu_reference,noop > $O/proto_procs.jsonl 2> $O/proto_procs.err || { echo PROCS_FAIL; tail -30 $O/proto_procs.err; exit 1; }
grep summary $O/proto_procs.jsonl
timeout -k 10 500 python -u tools/proto_compare.py --rounds 6 --folds gpu_batched,gpu_zero_copy,cpu_reference,noop > $O/proto_threads.jsonl 2> $O/proto_threads.err || { echo THREADS_FAIL; tail -30 $O/proto_threads.err; exit 1; }
grep summary $O/proto_threads.jsonl
echo ALL_OK
