# r02 call W: per-task protocol with the device-rows fold against the other
# GPU folds, the reference CPU fold and the no-op bound (threads, then procs).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2w; mkdir -p $O
timeout -k 10 500 python -u tools/proto_compare.py --rounds 6 > $O/proto_threads.jsonl 2> $O/proto_threads.err || { echo THREADS_FAIL; tail -30 $O/proto_threads.err; exit 1; }
grep summary $O/proto_threads.jsonl
timeout -k 10 500 python -u tools/proto_compare.py --procs --rounds 5 --folds gpu_device_rows,gpu_batched,cpu_reference,noop > $O/proto_procs.jsonl 2> $O/proto_procs.err || { echo PROCS_FAIL; tail -30 $O/proto_procs.err; exit 1; }
grep summary $O/proto_procs.jsonl
echo ALL_OK
