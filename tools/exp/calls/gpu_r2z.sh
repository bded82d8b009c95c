# r02 call Z: per-task protocol with ranks as processes kept alive across runs
# (rank pool), every fold; then threads again on the same box for reference.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2z; mkdir -p $O
timeout -k 10 600 python -u tools/proto_compare.py --procs --rounds 6 > $O/proto_pool.jsonl 2> $O/proto_pool.err || { echo POOL_FAIL; tail -30 $O/proto_pool.err; exit 1; }
grep summary $O/proto_pool.jsonl
timeout -k 10 600 python -u tools/proto_compare.py --rounds 6 > $O/proto_threads.jsonl 2> $O/proto_threads.err || { echo THREADS_FAIL; tail -30 $O/proto_threads.err; exit 1; }
grep summary $O/proto_threads.jsonl
echo ALL_OK
