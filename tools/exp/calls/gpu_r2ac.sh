# r02 call AC: per-task protocol with ranks as processes kept alive across runs
# (rank pool, 2 HW queues per rank, one pool at a time), every fold; then threads.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2ac; mkdir -p $O
timeout -k 10 600 python -u tools/proto_compare.py --procs --rounds 6 > $O/proto_pool.jsonl 2> $O/proto_pool.err || { echo POOL_FAIL; tail -30 $O/proto_pool.err; exit 1; }
grep summary $O/proto_pool.jsonl
timeout -k 10 600 python -u tools/proto_compare.py --rounds 6 > $O/proto_threads.jsonl 2> $O/proto_threads.err || { echo THREADS_FAIL; tail -30 $O/proto_threads.err; exit 1; }
grep summary $O/proto_threads.jsonl
echo ALL_OK
