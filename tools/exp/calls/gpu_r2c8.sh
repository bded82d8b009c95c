# r02 call C8: the round's final per-task protocol comparison on one box -- ranks as
# threads (every fold interleaved) and ranks as processes (fold server; the CPU fold
# without it) -- then the end-to-end bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2c8; mkdir -p $O
timeout -k 10 600 python -u tools/proto_compare.py --rounds 6 --folds gpu_pipelined,gpu_batched,cpu_reference,noop > $O/threads.jsonl 2> $O/threads.err || { echo PC_THREADS_FAIL; tail -20 $O/threads.err; exit 1; }
grep summary $O/threads.jsonl | cut -c1-220
timeout -k 10 500 python -u tools/proto_compare.py --procs --rounds 5 --folds gpu_batched,noop > $O/procs_server.jsonl 2> $O/procs_server.err || { echo PC_SERVER_FAIL; tail -20 $O/procs_server.err; exit 1; }
grep summary $O/procs_server.jsonl | cut -c1-220
BCP_FOLD_SERVER=0 timeout -k 10 500 python -u tools/proto_compare.py --procs --rounds 5 --folds cpu_reference,gpu_batched,noop > $O/procs_ranks.jsonl 2> $O/procs_ranks.err || { echo PC_RANKS_FAIL; tail -20 $O/procs_ranks.err; exit 1; }
grep summary $O/procs_ranks.jsonl | cut -c1-220
timeout -k 10 600 python -u tools/e2e_bench.py --reps 3 > $O/e2e.jsonl 2> $O/e2e.err || { echo E2E_FAIL; tail -20 $O/e2e.err; exit 1; }
python3 -c "
import json
for l in open('$O/e2e.jsonl'):
    d=json.loads(l)
    if 'GiBps' in d: print(d.get('config'), d.get('path'), d.get('fold', ''), d['GiBps'])
"
echo ALL_OK
