# r02 call AG: config 5 end to end (protocol now before the pipeline exists)
# and the interleaved protocol comparison, same box.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2ag; mkdir -p $O
timeout -k 10 500 python -u tools/e2e_bench.py --configs 5 --root /dev/shm/bcp_e2e --reps 3 > $O/e2e.jsonl 2> $O/e2e.err || { echo E2E_FAIL; tail -20 $O/e2e.err; exit 1; }
grep -h '"path"' $O/e2e.jsonl | python -c "import sys,json; [print(d.get('config'), d['path'][:60], d.get('GiBps'), d.get('warm_seconds'), d.get('cold_seconds'), d.get('verified')) for d in map(json.loads, sys.stdin)]"
timeout -k 10 500 python -u tools/proto_compare.py --rounds 5 --workloads c5_gen --folds gpu_batched,cpu_reference,noop > $O/proto.jsonl 2> $O/proto.err || { echo PROTO_FAIL; tail -20 $O/proto.err; exit 1; }
grep summary $O/proto.jsonl
echo ALL_OK
