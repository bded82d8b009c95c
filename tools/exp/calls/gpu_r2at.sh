# r02 call AT: end-to-end rates with the pipelined default (registered rows,
# implicit padding, batched fold service), config 1 + config 5.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2at; mkdir -p $O
timeout -k 10 500 python -u tools/e2e_bench.py --root /dev/shm/bcp_e2e --reps 3 > $O/e2e.jsonl 2> $O/e2e.err || { echo E2E_FAIL; tail -20 $O/e2e.err; exit 1; }
grep -h "\"box\"" $O/e2e.jsonl; grep -h '"path"' $O/e2e.jsonl | python -c "import sys,json; [print(d.get('config'), d['path'][:60], d.get('GiBps'), d.get('verified', d.get('sampled_ok'))) for d in map(json.loads, sys.stdin)]"
echo ALL_OK
