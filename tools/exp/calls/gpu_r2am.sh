# r02 call AM: config 5 end to end after parallel replica updates
# and the interleaved protocol comparison, same box.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2am; mkdir -p $O
timeout -k 10 500 python -u tools/e2e_bench.py --configs 5 --root /dev/shm/bcp_e2e --reps 3 > $O/e2e.jsonl 2> $O/e2e.err || { echo E2E_FAIL; tail -20 $O/e2e.err; exit 1; }
grep -h '"path"' $O/e2e.jsonl | python -c "import sys,json; [print(d.get('config'), d['path'][:60], d.get('GiBps'), d.get('warm_seconds'), d.get('cold_seconds'), d.get('verified')) for d in map(json.loads, sys.stdin)]"
echo ALL_OK
