# r02 call D7: end-to-end bench at the final code on /dev/shm (incl. the 12-lane
# protocol rebuild).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2d7; mkdir -p $O
timeout -k 10 700 python -u tools/e2e_bench.py --root /dev/shm/bcp_e2e --reps 3 > $O/e2e.jsonl 2> $O/e2e.err || { echo E2E_FAIL; tail -20 $O/e2e.err; rm -rf /dev/shm/bcp_e2e; exit 1; }
rm -rf /dev/shm/bcp_e2e
python3 -c "
import json
for l in open('$O/e2e.jsonl'):
    d=json.loads(l)
    if 'GiBps' in d: print(d.get('config'), d.get('path'), d['GiBps'])
"
echo ALL_OK
