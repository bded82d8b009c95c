# r02 call BK: final code, second box for the open overlap against the
# reference's P role, then the end-to-end bench with both CPU baselines.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2bk; mkdir -p $O
timeout -k 10 900 python -u tools/proto_compare.py --rounds 7 --folds gpu_pipelined,gpu_pipelined_serial,cpu_reference,cpu_pipelined,noop > $O/ab.jsonl 2> $O/ab.err || { echo AB_FAIL; tail -20 $O/ab.err; exit 1; }
grep -h '"box"' $O/ab.jsonl; grep summary $O/ab.jsonl
timeout -k 10 600 python -u tools/e2e_bench.py --root /dev/shm/bcp_e2e --reps 3 > $O/e2e.jsonl 2> $O/e2e.err || { echo E2E_FAIL; tail -20 $O/e2e.err; exit 1; }
python3 -c "
import json
for l in open('$O/e2e.jsonl'):
    d=json.loads(l)
    if 'GiBps' in d: print(d.get('config'), d.get('path'), d['GiBps'])
"
echo ALL_OK
