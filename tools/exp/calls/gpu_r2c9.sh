# r02 call C9: rank processes with the node fold server -- GPU fold and the reference
# CPU fold interleaved in ONE pool (the CPU fold runs in the ranks: the server has no
# test double), twice; then the end-to-end bench on /dev/shm.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2c9; mkdir -p $O
for i in 1 2; do
  timeout -k 10 500 python -u tools/proto_compare.py --procs --rounds 5 --folds gpu_batched,cpu_reference,noop > $O/procs_$i.jsonl 2> $O/procs_$i.err || { echo PC_FAIL $i; tail -20 $O/procs_$i.err; exit 1; }
  grep summary $O/procs_$i.jsonl | cut -c1-260
done
timeout -k 10 600 python -u tools/e2e_bench.py --root /dev/shm/bcp_e2e --reps 3 > $O/e2e.jsonl 2> $O/e2e.err || { echo E2E_FAIL; tail -20 $O/e2e.err; exit 1; }
rm -rf /dev/shm/bcp_e2e
python3 -c "
import json
for l in open('$O/e2e.jsonl'):
    d=json.loads(l)
    if 'GiBps' in d: print(d.get('config'), d.get('path'), d['GiBps'])
"
echo ALL_OK
