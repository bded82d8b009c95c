# r02 call AB: 9 rank processes on ONE GPU (config-5 shapes, pooled): HW
# queues per process 1 / 2 / default 4.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2ab; mkdir -p $O
for q in 1 2 4; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/proto_compare.py --procs --rounds 4 --workloads c5_gen --c5-stripes 600 --folds gpu_batched,cpu_reference > $O/pool_q$q.jsonl 2> $O/pool_q$q.err || { echo POOL_FAIL $q; tail -20 $O/pool_q$q.err; exit 1; }
  python3 -c "
import json
for l in open('$O/pool_q$q.jsonl'):
    d=json.loads(l)
    if 'fold' in d: print('q=$q', d['fold'], d['GiBps'], d['runs_s'])
"
done
echo ALL_OK
