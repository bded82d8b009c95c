# r02 call AD: pooled ranks (9 on one GPU, 2 HW queues each): which fold mode
# left in the ranks slows the batched fold?
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2ad; mkdir -p $O
for set in gpu_batched,cpu_reference gpu_streamed,gpu_batched,cpu_reference gpu_device_rows,gpu_batched,cpu_reference gpu_zero_copy,gpu_batched,cpu_reference; do
  tag=$(echo $set | tr ',' '-')
  timeout -k 10 300 python -u tools/proto_compare.py --procs --rounds 4 --workloads c5_gen --c5-stripes 600 --folds $set > $O/$tag.jsonl 2> $O/$tag.err || { echo POOL_FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
for l in open('$O/$tag.jsonl'):
    d=json.loads(l)
    if 'fold' in d: print('$tag', d['fold'], d['GiBps'], d['runs_s'])
"
done
echo ALL_OK
