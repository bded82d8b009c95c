# r02 call AE: does the rank's own setenv(GPU_MAX_HW_QUEUES=2) take effect?
# unset (rank sets 2) vs explicit 2 vs explicit 4, same box, twice each.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2ae; mkdir -p $O
for rep in 1 2; do
for q in unset 2 4; do
  if [ $q = unset ]; then env -u GPU_MAX_HW_QUEUES timeout -k 10 300 python -u tools/proto_compare.py --procs --rounds 3 --workloads c5_gen --c5-stripes 600 --folds gpu_batched,cpu_reference > $O/q${q}_$rep.jsonl 2> $O/q${q}_$rep.err || { echo FAIL; exit 1; }
  else GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/proto_compare.py --procs --rounds 3 --workloads c5_gen --c5-stripes 600 --folds gpu_batched,cpu_reference > $O/q${q}_$rep.jsonl 2> $O/q${q}_$rep.err || { echo FAIL; exit 1; }; fi
  python3 -c "
import json
for l in open('$O/q${q}_$rep.jsonl'):
    d=json.loads(l)
    if 'fold' in d: print('q=$q rep $rep', d['fold'], d['GiBps'], d['runs_s'])
"
done; done
echo ALL_OK
