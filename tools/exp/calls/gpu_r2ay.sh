# r02 call AY: pipelined piece size 256 KiB (default) vs 128 KiB, interleaved
# within each process; two processes per size, alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2ay; mkdir -p $O
for rep in 1 2; do for piece in 262144 131072; do
  BCP_PIPE_PIECE=$piece timeout -k 10 400 python -u tools/proto_compare.py --rounds 5 --folds gpu_pipelined,gpu_batched,cpu_reference > $O/p${piece}_$rep.jsonl 2> $O/p${piece}_$rep.err || { echo PROTO_FAIL; tail -20 $O/p${piece}_$rep.err; exit 1; }
  python3 -c "
import json
for l in open('$O/p${piece}_$rep.jsonl'):
    d=json.loads(l)
    if d.get('fold')=='gpu_pipelined' or d.get('fold')=='cpu_reference': print('piece=$piece rep=$rep', d['workload'], d['fold'], d['GiBps'], d.get('range_folds_per_window',''))
"
done; done
echo ALL_OK
