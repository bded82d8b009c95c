# r02 call AR: box probe + interleaved pipelined/batched/CPU/no-op comparison
# (a third box for the pipelined default).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2ar; mkdir -p $O
timeout -k 10 700 python -u tools/proto_compare.py --rounds 6 --folds gpu_pipelined,gpu_batched,cpu_reference,noop > $O/proto.jsonl 2> $O/proto.err || { echo PROTO_FAIL; tail -20 $O/proto.err; exit 1; }
grep -h '"box"' $O/proto.jsonl
grep summary $O/proto.jsonl
echo ALL_OK
