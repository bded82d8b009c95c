# r02 call AI: fold-service width K=1 vs K=2, config 1 gen, rebuild and config 5 gen, 8 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2ai; mkdir -p $O
timeout -k 10 700 python -u tools/proto_compare.py --rounds 8 --folds gpu_batched1,gpu_batched2,cpu_reference,noop > $O/proto.jsonl 2> $O/proto.err || { echo PROTO_FAIL; tail -20 $O/proto.err; exit 1; }
grep summary $O/proto.jsonl
echo ALL_OK
