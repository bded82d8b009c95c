# r02 call AH: fold-service width K and the per-lane folds, config 1 gen and
# config 5 gen, interleaved (threads).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2ah; mkdir -p $O
timeout -k 10 700 python -u tools/proto_compare.py --rounds 5 --workloads c1_gen,c5_gen --folds gpu_batched1,gpu_batched2,gpu_batched4,gpu_zero_copy,gpu_staged,cpu_reference,noop > $O/proto.jsonl 2> $O/proto.err || { echo PROTO_FAIL; tail -20 $O/proto.err; exit 1; }
grep summary $O/proto.jsonl
echo ALL_OK
