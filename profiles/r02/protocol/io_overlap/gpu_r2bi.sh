# r02 call BI: which half of the P-role I/O overlap costs config 5 -- the open
# after the receives (_serialwrite keeps it) or the early prefix write
# (_serialopen keeps it); interleaved, all three workloads.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2bi; mkdir -p $O
timeout -k 10 900 python -u tools/proto_compare.py --rounds 6 --folds gpu_pipelined,gpu_pipelined_serial,gpu_pipelined_serialopen,gpu_pipelined_serialwrite,noop,noop_serialopen > $O/ab.jsonl 2> $O/ab.err || { echo AB_FAIL; tail -20 $O/ab.err; exit 1; }
grep -h '"box"' $O/ab.jsonl; grep summary $O/ab.jsonl
echo ALL_OK
