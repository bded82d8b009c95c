# r02 call H: GPU tests (protocol + knobs), the protocol fold comparison with
# registered rows (default now), and the end-to-end pipeline with registered
# vs hipHostMalloc slabs.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2k; mkdir -p $O
timeout -k 10 600 python -u tools/proto_compare.py --rounds 8 --c1-files 4000 --c5-stripes 1500 --folds gpu_batched1,gpu_batched12,gpu_zero_copy,cpu_reference,noop > $O/proto_compare.jsonl 2> $O/proto_compare.err || { echo PROTO_FAIL; tail -20 $O/proto_compare.err; exit 1; }
grep summary $O/proto_compare.jsonl
echo ALL_OK
