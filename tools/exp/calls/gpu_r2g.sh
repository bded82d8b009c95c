# r02 call F: host memory kind of the P role's rows (config-5 protocol).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2g; mkdir -p $O
timeout -k 10 600 python -u tools/exp/host_kind_ab.py 400 0,4,1 > $O/host_kind_ab.jsonl 2> $O/host_kind_ab.err || { echo FAIL; tail -20 $O/host_kind_ab.err; exit 1; }
cat $O/host_kind_ab.jsonl
echo ALL_OK
